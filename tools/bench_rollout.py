"""Secondary benchmark: BASELINE configs c3 (policy-in-the-loop rollout) and c4
(PPO update with the RCCL gradient all-reduce).  Not the headline metric
(bench.py); prints one JSON line per measured phase on rank 0.

  python tools/bench_rollout.py --envs 4096 --agents 8 --size 20 --steps 16
  torchrun --nproc-per-node 8 tools/bench_rollout.py --envs 1024 --agents 16 --size 40 --train
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "primal-ppo_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--agents", type=int, default=8)
    ap.add_argument("--size", type=int, default=20)
    ap.add_argument("--fov", type=int, default=9)
    ap.add_argument("--steps", type=int, default=16, help="rollout length T")
    ap.add_argument("--train", action="store_true", help="also time PPO minibatch updates")
    ap.add_argument("--minibatch", type=int, default=256, help="rows per PPO minibatch (x N agents)")
    ap.add_argument("--updates", type=int, default=20)
    ap.add_argument("--update-warmup", type=int, default=12)
    ap.add_argument("--distributed-path", action="store_true",
                    help="time the update's distributed form (the c4 path: moments all-reduced, two graph segments "
                         "around the gradient-bucket all-reduce) at this world size -- with one process, a 1-rank "
                         "RCCL process group")
    ap.add_argument("--reference-maps", action="store_true",
                    help="runner.py:30 semantics: a fresh MapfGym() (random-size warehouse, padded to 40x60) "
                         "per env per rollout, instead of --size")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 or args.distributed_path:
        import torch.distributed as dist
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29517")
            dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
        else:
            dist.init_process_group("nccl", device_id=dev)
    from mapf_amd.config import EnvParameters, make_config
    from mapf_amd.env import BatchedMapfGym
    from mapf_amd.maps import generate_warehouse
    from mapf_amd.model import Model
    from mapf_amd.runner import DeviceRunner
    B, N, H, F = args.envs, args.agents, args.size, args.fov
    EnvParameters.N_AGENTS = N
    EnvParameters.FOV_SIZE = F
    from mapf_amd.runner import reference_maps
    Hh, Ww = (40, 60) if args.reference_maps else (H, H)
    env = BatchedMapfGym(make_config(B, Hh, Ww, num_agents=N, fov=F, num_channel=6, human_mode="random",
                                     goal_mode="random", fix_choice=1, seed=1234, env_offset=rank * B,
                                     shared_map=not args.reference_maps), device=dev)
    new_maps = reference_maps(env, seed=rank) if args.reference_maps else None
    env.reset_seeded(new_maps(0) if new_maps else generate_warehouse(H, H))
    model = Model(0, dev, global_model=True, numChannel=6, num_agents=N, fov=F)   # broadcasts rank 0's weights
    if args.distributed_path:
        model.distributed_update = True
    runner = DeviceRunner(env, model, n_steps=args.steps, seed=rank, new_maps=new_maps)
    runner.run()                       # warm-up (kernels, autotuning)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    mb, perf = runner.run()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out = {"phase": "rollout (policy forward + sampling + env.step + observe + GAE)", "n_gpus": world,
           "agent_steps_per_s": round(world * B * N * args.steps / dt, 1), "ms_per_step": round(dt / args.steps * 1e3, 3),
           "config": {"envs_per_gpu": B, "agents": N, "grid": "MapfGym() random 10-40 (40x60 padded), new per rollout"
                      if args.reference_maps else H, "fov": F, "T": args.steps}}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if args.train:
        rows = args.minibatch
        idx = np.arange(rows)            # host indices, as driver.py:125-130's mb_inds
        sl = lambda k: mb[k][idx]
        def upd():
            return model.train(sl("observations"), sl("vectors"), sl("returns"), sl("costReturns"), sl("values"),
                               sl("costValues"), sl("actions"), sl("ps"), None, sl("trainValid"), 1.0)
        # warm-up: MIOpen find for the backward convolutions, and GradScaler's first finite
        # step (the updates before it skip Adam; the first real one allocates Adam's state)
        for _ in range(args.update_warmup):
            upd()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        each = []
        for _ in range(args.updates):
            t1 = time.perf_counter()
            upd()                      # returns host numpy stats: synchronises every update
            each.append(round((time.perf_counter() - t1) * 1e3, 2))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        upd_obj = next(iter(model._updates.values()))
        form = ("eager" if upd_obj.graph is None else
                "two captured segments around the eager collectives" if isinstance(upd_obj.graph, tuple) else
                "one captured graph")
        allreduced = world > 1 or args.distributed_path
        if rank == 0:
            phase = ("PPO minibatch update (fwd+bwd+RCCL gradient all-reduce+Adam)" if allreduced else
                     "PPO minibatch update (fwd+bwd+Adam; one rank: no all-reduce)")
            print(json.dumps({"phase": phase, "n_gpus": world, "form": form,
                              "ms_median": float(np.median(each)), "ms_mean": round(dt / args.updates * 1e3, 3),
                              "updates_timed": args.updates, "ms_each": each,
                              "timing": "wall time per Model.train call (it returns host stats: one sync per update) "
                                        "through driver.py:125-130's call shape (host index array into the "
                                        "DeviceRunner's BatchValues), after --update-warmup updates",
                              "rows_per_update_per_gpu": rows, "agents": N,
                              "collectives": (f"RCCL, world size {world}" if allreduced else None),
                              "grad_bytes_allreduced": (4 * sum(p.numel() for p in model.network.parameters())
                                                        if allreduced else 0)}),
                  flush=True)
    if world > 1 or args.distributed_path:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
