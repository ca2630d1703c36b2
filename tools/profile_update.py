"""Profile one PPO minibatch update (Model.train, c4: 256 x 8 rows) with the torch
profiler: wall time per update and the GPU kernels by total time.

  python tools/profile_update.py [--rows 256] [--updates 5]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "primal-ppo_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=256)
    ap.add_argument("--updates", type=int, default=20)
    ap.add_argument("--agents", type=int, default=8)
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--split", type=int, default=None, help="net._SplitKLinear.SPLIT (row chunks)")
    ap.add_argument("--fp16-partials", action="store_true", help="split weight gradients with fp16 partials")
    ap.add_argument("--ab", default=None,
                    help="A/B a SCRIMPNet class switch (e.g. conv3_gemm, hip_conv): captured updates with it on / off, "
                         "alternating, each a fresh capture; prints one JSON line and exits")
    ap.add_argument("--shapes", action="store_true", help="profile eager updates grouped by aten op + input shapes")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    from mapf_amd.config import EnvParameters, make_config
    from mapf_amd.env import BatchedMapfGym
    from mapf_amd.maps import generate_warehouse
    from mapf_amd.model import Model
    from mapf_amd.runner import DeviceRunner
    from mapf_amd.net import _SplitKLinear
    if args.split:
        _SplitKLinear.SPLIT = args.split
    if args.fp16_partials:
        _SplitKLinear.out_dtype_ok = False
    N = args.agents
    EnvParameters.N_AGENTS = N
    EnvParameters.FOV_SIZE = 9
    env = BatchedMapfGym(make_config(args.rows, 20, 20, num_agents=N, fov=9, num_channel=6, human_mode="random",
                                     goal_mode="random", fix_choice=1, seed=1234), device=dev)
    env.reset_seeded(generate_warehouse(20, 20))
    model = Model(0, dev, global_model=True, numChannel=6, num_agents=N, fov=9)
    runner = DeviceRunner(env, model, n_steps=1, seed=0)
    mb, _ = runner.run()
    idx = np.arange(args.rows)         # host indices, as driver.py:125-130's mb_inds
    sl = lambda k: mb[k][idx]

    def upd():
        return model.train(sl("observations"), sl("vectors"), sl("returns"), sl("costReturns"), sl("values"),
                           sl("costValues"), sl("actions"), sl("ps"), None, sl("trainValid"), 1.0)
    import json
    if args.ab:
        from mapf_amd import net as netmod
        spec, _, vals = args.ab.partition("=")   # "conv3_gemm", "_LinearBG.enabled" or "_SplitKLinear.SPLIT=8,16"
        head, _, tail = spec.partition(".")
        owner, attr = ((model, tail) if head == "model" else      # "model.fused_optim": the Model instance's
                       (getattr(netmod, head), tail) if tail else (netmod.SCRIMPNet, spec))
        if vals:
            choices = [type(getattr(owner, attr))(v) for v in vals.split(",")]
        else:
            assert isinstance(getattr(owner, attr), bool), args.ab
            choices = [True, False]
        ab = {}
        for on in choices * 3:
            setattr(owner, attr, on)
            model._updates.clear()                 # a fresh capture with the switch in its new position
            for _ in range(3):
                upd()
            torch.cuda.synchronize()
            ts = []
            for _ in range(args.updates):
                t0 = time.perf_counter()
                upd()
                ts.append(time.perf_counter() - t0)
            ab.setdefault(str(on), []).append(round(float(np.median(ts)) * 1e3, 3))
            print(f"{args.ab}={on}: median {np.median(ts) * 1e3:.3f} ms", flush=True)
        print(json.dumps({"rows": args.rows, "agents": N, "ab": args.ab, "median_ms": ab}), flush=True)
        return
    res = {}
    for mode in ("graph", "eager", "graph"):      # Model.graph_update: one captured hipGraph per update
        model.graph_update = mode == "graph"
        for _ in range(3):
            upd()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.updates):
            t0 = time.perf_counter()
            upd()                                  # returns host stats: synchronises every update
            ts.append(time.perf_counter() - t0)
        res.setdefault(mode, []).append(float(np.median(ts)) * 1e3)
        print(f"update ({mode}): median {np.median(ts) * 1e3:.2f} ms, mean {np.mean(ts) * 1e3:.2f} ms for "
              f"{args.rows} x {N} rows", flush=True)
    print(json.dumps({"rows": args.rows, "agents": N, "median_ms": res}), flush=True)
    if args.no_profile:
        return
    from torch.profiler import ProfilerActivity, profile
    if args.shapes:                                # eager updates: which aten op (and input shapes) runs which kernel
        model.graph_update = False
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
            for _ in range(args.updates):
                upd()
            torch.cuda.synchronize()
        print(prof.key_averages(group_by_input_shape=True).table(
            sort_by="self_cuda_time_total", row_limit=80, max_name_column_width=40, max_shapes_column_width=110),
            flush=True)
        # the small torch ops, every shape: calls per update and device time
        small = ("aten::copy_", "aten::fill_", "aten::zero_", "aten::add", "aten::add_", "aten::sum", "aten::cat",
                 "aten::mul", "aten::mul_", "aten::div_", "aten::index", "aten::flip", "aten::clone", "aten::zeros",
                 "aten::relu", "aten::threshold_backward", "aten::sub", "aten::masked_fill_", "aten::where")
        for e in sorted(prof.key_averages(group_by_input_shape=True), key=lambda e: -e.self_device_time_total):
            if e.key in small and e.count >= args.updates:
                print(f"{e.key:24s} {e.count / args.updates:5.1f}/upd {e.self_device_time_total / args.updates:8.1f} us"
                      f"  {str(e.input_shapes)[:150]}", flush=True)
        return
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        for _ in range(args.updates):
            upd()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=70, max_name_column_width=150), flush=True)


if __name__ == "__main__":
    main()
