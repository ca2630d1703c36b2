"""Benchmark: lockstep agent-steps/sec for (env.step + observe), BASELINE.json's metric.

A "step" = one lockstep step of every env on the GPU: the random policy's
actions (Philox, on device) -> getActionStatus ... jointStep (human replans,
BFS maps on goal changes) -> getAllObservations (all agents' FOV observations
+ vectors), i.e. runner.py:64-100 with a random policy.

Paths (--path):
  rollout (default)  mapf_rollout_random: a random-policy rollout of T steps per
                     launch (T = --rollout-steps, default 256 = the reference's
                     N_STEPS, alg_parameters.py:68); each wave owns one env and
                     loops step -> observe -> its own search work.  Step t's
                     actions, outputs and observation are written to slot t of
                     [T]-leading rollout buffers -- the runner's per-rollout arrays
                     (runner.py:104-115), a fresh HBM line for every store;
                     --inplace: every step re-writes the same [B]-leading buffers
                     (the per-step API's; at c2 they stay in the Infinity Cache).
  fused              one mapf_step_observe_random launch per step (the path a
                     policy-in-the-loop rollout uses), hipGraph replays of 24 steps
  split              mapf_step_random + mapf_observe, two launches per step
The breakdown also times the one-launch-per-step path.

Default workload (N=1): BASELINE config c2 -- 4096 envs x 8 agents, 20x20
generalised warehouse, FOV 11, 6 channels, Human with random goals,
lifelong random goals.  Multi-GPU: one process per GPU (torch.distributed
launcher); every rank owns its own 4096 envs (weak scaling, no data-path
collective); value = all agent-steps / max-over-ranks time.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "primal-ppo_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import mapf_amd  # noqa: E402,F401  (sets the HIP graph-capture mode before the runtime starts)
import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def bfs_channel_bytes(C, F):
    """The BFS channel (C = 7): the agent's bfsMap over its FOV window (F*F int16) and at its
    own cell, read per agent-step -- bytes SURVEY.md §8(d)'s formula leaves out."""
    return F * F * 2 + 2 if C >= 7 else 0


def observe_bytes_per_agent(C, F, H, W, N):
    """C*F^2*4 + 16 (obs + vec writes) + (ceil(H*W/8) + 8N + 8)/N (reads),
    + the BFS channel's map reads."""
    return C * F * F * 4 + 16 + (-(-H * W // 8) + 8 * N + 8) / N + bfs_channel_bytes(C, F)


def fused_bytes_per_agent(C, F, H, W, N):
    """Algorithmic HBM bytes per agent-step of the fused step+observe:
    obs + vec writes (C*F^2*4 + 16); agent state read (cell, goal, last action: 9)
    and written (9); random action (4) and step outputs (status 1, reward 4, cost 4,
    train_valid 20, fixed 4, goal flag 4, constraint 4, total reward 4: 45);
    per env: obstacle bits ceil(H*W/8) + clock/human/path state 64; the BFS channel's map reads."""
    return C * F * F * 4 + 16 + 9 + 9 + 4 + 45 + (-(-H * W // 8) + 64) / N + bfs_channel_bytes(C, F)


def _oracle_rate(O, cfg, world, B, seconds, threads):
    """Agent-steps/s of `threads` OS threads, each stepping its own OracleBatch of B envs for
    ~`seconds` (ctypes drops the GIL inside oc_batch_run; the C oracle has no global state)."""
    import threading
    batches = [O.OracleBatch(cfg, world, B) for _ in range(threads)]
    steps = [0] * threads
    for b in batches:
        b.run(5)
    start = threading.Barrier(threads + 1)

    def work(i):
        start.wait()
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            batches[i].run(10)
            steps[i] += 10

    ts = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
    for t in ts:
        t.start()
    start.wait()
    t0 = time.perf_counter()
    for t in ts:
        t.join()
    dt = time.perf_counter() - t0
    return B * cfg.num_agents * sum(steps) / dt, sum(steps), dt


def host_threads():
    """Threads for the all-cores CPU baseline: this GPU's CPU share of the host.  The GPU box
    runs one job per GPU and gives each its share of the machine (OMP_NUM_THREADS, 16 there;
    nproc shows the whole machine's 256); elsewhere, every CPU this process may run on."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS", "")
    if share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return max(1, n)


def cgroup_cpus():
    """CPUs this job's cgroup may use (cpu.max quota / period), or None when unlimited/unknown."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        return None if quota == "max" else round(int(quota) / int(period), 2)
    except (OSError, ValueError):
        return None


def host_cpu():
    """CPU model and nproc of this host (the GPU box's nproc counts the whole machine)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return f"{model}, nproc {os.cpu_count()}"


def cpu_baseline(world, H, W, N, F, C, seconds):
    """The oracle (CPU restatement, oracle/mapf_oracle.c) timed on this host on a bounded sample:
    32 envs per thread sharing the workload's first map, stepped for ~`seconds/2` on one thread,
    then ~`seconds/2` on every thread of this GPU's CPU share (host_threads; SURVEY.md §8d: all
    host cores, count stated).  `value` and `cores` are that share's figures; `per_core_value`
    and `host_cores` let a reader scale to the whole machine."""
    from oracle import oracle as O
    world = world if world.ndim == 2 else world[0]
    B = 32
    cfg = O.make_config(H, W, N, F, C, human_mode=1, goal_mode=1, fix_choice=1, seed=1234)
    one, steps1, dt1 = _oracle_rate(O, cfg, world, B, seconds / 2, 1)
    P = host_threads()
    allc, stepsP, dtP = _oracle_rate(O, cfg, world, B, seconds / 2, P) if P > 1 else (one, steps1, dt1)
    host_cores = os.cpu_count() or P
    return {"value": round(allc, 1), "unit": "agent-steps/s", "cores": P, "kind": "port",
            "value_label": f"{P} of {host_cores} host cores (this GPU's CPU share of the box)",
            "cores_definition": "this GPU's CPU share of the host (OMP_NUM_THREADS, else the affinity mask)",
            "single_thread_value": round(one, 1), "per_core_value": round(allc / P, 1),
            # SURVEY.md §8d asks for all host cores: the box gives this job its share only (running
            # nproc threads there would time-slice the same share), so the whole machine's figure is
            # the measured per-thread rate x nproc -- an extrapolation, labelled as one
            "all_host_cores_value": round(allc / P * host_cores, 1),
            "all_host_cores_basis": f"extrapolated: measured per-thread rate of the {P}-thread run x {host_cores}",
            "cgroup_cpu_quota": cgroup_cpus(),
            "host_cores": host_cores, "host": host_cpu(),
            "sample": f"{P} threads x {B} envs x {N} agents, {H}x{W}, FOV {F}, {C} channels, random policy, "
                      f"{stepsP} lockstep env-batch steps (step+observe) in {dtP:.1f}s; one thread: {steps1} "
                      f"steps in {dt1:.1f}s; reference Python measured 3,442 agent-steps/s/core on the c2 "
                      f"shape (BASELINE.md)"}


# BASELINE.json configs as env-only workloads; envs are PER GPU.
#   c1  1 env x 4 agents, 10x10 warehouse, FOV 11           (the reference's CPU case)
#   c2  4096 x 8, 20x20 warehouse, FOV 11                   (headline: the default)
#   c4  8192 x 16 over 8 GPUs = 1024 per GPU, 40x40, FOV 9  (env part of the c4 training config)
#   c5  16384 x 64 over 8 GPUs = 2048 per GPU, 80x80 random maps p=0.3 (one per env, largest
#       4-connected component), FOV 11, 7 channels (BFS heuristic channel)
PRESETS = {
    "c1": dict(envs=1, agents=4, size=10, fov=11, channels=6, maps="warehouse"),
    "c2": dict(envs=4096, agents=8, size=20, fov=11, channels=6, maps="warehouse"),
    "c4": dict(envs=1024, agents=16, size=40, fov=9, channels=6, maps="warehouse"),
    "c5": dict(envs=2048, agents=64, size=80, fov=11, channels=7, maps="random"),
}


def make_maps(kind, B, H, W, rank):
    from mapf_amd.maps import generate_warehouse, keep_largest_component, random_map
    if kind == "warehouse":
        return generate_warehouse(H, W), True
    rng = np.random.default_rng(1234 + rank)
    return np.stack([keep_largest_component(random_map(rng, H, W, 0.3)) for _ in range(B)]), False


# committed rocprofv3 --pmc passes (WRITE_SIZE + FETCH_SIZE, tools/pmc_report.py), by the
# workload's (B, N, H, W, F, C), the kernel instantiation (mapf_rollout_plan) and slot buffers
C2, C4, C5 = (4096, 8, 20, 20, 11, 6), (1024, 16, 40, 40, 9, 6), (2048, 64, 80, 80, 11, 7)
PMC_REPORTS = {(C2, "observe_kernel", False): "r01_pmc_observe_c2.json",
               (C2, "step_observe_kernel", False): "r01_pmc_step_observe_c2.json",
               (C2, "rollout_random_kernel<false,4>", False): "r03c_pmc_rollout_c2.json",
               (C2, "rollout_random_kernel<true,4>", True): "r06u_pmc_rollout_c2_slots.json",
               (C4, "rollout_wide3_kernel<u64,1,false>", False): "r03b_pmc_rollout_wide3_c4.json",
               (C4, "rollout_wide3_kernel<u64,1,true>", True): "r06u_pmc_rollout_c4_slots.json",
               (C5, "rollout_wide_kernel<Row2,2,true>", False): "r03b_pmc_rollout_wide_c5.json",
               (C5, "rollout_wide_kernel<Row2,2,true>", True): "r06u_pmc_rollout_c5_slots.json"}


def pmc_traffic_per_step(B, N, H, W, F, C, kernel, slots=False):
    """HBM bytes per lockstep step of `kernel` (MB) from the committed PMC report of this
    workload (per launch / steps per launch) -- null where none is committed."""
    path = os.path.join(ROOT, "profiles", PMC_REPORTS.get(((B, N, H, W, F, C), kernel, bool(slots)), "-"))
    if not os.path.exists(path):
        return None
    with open(path) as f:
        rep = json.load(f)
    # WRITE + 2 x FETCH: FETCH_SIZE counts 64 B per 128-B line read, for these kernels' narrow reads as
    # for wide streams (round-5 calibration, profiles/r05_fetch_calibration.json); reports written
    # before it stored WRITE + FETCH as traffic_bytes
    t = rep["write_bytes"] + rep["fetch_bytes_x2"] if "fetch_bytes_x2" in rep else rep["traffic_bytes"]
    return t / rep.get("steps_per_launch", 1) / 1e6


def launch_ranks(n):
    """`--gpus N` with no launcher around us: start N ranks of this same command under
    torch.distributed.run (one process per GPU, 127.0.0.1 rendezvous) as a CHILD process and
    return its exit code -- this process has not touched the GPU (the reference's rollout fan-out,
    driver.py:84-94, is the same one-process-per-worker shape)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "1")))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", default="c2", choices=sorted(PRESETS),
                    help="BASELINE.json workload preset (c2 = the headline metric); explicit flags override")
    ap.add_argument("--steps", type=int, default=1024)
    ap.add_argument("--warmup", type=int, default=64)
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU")
    ap.add_argument("--agents", type=int, default=None)
    ap.add_argument("--size", type=int, default=None)
    ap.add_argument("--fov", type=int, default=None)
    ap.add_argument("--channels", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--path", default="rollout", choices=["rollout", "fused", "split"])
    ap.add_argument("--split", action="store_true", help="= --path split")
    ap.add_argument("--rollout-steps", type=int, default=256, help="steps per mapf_rollout_random launch")
    ap.add_argument("--inplace", action="store_true",
                    help="rollout path: every step re-writes the same [B]-leading buffers instead of slot t of "
                         "[T]-leading rollout buffers (the default, runner.py:104-115)")
    ap.add_argument("--slots", action="store_true", help=argparse.SUPPRESS)   # the default since round 4
    ap.add_argument("--slot-gb", type=float, default=40.0,
                    help="cap on the slot buffers (GB): launches of fewer steps where 256 slots would exceed it")
    ap.add_argument("--tune", default="",
                    help="launch forms, mapf_tuning fields of include/mapf.h as k=v[,k=v...] (identical results)")
    ap.add_argument("--graph-steps", type=int, default=24,
                    help="fused/split paths: steps per captured hipGraph, a multiple of 3; 0 = direct")
    ap.add_argument("--kernel-launches", type=int, default=None,
                    help="launches timed with HIP events for the roofline kernel (default: per path)")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: --envs per GPU (SURVEY.md §8d: 4096 per GPU); strong: --envs in total, "
                         "split evenly over the ranks")
    ap.add_argument("--no-paths", action="store_true",
                    help="skip the per-path breakdown (slot-buffer rollout, one launch per step)")
    args = ap.parse_args()
    if args.split:
        args.path = "split"
    preset = PRESETS[args.config]
    for k in ("envs", "agents", "size", "fov", "channels"):
        if getattr(args, k) is None:
            setattr(args, k, preset[k])

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    if world_size != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but the launcher started WORLD_SIZE={world_size} ranks")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # MAPF_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share devices round-robin;
    # RCCL refuses two ranks on one GPU).  The env path has no collective either way: the
    # backend only carries the barriers and the max-over-ranks time.
    backend = os.environ.get("MAPF_BENCH_BACKEND", "nccl")
    dev_idx = local_rank % max(1, torch.cuda.device_count()) if backend == "gloo" else local_rank
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    dist = None
    if world_size > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        world_size = dist.get_world_size()            # the ranks that actually joined
    # distinct GPUs under the ranks (a gloo rehearsal shares fewer devices round-robin)
    devices_used = min(world_size, max(1, torch.cuda.device_count())) if backend == "gloo" else world_size

    from mapf_amd.config import make_config
    from mapf_amd.env import BatchedMapfGym

    B, N, H, W, F, C = args.envs, args.agents, args.size, args.size, args.fov, args.channels
    if args.scaling == "strong":
        if B % world_size:
            raise SystemExit(f"--scaling strong: {B} envs do not split over {world_size} ranks")
        B //= world_size
    world, shared = make_maps(preset["maps"], B, H, W, rank)
    env = BatchedMapfGym(make_config(B, H, W, num_agents=N, fov=F, num_channel=C, human_mode="random",
                                     goal_mode="random", fix_choice=1, seed=1234, env_offset=rank * B,
                                     shared_map=shared), device=dev, tuning=args.tune)
    env.reset_seeded(world)
    path = args.path
    if path == "rollout" and not env.rollout_fused:
        path = "fused"                       # the one-launch rollout does not cover this config
    obs, vec, acts = env.obs, env.vec, env.actions
    K = args.steps
    slot_bytes = B * N * ((C * F * F + 4) * 4 + 4 + 45) + B * 4          # one step's slot of every buffer
    TS = max(1, min(args.rollout_steps, int(args.slot_gb * 1e9 // slot_bytes)))
    slotted = path == "rollout" and not args.inplace
    T = max(1, min(args.rollout_steps, K, TS if slotted else K))

    roll = None
    if slotted:    # [T]-slot rollout buffers (runner.py's per-rollout arrays): TS slots, launches of T <= TS steps
        roll = dict(actions=torch.zeros(TS, B, N, dtype=torch.int32, device=dev),
                    obs=torch.zeros(TS, B, N, C, F, F, device=dev), vec=torch.zeros(TS, B, N, 4, device=dev),
                    out={k: torch.zeros((TS,) + tuple(v.shape), dtype=v.dtype, device=dev)
                         for k, v in env.out.items()})

    launchers = {}

    def rollout(n):
        if roll is None:
            env.rollout_random(n)
        else:                        # slots [0, n): the call prepared once per launch length
            if n not in launchers:
                launchers[n] = env.rollout_launcher(n, slots=True, actions=roll["actions"][:n], obs=roll["obs"][:n],
                                                    vec=roll["vec"][:n], out={k: v[:n] for k, v in roll["out"].items()})
            launchers[n]()

    def one_step():
        if path == "split":
            env.step_random(acts)    # random policy's actions drawn in the step kernel
            env.observe(obs, vec)
        else:
            env.step_observe(acts, obs, vec, random_policy=True)

    # warm-up: the timed path and the per-step path of the breakdown
    for _ in range(args.warmup):
        one_step()
    if path == "rollout":
        rollout(T)                   # every launch of the roofline kernel runs T steps (rocprof averages agree)
    torch.cuda.synchronize()

    # fused: the K timed steps are replays of a hipGraph holding G consecutive steps
    # (every kernel of every step runs; the graph only removes host launch cost).  Not for
    # configs that step and observe in separate launches (N > 8 or C = 7): their search
    # work runs on a second stream joined two steps later, which a capture cannot hold
    # open, and at 30-200 us per step the host's launch cost is hidden anyway.
    G = args.graph_steps
    graph = None
    if path != "rollout" and G > 0 and env.fused:
        assert G % 3 == 0, "--graph-steps must be a multiple of 3"
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(G):
                one_step()
        torch.cuda.synchronize()
        graph.replay()               # these G steps are warm-up too
        torch.cuda.synchronize()

    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if path == "rollout":
        done = 0
        while done < K:
            n = min(T, K - done)
            rollout(n)
            done += n
    else:
        n_replay, n_direct = (K // G, K % G) if graph is not None else (0, K)
        for _ in range(n_replay):
            graph.replay()
        for _ in range(n_direct):
            one_step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # Per-kernel timing: HIP events around each launch on the launch stream
    # (torch's current stream, which the env launches on), direct launches.
    #  rollout: each mapf_rollout_random launch of T steps -- the roofline kernel;
    #  fused:   one step_observe launch per step (previous step's search riding in it);
    #  split:   step / search flushed alone / observe.
    def event_ms(fn, n):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        for a, b in ev:
            a.record()
            fn()
            b.record()
        torch.cuda.synchronize()
        return float(np.mean([a.elapsed_time(b) for a, b in ev]))

    KT = args.kernel_launches or (max(1, min(20, K // T)) if path == "rollout" else min(K, 300))
    # every breakdown path is warmed up before it is timed (first launches of a path pay code
    # object loads, instruction-cache misses and, for the split path, its first search work),
    # and timed over at least 100 launches whatever --steps is
    KS = min(max(K, 100), 300)
    for _ in range(20):
        env.step_observe(acts, obs, vec, random_policy=True)
    fused_ms = event_ms(lambda: env.step_observe(acts, obs, vec, random_policy=True), KS)
    env.flush()
    for _ in range(20):
        env.step_random(acts)
        env.flush()
        env.observe(obs, vec)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(KS)]
    for k in range(KS):
        e0, e1, e2, e3 = ev[k]
        e0.record()
        env.step_random(acts)
        e1.record()
        env.flush()
        e2.record()
        env.observe(obs, vec)
        e3.record()
    torch.cuda.synchronize()
    step_ms = float(np.mean([ev[k][0].elapsed_time(ev[k][1]) for k in range(KS)]))
    search_ms = float(np.mean([ev[k][1].elapsed_time(ev[k][2]) for k in range(KS)]))
    obs_ms = float(np.mean([ev[k][2].elapsed_time(ev[k][3]) for k in range(KS)]))
    # the roofline kernel is timed over launches of --rollout-steps steps (the production launch
    # length, the reference's N_STEPS = 256) whatever --steps is: a short timed run (one launch
    # of K < 256 steps) pays the launch's ramp once over few steps, which `value` includes
    TR = TS if roll is not None else max(1, args.rollout_steps)
    if path == "rollout":
        KT = args.kernel_launches or max(3, min(20, K // T))
        if TR != T:
            rollout(TR)
            torch.cuda.synchronize()
    roll_ms = event_ms(lambda: rollout(TR), KT) if path == "rollout" else None

    # The same workload down each path, each with its own roofline fraction:
    #  rollout_inplace  mapf_rollout_random, every step re-writes the [B]-leading buffers
    #                   (95 MB at c2: they stay resident in the 256 MiB Infinity Cache);
    #  rollout_slots    mapf_rollout_random, step t writes slot t of [T]-leading rollout
    #                   buffers (runner.py:104-115's per-rollout arrays): every store is a
    #                   fresh HBM line;
    #  step_observe     one launch per step (the policy-in-the-loop path).
    paths = None
    if rank == 0 and not args.no_paths:
        bpa_f = fused_bytes_per_agent(C, F, H, W, N)

        def entry(ms_step, bpa, note):
            gbs = bpa * B * N / (ms_step * 1e-3) / 1e9
            return {"ms_per_step": round(ms_step, 5), "agent_steps_per_s": round(B * N / (ms_step * 1e-3), 1),
                    "achieved_gbs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                    "bytes_per_agent_step": round(bpa, 2), "timing": note}
        paths = {}
        if env.fused:
            paths["step_observe"] = entry(fused_ms, bpa_f, f"HIP events, {KS} direct launches")
        else:   # mapf_step_observe = step launch, then observe with the step's search forked beside it
            paths["split"] = entry(fused_ms, bpa_f, f"HIP events around {KS} mapf_step_observe calls (step, "
                                                    f"observe + forked search; breakdown_ms.split has them serial)")
        def entry_inplace(ms_step, bpa, note):
            e = entry(ms_step, bpa, note)
            if B * N * C * F * F * 4 < 128e6:
                # re-written in place, the buffer stays in the 256 MiB Infinity Cache (the PMC EA writes
                # equal the algorithmic bytes but are absorbed on-die): no HBM roofline applies
                e["frac"] = None
                e["bound"] = ("infinity_cache: the %.0f MB [B] buffer is re-written every step and stays resident; "
                              "the HBM-bound form of the same work is rollout_slots" % (B * N * C * F * F * 4 / 1e6))
            return e
        if env.rollout_fused:
            if roll is None:
                paths["rollout_inplace"] = entry_inplace(roll_ms / TR, bpa_f, f"HIP events, {KT} launches of {TR} steps")
                TS2 = min(TS, max(8, int(25e9 // slot_bytes)))   # <= ~25 GB of slots
                sl = dict(actions=torch.zeros(TS2, B, N, dtype=torch.int32, device=dev),
                          obs=torch.zeros(TS2, B, N, C, F, F, device=dev), vec=torch.zeros(TS2, B, N, 4, device=dev),
                          out={k: torch.zeros((TS2,) + tuple(v.shape), dtype=v.dtype, device=dev)
                               for k, v in env.out.items()})
                run_sl = lambda: env.rollout_random(TS2, slots=True, **sl)   # noqa: E731
                run_sl()
                ms = event_ms(run_sl, max(2, min(8, KT)))
                paths["rollout_slots"] = entry(ms / TS2, bpa_f, f"HIP events, {max(2, min(8, KT))} launches of "
                                                                f"{TS2} steps, {TS2} slots")
                del sl
                torch.cuda.empty_cache()
            else:
                paths["rollout_slots"] = entry(roll_ms / TR, bpa_f, f"HIP events, {KT} launches of {TR} steps")
                run_ip = lambda: env.rollout_random(args.rollout_steps)   # noqa: E731
                run_ip()
                ms = event_ms(run_ip, max(3, min(8, KT)))
                paths["rollout_inplace"] = entry_inplace(ms / args.rollout_steps, bpa_f,
                                                         f"HIP events, {max(3, min(8, KT))} launches of "
                                                         f"{args.rollout_steps} steps")
    counters = env.counters()

    if rank == 0:
        total_agent_steps = world_size * B * N * K
        value = total_agent_steps / elapsed
        if path == "rollout":
            # the template instantiation the library launched (mapf_rollout_plan), e.g.
            # rollout_random_kernel<true,4> at c2 (slot buffers, the 16 waves of a CU in one workgroup)
            kname = env.rollout_kernel_name(slots=roll is not None)
            bpa, kms, steps_pl = fused_bytes_per_agent(C, F, H, W, N), roll_ms, TR
        elif path == "split" or not env.fused:   # two launches per step: the observe kernel is the roofline one
            kname, bpa, kms, steps_pl = "observe_kernel", observe_bytes_per_agent(C, F, H, W, N), obs_ms, 1
        else:
            kname, bpa, kms, steps_pl = "step_observe_kernel", fused_bytes_per_agent(C, F, H, W, N), fused_ms, 1
        achieved = bpa * B * N * steps_pl / (kms * 1e-3) / 1e9
        traffic = pmc_traffic_per_step(B, N, H, W, F, C, kname, slots=roll is not None)
        ic_resident = path == "rollout" and roll is None and B * N * C * F * F * 4 < 128e6
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "agent-steps/s", "n_gpus": world_size,
            "steps": K, "warmup": args.warmup, "ms_per_step": round(elapsed / K * 1e3, 4),
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "int32",
            "data": "synthetic (seeded warehouse episodes on device, uniform random policy)",
            "config": {"workload": f"{args.config}: {B} envs x {N} agents per GPU, {H}x{W} "
                                   f"{'warehouse' if shared else 'random p=0.3 maps (one per env)'}, FOV {F}, "
                                   f"{C} channels, random policy, env.step+observe",
                       "num_envs_per_gpu": B, "num_agents": N, "grid": [H, W], "fov": F, "channels": C,
                       "human": "Human (random goals, device A*)", "goals": "lifelong, random", "keep_bfs": True,
                       "path": path + (f" (T={T} steps per launch, " + (f"[{TS}]-slot rollout buffers" if roll
                                                                         else "[B] buffers re-written in place") + ")"
                                       if path == "rollout" else ""),
                       "kernel_form": env.rollout_plan(slots=roll is not None) if path == "rollout" else None,
                       "total_envs": B * world_size,
                       "parallelism": f"env-shards x{world_size}",
                       "devices_used": devices_used,
                       "collective_backend": backend if world_size > 1 else None},
            "breakdown_ms": {"rollout_launch": round(roll_ms, 4) if roll_ms else None,
                             "rollout_per_step": round(roll_ms / TR, 5) if roll_ms else None,
                             "rollout_steps_per_launch": TR if roll_ms else None,
                             "step_observe_launch": round(fused_ms, 4),
                             "split": {"step_kernel": round(step_ms, 4), "search_kernel": round(search_ms, 4),
                                       "observe_kernel": round(obs_ms, 4)},
                             "timing": f"HIP events around direct launches ("
                                       + (f"{KT} rollout launches, " if path == "rollout" else "") + f"{KS} of each "
                                       f"per-step path; split: search flushed alone); value timed over the {path} "
                                       f"path" + (f" with hipGraph replays of {G} steps" if graph else "")},
            "roofline": {"kernel": kname, "bound": "infinity_cache" if ic_resident else "hbm",
                         "achieved": round(achieved, 1),
                         "peak": None if ic_resident else HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": None if ic_resident else round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": round(traffic * steps_pl, 3) if traffic is not None else None,
                         "traffic_unit": "MB/launch (PMC: WRITE_SIZE + 2 x FETCH_SIZE)", "steps_per_launch": steps_pl,
                         "algorithmic_mb": round(bpa * B * N * steps_pl / 1e6, 3), "bytes_per_agent_step": bpa,
                         "agents_per_step": B * N,
                         "residency": ("--inplace: the re-written [B] observation buffer (%.0f MB) stays in the 256 MiB "
                                       "Infinity Cache, so no HBM roofline applies (the HBM-bound form of the same work "
                                       "is the default slot-buffer path)" % (B * N * C * F * F * 4 / 1e6))
                         if ic_resident else "HBM: every store a fresh line" if roll is not None else "HBM"},
            "device_counters": [int(x) for x in counters[:8]],
        }
        if paths:
            line["paths"] = paths
        # States the reference does not survive, counted and resolved on the device:
        # empty viable sets (it raises) and fixActions deadlocks (it never returns).  Any other
        # counter is an impossible state: the line is then marked invalid.
        line["reference_unsurvivable_states"] = {"empty_viable": int(counters[2]), "fix_deadlock": int(counters[1])}
        bad = {i: int(counters[i]) for i in (0, 3, 4, 5, 6) if counters[i]}
        if bad:
            line["valid"] = False
            line["invalid_reason"] = f"device error counters {bad}"
            print(f"bench: device error counters {bad}", file=sys.stderr)
        if devices_used < world_size:
            line["rehearsal"] = (f"{world_size} ranks on {devices_used} GPU(s) (MAPF_BENCH_BACKEND={backend}): "
                                 "exercises the multi-rank launch, barriers and max-over-ranks timing; "
                                 "not a scaling result")
        if B * N < 1024:
            line["note"] = (f"{B * N} agents per GPU: one rollout step is a chain of dependent wave-level "
                            "phases (latency-bound, a few us), so a single CPU thread stepping small "
                            "batches can be faster; the GPU path is for thousands of envs (c2-c5)")
        if not args.no_cpu:
            # north_star: "1/2/4/8-GPU throughput and the CPU baseline reported in the same run" -- so
            # every line carries it, multi-rank ones too: rank 0 times it after the timed region and
            # the final barrier (the other ranks' GPU work is done), on a shorter sample when N > 1
            secs = args.cpu_seconds if world_size == 1 else min(args.cpu_seconds, 6.0)
            line["cpu_baseline"] = cpu_baseline(world, H, W, N, F, C, secs)
            if world_size > 1:
                line["cpu_baseline"]["timed_on"] = (f"rank 0's host after the {world_size}-rank timed region "
                                                    f"(other ranks idle), {secs:.0f} s sample")
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    env.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
