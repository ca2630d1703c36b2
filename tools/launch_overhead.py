"""Where the time of a short timed region goes (bench.py at --steps 20: ONE rollout launch of
20 steps): host wall around rollout()+synchronize vs the launch's HIP-event time, the host
time of the call alone, and an idle synchronize.

    python tools/launch_overhead.py [--steps 20] [--reps 30]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "primal-ppo_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--config", default="c2")
    a = ap.parse_args()
    from mapf_amd.config import make_config
    from mapf_amd.env import BatchedMapfGym
    p = bench.PRESETS[a.config]
    B, N, H, F, C = p["envs"], p["agents"], p["size"], p["fov"], p["channels"]
    world, shared = bench.make_maps(p["maps"], B, H, H, 0)
    env = BatchedMapfGym(make_config(B, H, H, num_agents=N, fov=F, num_channel=C, human_mode="random",
                                     goal_mode="random", fix_choice=1, seed=1234, shared_map=shared))
    env.reset_seeded(world)
    for _ in range(5):
        env.rollout_random(a.steps)
    torch.cuda.synchronize()
    wall, ev, call, idle = [], [], [], []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        env.rollout_random(a.steps)
        t1 = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        wall.append((t2 - t0) * 1e6)
        call.append((t1 - t0) * 1e6)
        ev.append(e0.elapsed_time(e1) * 1e3)
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        idle.append((time.perf_counter() - t3) * 1e6)
    med = lambda x: float(np.median(x))   # noqa: E731
    print(f"{a.config} T={a.steps}: wall {med(wall):.1f} us, HIP events {med(ev):.1f} us, host call {med(call):.1f} us, "
          f"idle sync {med(idle):.1f} us; wall/step {med(wall) / a.steps:.2f} us, kernel/step {med(ev) / a.steps:.2f} us",
          flush=True)


if __name__ == "__main__":
    main()
