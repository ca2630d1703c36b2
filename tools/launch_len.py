"""Rollout launch length vs time: HIP-event time of one mapf_rollout_random launch of T steps
for several T (c2 workload by default), to separate the per-launch overhead from the per-step
cost (time = a + b * T)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "primal-ppo_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from mapf_amd.config import make_config  # noqa: E402
from mapf_amd.env import BatchedMapfGym  # noqa: E402

cfg = os.environ.get("CFG", "c2")
p = bench.PRESETS[cfg]
B, N, H, F, C = p["envs"], p["agents"], p["size"], p["fov"], p["channels"]
world, shared = bench.make_maps(p["maps"], B, H, H, 0)
env = BatchedMapfGym(make_config(B, H, H, num_agents=N, fov=F, num_channel=C, human_mode="random",
                                 goal_mode="random", fix_choice=1, seed=1234, shared_map=shared), tuning=os.environ.get("TUNE", ""))
env.reset_seeded(world)
env.rollout_random(64)
torch.cuda.synchronize()
res = []
for T in (1, 2, 5, 10, 20, 40, 80, 160):
    ts = []
    for _ in range(6):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        env.rollout_random(T)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ms = float(np.median(ts))
    res.append((T, ms))
    print(f"{cfg} T={T:4d}: {ms * 1e3:8.1f} us  ({ms * 1e3 / T:6.2f} us/step)", flush=True)
Ts, ms = np.array(res).T
b1, a1 = np.polyfit(Ts, ms * 1e3, 1)
print(f"fit: {a1:.1f} us per launch + {b1:.2f} us per step")
