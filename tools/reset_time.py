"""Seeded reset time per config (HIP events): mapf_reset with host maps, and the on-device
map generation + reset (mapf_reset_generated) -- both end with every agent's BFS map and
every human's first and next paths (reset_searches)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "primal-ppo_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from mapf_amd.config import make_config  # noqa: E402
from mapf_amd.env import BatchedMapfGym  # noqa: E402

for cfg in os.environ.get("CFGS", "c2,c4,c5").split(","):
    p = bench.PRESETS[cfg]
    B, N, H, F, C = p["envs"], p["agents"], p["size"], p["fov"], p["channels"]
    world, shared = bench.make_maps(p["maps"], B, H, H, 0)
    env = BatchedMapfGym(make_config(B, H, H, num_agents=N, fov=F, num_channel=C, human_mode="random",
                                     goal_mode="random", fix_choice=1, seed=1234, shared_map=shared))
    env.reset_seeded(world)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    env.reset_seeded(world)
    b.record()
    torch.cuda.synchronize()
    print(f"{cfg}: reset_seeded {a.elapsed_time(b):.1f} ms ({B * N} BFS maps, {B} human paths x 2)", flush=True)
    env.close()
