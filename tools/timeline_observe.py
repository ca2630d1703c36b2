"""Block timeline of the standalone observe kernel (MAPF_STAMPS diagnostic build),
for the configs whose step is not fused (c4, c5): bench.py presets.

    CONFIG=c5 python tools/timeline_observe.py   (uses primal-ppo_amd/lib/libmapf_stamps.so)

Stamps per workgroup (100 MHz realtime): 0 start, 1 state staged (loads issued
and stored), 2 after the block barrier, 4 after observation phases 1-3 (LDS
bit-stream built), 3 float4 stores issued.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "primal-ppo_amd")]
os.environ.setdefault("MAPF_LIB", os.path.join(ROOT, "primal-ppo_amd", "lib", "libmapf_stamps.so"))

import torch  # noqa: E402

import bench  # noqa: E402
from mapf_amd.config import make_config  # noqa: E402
from mapf_amd.env import BatchedMapfGym  # noqa: E402


def q(x):
    x = np.asarray(x, dtype=np.float64) / 100.0
    return "min %7.2f  p10 %7.2f  p50 %7.2f  p90 %7.2f  max %7.2f us" % tuple(np.percentile(x, [0, 10, 50, 90, 100]))


def main():
    p = bench.PRESETS[os.environ.get("CONFIG", "c5")]
    B, N, H, F, C = p["envs"], p["agents"], p["size"], p["fov"], p["channels"]
    world, shared = bench.make_maps(p["maps"], B, H, H, 0)
    env = BatchedMapfGym(make_config(B, H, H, num_agents=N, fov=F, num_channel=C, human_mode="random",
                                     goal_mode="random", fix_choice=1, seed=1234, shared_map=shared))
    env.reset_seeded(world)
    for _ in range(30):
        env.step_random()
        env.observe()
    torch.cuda.synchronize()
    E = max(64 // N, 1)
    nblk = (B + E - 1) // E
    for rep in range(3):
        for _ in range(4):
            env.step_random()
            env.observe()
        torch.cuda.synchronize()
        tl = env.timeline(min(nblk, 8192)).astype(np.int64)
        t0 = tl[:, 0].min()
        print(f"--- launch {rep}: {nblk} blocks, span {(tl[:, 3].max() - t0) / 100:.2f} us")
        print("  starts           ", q(tl[:, 0] - t0))
        print("  stage state      ", q(tl[:, 1] - tl[:, 0]))
        print("  barrier          ", q(tl[:, 2] - tl[:, 1]))
        print("  phases 1-3       ", q(tl[:, 4] - tl[:, 2]))
        print("  stores issue     ", q(tl[:, 3] - tl[:, 4]))
        print("  ends             ", q(tl[:, 3] - t0))


if __name__ == "__main__":
    main()
