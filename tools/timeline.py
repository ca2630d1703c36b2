"""Block timeline of the fused step+observe kernel (MAPF_STAMPS diagnostic build).

    python tools/timeline.py        (uses primal-ppo_amd/lib/libmapf_stamps.so)

Each workgroup's thread 0 stamps the 100 MHz realtime counter at: 0 start,
1 step done (wave 0; search blocks: search done), 2 LDS ready (after the
block barrier), 3 observation stores issued.  Printed: quantiles of each
phase over the step blocks, start spread (dispatch ramp), and per-XCD spans.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "primal-ppo_amd")]
os.environ.setdefault("MAPF_LIB", os.path.join(ROOT, "primal-ppo_amd", "lib", "libmapf_stamps.so"))

import torch  # noqa: E402

from mapf_amd.config import make_config  # noqa: E402
from mapf_amd.env import BatchedMapfGym  # noqa: E402
from mapf_amd.maps import generate_warehouse  # noqa: E402


def q(x):
    x = np.asarray(x, dtype=np.float64) / 100.0     # 100 MHz ticks -> us
    return "min %6.2f  p10 %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f us" % tuple(np.percentile(x, [0, 10, 50, 90, 100]))


def main():
    B = int(os.environ.get("ENVS", "4096"))
    os.environ.setdefault("TUNE", "band_blocks=256")    # mapf_tuning fields (the zero band on by default here)
    env = BatchedMapfGym(make_config(B, 20, 20, num_agents=8, fov=11, num_channel=6, human_mode="random",
                                     goal_mode="random", fix_choice=1, seed=1234), tuning=os.environ.get("TUNE", ""))
    tu = env.tuning()
    nsearch, nband = tu["search_blocks"], tu["band_blocks"]
    env.reset_seeded(generate_warehouse(20, 20))
    for _ in range(60):
        env.step_observe(random_policy=True)
    torch.cuda.synchronize()
    nstep = (B + 3) // 4
    b2b = int(os.environ.get("BACK2BACK", "1"))    # launches back to back; the last one is recorded
    for rep in range(3):
        for _ in range(b2b):
            env.step_observe(random_policy=True)
        torch.cuda.synchronize()
        tl = env.timeline(nband + nsearch + nstep).astype(np.int64)
        t0 = tl[:, 0].min()
        bd, s, st = tl[:nband], tl[nband:nband + nsearch], tl[nband + nsearch:]
        end = max(st[:, 3].max(), s[:, 1].max(), bd[:, 1].max() if nband else 0)
        print(f"--- launch {rep}: span {(end - t0) / 100:.2f} us (first start -> last stamp)")
        print("  step starts      ", q(st[:, 0] - t0))
        print("  step (wave 0)    ", q(st[:, 1] - st[:, 0]))
        print("  barrier wait     ", q(st[:, 2] - st[:, 1]))
        print("  obs phases 1-3   ", q(st[:, 4] - st[:, 2]))
        print("  obs stores issue ", q(st[:, 3] - st[:, 4]))
        print("  block ends       ", q(st[:, 3] - t0))
        if nband:
            print("  band starts      ", q(bd[:, 0] - t0))
            print("  band blocks      ", q(bd[:, 1] - bd[:, 0]))
        print("  search starts    ", q(s[:, 0] - t0))
        print("  search blocks    ", q(s[:, 1] - s[:, 0]))
        xcc = tl[:, 7] & 0xF
        for x in np.unique(xcc):
            m = xcc[nband + nsearch:] == x
            print(f"  xcc {x}: {m.sum():4d} step blocks, start {(st[m, 0].min() - t0) / 100:5.2f}.."
                  f"{(st[m, 0].max() - t0) / 100:5.2f} us, end max {(st[m, 3].max() - t0) / 100:6.2f} us")


if __name__ == "__main__":
    main()
