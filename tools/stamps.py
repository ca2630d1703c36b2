"""Phase breakdown of the step kernel from the MAPF_STAMPS diagnostic build.

    MAPF_LIB=primal-ppo_amd/lib/libmapf_stamps.so python tools/stamps.py

Prints the mean s_memtime cycles per wave spent in each phase of step_kernel
(c2 workload).  Read the SHARES, not the absolute length: stamps serialise.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "primal-ppo_amd")]
os.environ.setdefault("MAPF_LIB", os.path.join(ROOT, "primal-ppo_amd", "lib", "libmapf_stamps.so"))

import torch  # noqa: E402

from mapf_amd.config import make_config  # noqa: E402
from mapf_amd.env import BatchedMapfGym  # noqa: E402
from mapf_amd.maps import generate_warehouse  # noqa: E402

PHASES = ["loads+masks", "conflicts(j-loop)", "status+reward+outputs", "fixActions", "move+goals",
          "human", "final outputs"]


def main():
    B = int(os.environ.get("ENVS", "4096"))
    env = BatchedMapfGym(make_config(B, 20, 20, num_agents=8, fov=11, num_channel=6, human_mode="random",
                                     goal_mode="random", fix_choice=1, seed=1234), tuning=os.environ.get("TUNE", ""))
    env.reset_seeded(generate_warehouse(20, 20))
    split = os.environ.get("SPLIT", "0") == "1"     # default: the fused step+observe launch
    roll = os.environ.get("ROLLOUT", "0") == "1"    # the multi-step rollout launch (last step's phases)

    def one():
        if roll:
            env.rollout_random(32)
        elif split:
            env.step_random()
            env.observe()
        else:
            env.step_observe(random_policy=True)
    for _ in range(50):
        one()
    torch.cuda.synchronize()
    env.profile(reset=True)
    n = 200
    for _ in range(n):
        one()
    torch.cuda.synchronize()
    p = env.profile(reset=False)     # sums over the waves of the last step launch
    waves = max(int(p[15]), 1)
    n = 1
    tot = sum(int(x) for x in p[:7])
    print(f"waves sampled: {waves} ({waves / n:.0f} per step)")
    for k, name in enumerate(PHASES):
        print(f"  {name:26s} {int(p[k]) / waves:9.0f} cycles/wave  {100.0 * int(p[k]) / max(tot, 1):5.1f}%")
    print(f"  {'total':26s} {tot / waves:9.0f} cycles/wave")
    # per-wave distribution of the last launch: percentiles of each phase, and the
    # mean breakdown of the slowest 5 % of waves
    import numpy as np
    wp = env.wave_profile(min(65536, 4096 * 2))
    wp = wp[wp[:, 7] == 1][:, :7].astype(np.float64)
    if len(wp):
        tot_w = wp.sum(1)
        print("per-wave percentiles (p10 / p50 / p90 / p99 / max cycles):")
        for k, name in enumerate(PHASES + ["total"]):
            col = tot_w if k == 7 else wp[:, k]
            print(f"  {name:26s} " + " / ".join(f"{v:8.0f}" for v in np.percentile(col, [10, 50, 90, 99, 100])))
        slow = wp[tot_w >= np.percentile(tot_w, 95)]
        print("slowest 5% of waves, mean cycles per phase:")
        for k, name in enumerate(PHASES):
            print(f"  {name:26s} {slow[:, k].mean():9.0f}")


if __name__ == "__main__":
    main()
