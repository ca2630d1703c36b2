"""Experiment: where the split path's search launch spends its time at c4 / c5.
Per variant: HIP-event times of step / search (flushed alone) / observe per step, and the
work items per step (human replans, agent BFS maps) from the device counters."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "primal-ppo_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from mapf_amd.config import make_config  # noqa: E402
from mapf_amd.env import BatchedMapfGym  # noqa: E402

K = int(os.environ.get("K", "120"))
torch.cuda.set_device(0)
for cfgname in os.environ.get("CFGS", "c4,c5").split(","):
    p = bench.PRESETS[cfgname]
    B, N, H, F, C = p["envs"], p["agents"], p["size"], p["fov"], p["channels"]
    world, shared = bench.make_maps(p["maps"], B, H, H, 0)
    for human, keep_bfs, ch in (("random", True, C), ("random", False, 6), ("looping", True, C)):
        env = BatchedMapfGym(make_config(B, H, H, num_agents=N, fov=F, num_channel=ch, human_mode=human,
                                         goal_mode="random", fix_choice=1, seed=1234, shared_map=shared,
                                         keep_bfs=keep_bfs))
        env.reset_seeded(world)
        for _ in range(20):
            env.step_random()
            env.observe()
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(K)]
        items = np.zeros(2)
        for k in range(K):
            e0, e1, e2, e3 = ev[k]
            e0.record()
            env.step_random()
            e1.record()
            c = env.counters() if k % 10 == 0 else None
            e1b = torch.cuda.Event(enable_timing=True)
            env.flush()
            e2.record()
            env.observe()
            e3.record()
            if c is not None:
                items += [c[8:11].sum(), c[12:15].sum()]
        torch.cuda.synchronize()
        t = lambda a, b: float(np.median([ev[k][a].elapsed_time(ev[k][b]) for k in range(K)])) * 1e3  # noqa: E731
        print(f"{cfgname} human={human} keep_bfs={keep_bfs} C={ch}: step {t(0, 1):.1f} us, search {t(1, 2):.1f} us, "
              f"observe {t(2, 3):.1f} us; per step ~{items[0] / (K / 10):.1f} replans, {items[1] / (K / 10):.1f} BFS maps",
              flush=True)
        env.close()
