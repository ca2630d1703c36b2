import os, sys
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "primal-ppo_amd")]
import torch, bench
from mapf_amd.config import make_config
from mapf_amd.env import BatchedMapfGym
for cfgname in ("c5", "c4", "c2"):
    p = bench.PRESETS[cfgname]
    B, N, H, F, C = p["envs"], p["agents"], p["size"], p["fov"], p["channels"]
    world, shared = bench.make_maps(p["maps"], B, H, H, 0)
    env = BatchedMapfGym(make_config(B, H, H, num_agents=N, fov=F, num_channel=C, human_mode="random",
                                     goal_mode="random", fix_choice=1, seed=1234, shared_map=shared))
    env.reset_seeded(world)
    for _ in range(50):
        env.step_random(); env.observe()
    tot = [0, 0]
    for _ in range(30):
        env.step_random()
        c = env.counters()
        tot[0] += int(c[8:11].sum()); tot[1] += int(c[12:15].sum())
        env.observe()
    print(cfgname, "per step: replans", tot[0] / 30, "bfs maps", tot[1] / 30, flush=True)
