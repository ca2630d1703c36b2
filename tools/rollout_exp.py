"""Experiment: c2 random-policy steps per second through mapf_rollout_random
(T steps per launch) vs one mapf_step_observe_random launch per step."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "primal-ppo_amd")]

import torch  # noqa: E402

from mapf_amd.config import make_config  # noqa: E402
from mapf_amd.env import BatchedMapfGym  # noqa: E402
from mapf_amd.maps import generate_warehouse  # noqa: E402

B, N, H, F, C = 4096, 8, 20, 11, 6
K = int(os.environ.get("K", "960"))
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
env = BatchedMapfGym(make_config(B, H, H, num_agents=N, fov=F, num_channel=C, human_mode="random",
                                 goal_mode="random", fix_choice=1, seed=1234), device=dev)
env.reset_seeded(generate_warehouse(H, H))
print("rollout fused:", env.rollout_fused, flush=True)


def timed(fn, steps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    while n < K:
        fn()
        n += steps
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


for T in (8, 24, 96):
    us = timed(lambda: env.rollout_random(T), T)
    print(f"rollout T={T} slots=0: {us:.2f} us/step {B * N / us * 1e6:.3e} agent-steps/s", flush=True)
for T in (24,):
    bufs = dict(actions=torch.zeros(T, B, N, dtype=torch.int32, device=dev),
                obs=torch.zeros(T, B, N, C, F, F, device=dev), vec=torch.zeros(T, B, N, 4, device=dev),
                out={k: torch.zeros((T,) + tuple(v.shape), dtype=v.dtype, device=dev) for k, v in env.out.items()})
    us = timed(lambda: env.rollout_random(T, slots=True, **bufs), T)
    print(f"rollout T={T} slots=1: {us:.2f} us/step {B * N / us * 1e6:.3e} agent-steps/s", flush=True)
    del bufs
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for _ in range(24):
        env.step_observe(random_policy=True)
us = timed(g.replay, 24)
print(f"step_observe graph x24: {us:.2f} us/step {B * N / us * 1e6:.3e} agent-steps/s", flush=True)
print("counters", env.counters()[:8])
