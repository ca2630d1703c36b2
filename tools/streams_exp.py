"""Experiment: the c2 batch split into S env shards (one handle each, env_offset
like the multi-GPU shards) stepped on S HIP streams, so one shard's latency-bound
step phase can overlap another shard's observation store drain.

Prints one line per variant: us per lockstep step of ALL envs.
"""
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
world = generate_warehouse(H, H)
obs = torch.zeros(B, N, C, F, F, device=dev)
vec = torch.zeros(B, N, 4, device=dev)


def make(S):
    envs = []
    for s in range(S):
        bs = B // S
        e = BatchedMapfGym(make_config(bs, H, H, num_agents=N, fov=F, num_channel=C, human_mode="random",
                                       goal_mode="random", fix_choice=1, seed=1234, env_offset=s * bs,
                                       shared_map=True), device=dev)
        e.reset_seeded(world)
        envs.append((e, obs[s * bs:(s + 1) * bs], vec[s * bs:(s + 1) * bs]))
    return envs


def run_direct(S, delay):
    envs = make(S)
    streams = [torch.cuda.Stream() for _ in range(S)]
    cur = torch.cuda.current_stream()
    for _ in range(30):
        for e, o, v in envs:
            e.step_observe(e.actions, o, v, random_policy=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s, st in enumerate(streams):
        st.wait_stream(cur)
        if delay and s:
            with torch.cuda.stream(st):
                torch.cuda._sleep(delay * s)
    for _ in range(K):
        for (e, o, v), st in zip(envs, streams):
            with torch.cuda.stream(st):
                e.step_observe(e.actions, o, v, random_policy=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    for e, _, _ in envs:
        e.close()
    return dt / K * 1e6


def run_graph(S, delay, G=24):
    envs = make(S)
    streams = [torch.cuda.Stream() for _ in range(S)]
    for _ in range(30):
        for e, o, v in envs:
            e.step_observe(e.actions, o, v, random_policy=True)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream()
    with torch.cuda.graph(g, stream=cap):
        for s, st in enumerate(streams):
            st.wait_stream(cap)
        for s, ((e, o, v), st) in enumerate(zip(envs, streams)):
            with torch.cuda.stream(st):
                if delay and s:
                    torch.cuda._sleep(delay * s)
                for _ in range(G):
                    e.step_observe(e.actions, o, v, random_policy=True)
        for st in streams:
            cap.wait_stream(st)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K // G):
        g.replay()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    for e, _, _ in envs:
        e.close()
    return dt / (K // G * G) * 1e6


for S, delay, mode in [(1, 0, "graph"), (1, 0, "direct"), (2, 0, "direct"), (2, 10000, "direct"),
                       (2, 20000, "direct"), (2, 0, "graph"), (2, 10000, "graph"), (2, 20000, "graph"),
                       (4, 0, "direct"), (4, 6000, "direct"), (4, 6000, "graph"), (2, 40000, "graph")]:
    us = (run_graph if mode == "graph" else run_direct)(S, delay)
    print(f"S={S} delay={delay} {mode}: {us:.2f} us/step  {B * N / us * 1e6:.3e} agent-steps/s", flush=True)
