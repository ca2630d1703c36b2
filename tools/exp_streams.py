"""Experiment: does the c3 acting forward gain from running batch chunks on two HIP streams (kernels of
different kinds overlapping each other's latency / VALU-bound phases)?  Times SCRIMPNet's acting
forward (no grad, _forward_fused) on 4096 x 8 agents: whole batch; K chunks in order on one stream;
K chunks alternating over two streams.  Prints one JSON line.

    python tools/exp_streams.py [--envs 4096] [--chunks 2] [--reps 10]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "primal-ppo_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--agents", type=int, default=8)
    ap.add_argument("--chunks", type=int, default=2)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    from mapf_amd.model import Model
    dev = torch.device("cuda", 0)
    B, N = args.envs, args.agents
    model = Model(0, dev, global_model=False, numChannel=6, num_agents=N, fov=9)
    net = model.network
    obs = (torch.rand(B, N, 6, 9, 9, device=dev) < 0.2).float()
    vec = torch.randn(B, N, 4, device=dev)
    K = args.chunks
    cb = B // K
    streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]

    def whole():
        net(obs, vec)

    def chunks_one():
        for k in range(K):
            net(obs[k * cb:(k + 1) * cb], vec[k * cb:(k + 1) * cb])

    def chunks_two():
        main_s = streams[0]
        streams[1].wait_stream(main_s)
        for k in range(K):
            with torch.cuda.stream(streams[k % 2]):
                net(obs[k * cb:(k + 1) * cb], vec[k * cb:(k + 1) * cb])
        main_s.wait_stream(streams[1])

    res = {}
    with torch.no_grad():
        for name, fn in (("whole", whole), ("chunks_one_stream", chunks_one), ("chunks_two_streams", chunks_two)) * 2:
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.reps):
                fn()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / args.reps * 1e3
            res.setdefault(name, []).append(round(ms, 3))
            print(f"{name}: {ms:.3f} ms", flush=True)
    print(json.dumps({"agents": B * N, "chunks": K, "ms": res}), flush=True)


if __name__ == "__main__":
    main()
