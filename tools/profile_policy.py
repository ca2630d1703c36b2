"""Where the c3 rollout's time goes: the policy forward (SCRIMPNet under autocast)
on one rollout step's batch (4096 envs x 8 agents, FOV 9), torch profiler table.

    python tools/profile_policy.py [--envs 4096] [--agents 8]
"""
import argparse
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
    ap.add_argument("--nchw", action="store_true", help="keep the network NCHW")
    ap.add_argument("--no-find", action="store_true", help="torch.backends.cudnn.benchmark off (no MIOpen find)")
    ap.add_argument("--torch-path", action="store_true", help="the PyTorch forward, not the fused acting path")
    ap.add_argument("--miopen-conv", action="store_true", help="MIOpen for every convolution (no mapf_conv_nhwc_f16)")
    ap.add_argument("--unfused-linear", action="store_true", help="hipBLASLt linears + separate epilogue kernels")
    ap.add_argument("--no-profile", action="store_true")
    args = ap.parse_args()
    from mapf_amd.model import Model
    dev = torch.device("cuda", 0)
    B, N = args.envs, args.agents
    model = Model(0, dev, global_model=False, numChannel=6, num_agents=N, fov=9)
    obs = (torch.rand(B, N, 6, 9, 9, device=dev) < 0.2).float()
    vec = torch.randn(B, N, 4, device=dev)
    if args.nchw:
        model.network = model.network.to(memory_format=torch.contiguous_format)
    if args.no_find:
        torch.backends.cudnn.benchmark = False
    model.network.fused_acting = not args.torch_path
    model.network.own_conv = not args.miopen_conv
    model.network.fused_linear = not args.unfused_linear
    for _ in range(3):
        model.step(obs, vec, None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        model.step(obs, vec, None)
    torch.cuda.synchronize()
    print(f"model.step: {(time.perf_counter() - t0) / 10 * 1e3:.2f} ms for {B * N} agents "
          f"(own conv {model.network.own_conv}, fused linear {model.network.fused_linear})", flush=True)
    if args.no_profile:
        return
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        for _ in range(3):
            model.step(obs, vec, None)
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25), flush=True)


if __name__ == "__main__":
    main()
