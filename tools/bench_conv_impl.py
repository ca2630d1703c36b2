"""A/B the two implicit-GEMM conv forms (mapf_conv_select: 2 image-resident, 0 per-tap staged) on
the c3 acting forward's shapes (32,768 agents, FOV 9), interleaved in one process: rounds x impls,
each timed with HIP events over --iters launches on random data, checked against torch at a small
batch first.  Prints one JSON line per (round, shape, impl)."""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "primal-ppo_amd")]
from mapf_amd import _lib  # noqa: E402

# (name, Cin, Cout, ks, H, pooled)
SHAPES = [("conv1a", 128, 128, 3, 9, False), ("conv1b_pool", 128, 128, 3, 9, True), ("conv2", 128, 256, 2, 4, False),
          ("conv2a", 256, 256, 2, 5, False), ("conv2b_pool", 256, 256, 2, 6, True)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=32768)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    L = _lib.lib()
    dev = "cuda"
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    cl = torch.channels_last
    data = {}
    for name, ci, co, ks, H, pool in SHAPES:
        Ho = H + 2 - ks + 1
        g = torch.Generator(device=dev).manual_seed(1)
        w = (torch.randn(co, ci, ks, ks, device=dev, generator=g) / (ci * ks * ks) ** 0.5).half()
        b = torch.randn(co, device=dev, generator=g).half()
        wp = w.permute(0, 2, 3, 1).contiguous()
        x = torch.randn(args.agents, ci, H, H, device=dev, generator=g).half().contiguous(memory_format=cl)
        Hy = Ho // 2 if pool else Ho
        y = torch.empty(args.agents, co, Hy, Hy, dtype=torch.float16, device=dev).contiguous(memory_format=cl)
        ref = torch.nn.functional.conv2d(x[:64].float(), w.float(), None, 1, 1).half().float() + b.float().view(1, -1, 1, 1)
        ref = torch.relu(ref.half().float())
        if pool:
            ref = torch.nn.functional.max_pool2d(ref, 2)
        data[name] = (ci, co, ks, H, pool, wp, b, x, y, ref.half(), 2.0 * args.agents * Ho * Ho * co * ci * ks * ks)

    def run(name, n):
        ci, co, ks, H, pool, wp, b, x, y, _, _ = data[name]
        if pool:
            return L.mapf_conv_nhwc_pool_f16(p(x), p(wp), p(b), p(y), n, H, H, ci, co, ks, 1, st)
        return L.mapf_conv_nhwc_f16(p(x), p(wp), p(b), p(y), n, H, H, ci, co, ks, 1, 1, st)

    for rnd in range(args.rounds):
        for name in data:
            for impl in (2, 0):
                _lib.check(L.mapf_conv_select(impl))
                *_, y, ref, flop = data[name]
                rc = run(name, 64)
                torch.cuda.synchronize()
                err = (y[:64].float() - ref.float()).abs().max().item() if rc == 0 else float("nan")
                for _ in range(3):
                    run(name, args.agents)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    run(name, args.agents)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / args.iters
                print(json.dumps({"round": rnd, "shape": name, "impl": impl, "rc": rc, "max_err": round(err, 5),
                                  "us": round(us, 1), "pflops": round(flop / us / 1e9, 3)}), flush=True)
    _lib.check(L.mapf_conv_select(1))


if __name__ == "__main__":
    main()
