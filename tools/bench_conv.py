"""Time mapf_conv_nhwc_f16 / mapf_conv_first_f32 builds on the acting forward's shapes (c3: 32,768
agents, FOV 9) -- each library given on the command line is loaded side by side in one process
(experiment builds of csrc/mapf_conv.hip with other tile configurations), checked against torch's
conv at a small batch, then timed with HIP events.  Prints one line per (library, shape)."""
import argparse
import ctypes
import json

import torch

SHAPES = [("conv1a", 128, 128, 3, 9), ("conv2", 128, 256, 2, 4), ("conv2a", 256, 256, 2, 5), ("conv2b", 256, 256, 2, 6)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--agents", type=int, default=32768)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = "cuda"
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa
    cl = torch.channels_last
    libs = [(path, ctypes.CDLL(path)) for path in args.libs]
    for name, ci, co, ks, H in SHAPES:
        Ho = H + 2 - ks + 1
        flop = 2.0 * args.agents * Ho * Ho * co * ci * ks * ks
        g = torch.Generator(device=dev).manual_seed(1)
        w = (torch.randn(co, ci, ks, ks, device=dev, generator=g) / (ci * ks * ks) ** 0.5).half()
        b = torch.randn(co, device=dev, generator=g).half()
        wp = w.permute(0, 2, 3, 1).contiguous()
        xs = torch.randn(64, ci, H, H, device=dev, generator=g).half().contiguous(memory_format=cl)
        ref = torch.relu((torch.nn.functional.conv2d(xs.float(), w.float(), None, 1, 1).half().float()
                          + b.float().view(1, -1, 1, 1)).half().float()).half()
        x = torch.randn(args.agents, ci, H, H, device=dev, generator=g).half().contiguous(memory_format=cl)
        y = torch.empty(args.agents, co, Ho, Ho, dtype=torch.float16, device=dev).contiguous(memory_format=cl)
        for path, L in libs:
            ys = torch.full((64, co, Ho, Ho), float("nan"), dtype=torch.float16, device=dev).contiguous(memory_format=cl)
            rc = L.mapf_conv_nhwc_f16(p(xs), p(wp), p(b), p(ys), 64, H, H, ci, co, ks, 1, 1, st)
            torch.cuda.synchronize()
            err = (ys.float() - ref.float()).abs().max().item() if rc == 0 else float("nan")
            for _ in range(3):
                L.mapf_conv_nhwc_f16(p(x), p(wp), p(b), p(y), args.agents, H, H, ci, co, ks, 1, 1, st)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                L.mapf_conv_nhwc_f16(p(x), p(wp), p(b), p(y), args.agents, H, H, ci, co, ks, 1, 1, st)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.iters
            print(json.dumps({"lib": path.split("/")[-1], "shape": name, "rc": rc, "max_err": err, "us": round(us, 1),
                              "tflops": round(flop / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
