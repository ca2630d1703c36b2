"""A/B the 512 x 512 fused linears' forms (row tiles: mapf_linear512_select 2 / 1; K-ring stages:
mapf_linear512_stages 2 / 3 / 4) at the c3 acting
forward's shape (32,768 agents x 17 tokens = 557,056 rows), interleaved in one process on random
data.  Prints one JSON line per (round, kernel, row_tiles)."""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "primal-ppo_amd")]
from mapf_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32768 * 17)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--stages", default="2,3,4", help="K-ring stages to time")
    ap.add_argument("--only", default=None, help="comma-separated kernels (default: all)")
    ap.add_argument("--forms", default=None,
                    help="comma-separated row_tiles:stages:kdepth forms, e.g. 1:2:32,2:2:64 (default: row tiles 2 "
                         "and 1 x --stages at kdepth 32)")
    args = ap.parse_args()
    L = _lib.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    R = args.rows
    g = torch.Generator(device="cuda").manual_seed(0)
    a = torch.randn(R, 512, device="cuda", generator=g).half()
    w = (torch.randn(512, 512, device="cuda", generator=g) / 512 ** 0.5).half()
    b = (torch.randn(512, device="cuda", generator=g) * 0.1).half()
    gamma, beta = torch.ones(512, device="cuda"), torch.zeros(512, device="cuda")
    out = torch.empty(R, 512, dtype=torch.float16, device="cuda")
    x = torch.randn(R, 512, device="cuda", generator=g)
    z = torch.empty(R, 512, dtype=torch.float16, device="cuda")
    tA = torch.rand(R // 17, 16, device="cuda", generator=g)
    tVV = torch.randn(R // 17, 512, device="cuda", generator=g).half()
    tcls, tpos = torch.randn(512, device="cuda", generator=g), torch.randn(17, 512, device="cuda", generator=g)
    kern = {"gelu_dropout": lambda: L.mapf_linear512_gelu_dropout(p(a), p(w), p(b), p(out), R, 0.2, 1, st),
            "residual_layernorm": lambda: L.mapf_linear512_residual_layernorm(p(a), p(w), p(b), p(x), p(gamma), p(beta),
                                                                               p(z), R, 1e-5, 0.2, 2, st),
            "rows_x17": lambda: L.mapf_linear512_residual_layernorm_rows(p(a), p(w), p(b), p(x), p(gamma), p(beta), p(z),
                                                                         R, 1e-5, 0.2, 3, 17, st),
            "tokens": lambda: L.mapf_linear512_tokens_residual_layernorm(p(a), p(w), p(b), p(x), p(gamma), p(beta), p(z),
                                                                         R // 17, 16, 1e-5, 0.2, 4, p(tA), p(tVV),
                                                                         p(tcls), p(tpos), 0.2, 5, st)}
    flop = 2.0 * R * 512 * 512
    for rnd in range(args.rounds):
        for name, fn in kern.items():
            if args.only and name not in args.only.split(","):
                continue
            forms = ([tuple(map(int, f.split(":"))) for f in args.forms.split(",")] if args.forms else
                     [(m, s_, 32) for m in (2, 1) for s_ in map(int, args.stages.split(","))])
            for mt, stages, kd in forms:
                _lib.check(L.mapf_linear512_select(mt))
                _lib.check(L.mapf_linear512_stages(stages))
                _lib.check(L.mapf_linear512_kdepth(kd))
                for _ in range(2):
                    _lib.check(fn())
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / args.iters
                print(json.dumps({"round": rnd, "kernel": name, "row_tiles": mt, "stages": stages, "kdepth": kd, "lib": os.path.basename(os.environ.get("MAPF_LIB", "libmapf.so")), "us": round(us, 1),
                                  "pflops": round(flop / us / 1e9, 3)}), flush=True)
    _lib.check(L.mapf_linear512_select(0))
    _lib.check(L.mapf_linear512_stages(0))
    _lib.check(L.mapf_linear512_kdepth(0))


if __name__ == "__main__":
    main()
