"""A/B the two forms of mapf_attention_bwd_f16 (mapf_attention_bwd_select: 1 MFMA, 0 VALU) at the PPO
update's shapes: --seqs sequences (2,048 = a 256 x 8-row minibatch) of 17 tokens, 16 heads of 32 --
the first block (fused qkv, 17 query rows) and the last block (token 0's query, separate k / v).
Interleaved in one process; one JSON line per (round, shape, form) with us per call and the HBM rate
of the bytes it must move (q, k, v, o, dO in; dq, dk, dv out)."""
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
    ap.add_argument("--seqs", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    L = _lib.lib()
    B, n, d = args.seqs, 17, 512
    g = torch.Generator(device="cuda").manual_seed(0)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = lambda t, off=0: ctypes.c_void_p(t.data_ptr() + 2 * off)  # noqa: E731
    qkv = torch.randn(B, n, 3 * d, device="cuda", generator=g).half()
    q1, kv = torch.randn(B, d, device="cuda", generator=g).half(), torch.randn(B, n, 2 * d, device="cuda", generator=g).half()
    shapes = {
        "qkv_17_rows": dict(q=(qkv, 0), k=(qkv, d), v=(qkv, 2 * d), rows=n, q_ts=3 * d, q_ss=3 * d * n, kv_ts=3 * d,
                            kv_ss=3 * d * n, gq=torch.empty_like(qkv), gkv=None),
        "token0_query": dict(q=(q1, 0), k=(kv, 0), v=(kv, d), rows=1, q_ts=d, q_ss=d, kv_ts=2 * d, kv_ss=2 * d * n,
                             gq=torch.empty_like(q1), gkv=torch.empty_like(kv)),
    }
    for rnd in range(args.rounds):
        for name, sh in shapes.items():
            rows = sh["rows"]
            o = torch.randn(B, rows, d, device="cuda", generator=g).half()
            do = torch.randn(B, rows, d, device="cuda", generator=g).half()
            gq = sh["gq"]
            gkv = gq if sh["gkv"] is None else sh["gkv"]
            koff = sh["k"][1] if sh["gkv"] is None else 0
            voff = sh["v"][1] if sh["gkv"] is None else d
            nbytes = 2 * (B * rows * d * 3 + B * n * d * 2) + 2 * (B * rows * d + B * n * d * 2)
            for form in (0, 1):
                _lib.check(L.mapf_attention_bwd_select(form))
                fn = lambda: L.mapf_attention_bwd_f16(  # noqa: E731
                    p(*sh["q"]), p(*sh["k"]), p(*sh["v"]), p(o), p(do), p(gq, 0), p(gkv, koff), p(gkv, voff), B, n, rows,
                    sh["q_ts"], sh["q_ss"], sh["kv_ts"], sh["kv_ss"], d, rows * d, 16, 32, d ** -0.5, st)
                for _ in range(3):
                    _lib.check(fn())
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / args.iters
                print(json.dumps({"round": rnd, "shape": name, "form": "mfma" if form else "valu", "us": round(us, 1),
                                  "tb_s": round(nbytes / us / 1e6, 2)}), flush=True)
    _lib.check(L.mapf_attention_bwd_select(1))


if __name__ == "__main__":
    main()
