"""diag_graph19: the captured reduction's output is right on the first replay and wrong later, with or
without churn, through .backward() or autograd.grad.  Hypothesis: a split (multi-block, "global")
reduction's zeroed semaphores -- a hipMemsetAsync in the captured stream -- are not re-zeroed on
replay, so the last-block test fails and the output is never written (stale block contents).
Each case captures one op with a STATIC input; between replays the output is poisoned with NaN, so
an output the replay does not write shows up.
  memset   a raw hipMemsetAsync(buf, 0) + buf.add_(1) captured; buf poisoned to 7 between replays"""
import ctypes
import sys

import torch


def case(name, x, fn):
    out = {}

    def body():
        out["y"] = fn(x)
    for _ in range(2):
        body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            body()
    torch.cuda.current_stream().wait_stream(s)
    ref = fn(x)
    res = []
    for _ in range(5):
        out["y"].fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        res.append(bool(torch.allclose(out["y"], ref, rtol=1e-5, atol=1e-5)))
    print(f"{name:40s} replay output == eager after NaN poison: {res}", flush=True)


def memset_case():
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    buf = torch.zeros(64, dtype=torch.int32, device="cuda")
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            rc = hip.hipMemsetAsync(ctypes.c_void_p(buf.data_ptr()), 0, 256, ctypes.c_void_p(s.cuda_stream))
            buf.add_(1)
    torch.cuda.current_stream().wait_stream(s)
    res = []
    for _ in range(5):
        buf.fill_(7)
        g.replay()
        torch.cuda.synchronize()
        res.append(int(buf.max()))
    print(f"{'captured hipMemsetAsync(0) + add_(1)':40s} rc {rc}; buf after replays (want 1): {res}", flush=True)


torch.manual_seed(0)
x = torch.randn(1088, 1536, device="cuda")
case("x32[1088,1536].sum(0)", x, lambda t: t.sum(0))
case("x32[64,1536].sum(0)", x[:64].contiguous(), lambda t: t.sum(0))
case("x32[8192,1536].sum(0)", torch.randn(8192, 1536, device="cuda"), lambda t: t.sum(0))
case("x32[1088,1536].sum()", x, lambda t: t.sum().reshape(1))
case("x16[1088,1536].sum(0)", x.half(), lambda t: t.sum(0).float())
case("x32[1088,1536].sum(1)", x, lambda t: t.sum(1))
case("x32[1088,1536].pow(2).mean()", x, lambda t: t.pow(2).mean().reshape(1))
memset_case()
sys.stdout.flush()
