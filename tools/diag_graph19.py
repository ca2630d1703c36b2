"""diag_graph18's every-replay reproducer (loss through b.half().float(), b an fp32 leaf) under
variants that separate the autograd plumbing from the kernels:
  backward        .backward() into b.grad (set to None in the body)           -- fails in diag_graph18
  autograd.grad   torch.autograd.grad(loss, [w, b]) -- no AccumulateGrad node
  grad_inplace    b.grad preallocated before capture, body does .zero_() then .backward() accumulates in place
  no_churn        .backward(), replays without churn in between
  big_churn       .backward(), churn of >= 2 MiB tensors only (large pool)
  no_warmup       .backward(), capture without eager warm-ups
  same_stream     .backward(), warm-ups on the capture stream
For every churned replay: whether b's gradient equals the first replay's, its non-finite count and
max |diff|."""
import torch

SMALL = [1 << (k % 17) for k in range(2000)]
BIG = [(2 << 20) + (k << 12) for k in range(24)]


def churn(sizes):
    ts = [torch.full((n // 4,), float("nan"), device="cuda") for n in sizes]
    torch.cuda.synchronize()
    del ts


def run(variant, rows=1088, din=512, dout=1536):
    torch.manual_seed(0)
    w = torch.nn.Parameter(torch.randn(dout, din, device="cuda") * 0.05)
    b = torch.nn.Parameter(torch.randn(dout, device="cuda") * 0.05)
    x = torch.randn(rows, din, device="cuda")
    out = {}

    def loss_fn():
        y = (x.half() @ w.half().t()).float() * 0 + b.half().float()
        return y.float().pow(2).mean() * 256.0

    def body():
        if variant == "autograd.grad":
            out["gw"], out["gb"] = torch.autograd.grad(loss_fn(), [w, b])
            return
        if variant == "grad_inplace":
            w.grad.zero_()
            b.grad.zero_()
        else:
            w.grad = b.grad = None
        loss_fn().backward()
        out["gw"], out["gb"] = w.grad, b.grad

    if variant == "grad_inplace":
        w.grad, b.grad = torch.zeros_like(w), torch.zeros_like(b)
    cap = torch.cuda.Stream()
    if variant != "no_warmup":
        for _ in range(2):
            s = cap if variant == "same_stream" else torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                body()
            torch.cuda.current_stream().wait_stream(s)
            out.clear()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    cap.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cap):
        with torch.cuda.graph(g, stream=cap):
            body()
    torch.cuda.current_stream().wait_stream(cap)
    g.replay()
    torch.cuda.synchronize()
    ref = out["gb"].clone()
    eager = None
    res = []
    for _ in range(6):
        if variant == "big_churn":
            churn(BIG)
        elif variant != "no_churn":
            churn([4 * n for n in SMALL])
        g.replay()
        torch.cuda.synchronize()
        gb = out["gb"]
        d = (gb - ref).abs()
        res.append((bool(torch.equal(gb, ref)), int((~torch.isfinite(gb)).sum()),
                    float(d[torch.isfinite(d)].max()) if torch.isfinite(d).any() else float("nan")))
    with torch.no_grad():
        eager = (2 * 256.0 / (rows * dout)) * b.half().float() * rows
    print(f"{variant:14s} first replay vs closed form max|diff| {float((ref - eager).abs().max()):.3e}; "
          f"churned replays (equal, nonfinite, max|diff|): {res}", flush=True)


for v in ["backward", "autograd.grad", "grad_inplace", "no_churn", "big_churn", "no_warmup", "same_stream"]:
    run(v)
