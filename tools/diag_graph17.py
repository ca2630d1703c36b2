"""Captured torch reductions vs small-pool churn (diag_graph16: a plain nn.Linear's captured backward
gives a different bias gradient on replays after small NaN tensors were allocated and freed -- the
bias gradient is a sum over rows).  Each case captures one reduction (after two eager warm-ups on a
side stream whose outputs are freed), replays it once, then [churn, replay] x 6 and prints whether
the output still equals the first replay's."""
import torch

SMALL = [1 << (k % 17) for k in range(2000)]


def churn():
    ts = [torch.full((n,), float("nan"), device="cuda") for n in SMALL]
    torch.cuda.synchronize()
    del ts


def case(name, make, fn):
    torch.manual_seed(0)
    x = make()
    out = {}

    def body():
        out["y"] = fn(x)
    for _ in range(2):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            body()
        torch.cuda.current_stream().wait_stream(s)
        out.clear()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            body()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    ref = out["y"].clone()
    res = []
    for _ in range(6):
        churn()
        g.replay()
        torch.cuda.synchronize()
        res.append(bool(torch.equal(out["y"], ref)))
    print(f"{name:34s} replay == first replay after churn: {res}", flush=True)


a16 = torch.randn(1088, 1536, device="cuda").half()
v16 = torch.randn(1536, device="cuda").half()
case("static v16.float() [1536]", lambda: v16, lambda x: x.float())
case("a16.sum(0).float()", lambda: a16, lambda x: x.sum(0).float())
case("a16.sum(0, fp32)", lambda: a16, lambda x: x.sum(0, dtype=torch.float32))
case("(a16 * 2).sum(0).float()", lambda: a16, lambda x: (x * 2).sum(0).float())
case("a16.sum(0) -> empty fp32 .copy_", lambda: a16, lambda x: torch.empty(1536, device="cuda").copy_(x.sum(0)))
case("a16.float().sum(0)", lambda: a16, lambda x: x.float().sum(0))
