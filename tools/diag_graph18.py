"""Which form of a Linear's captured backward reads memory the graph does not own (diag_graph16: an
nn.Linear(512, 1536) under fp16 autocast; diag_graph17: plain reductions are fine)?  Each case:
warm-ups (freed), capture fwd+bwd, then [small NaN churn, replay] x 6; prints whether the bias
gradient (and the weight gradient) equal the first replay's."""
import torch
import torch.nn.functional as F

SMALL = [1 << (k % 17) for k in range(2000)]


def churn():
    ts = [torch.full((n,), float("nan"), device="cuda") for n in SMALL]
    torch.cuda.synchronize()
    del ts


def case(name, fwd, rows=1088, din=512, dout=1536):
    torch.manual_seed(0)
    w = torch.nn.Parameter(torch.randn(dout, din, device="cuda") * 0.05)
    b = torch.nn.Parameter(torch.randn(dout, device="cuda") * 0.05)
    x = torch.randn(rows, din, device="cuda")

    def body():
        w.grad = b.grad = None
        loss = fwd(x, w, b).float().pow(2).mean()
        (loss * 256.0).backward()
    for _ in range(2):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            body()
        torch.cuda.current_stream().wait_stream(s)
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
    rb, rw = b.grad.clone(), w.grad.clone()
    res = []
    for _ in range(6):
        churn()
        g.replay()
        torch.cuda.synchronize()
        res.append((bool(torch.equal(b.grad, rb)), bool(torch.equal(w.grad, rw))))
    print(f"{name:44s} (bias, weight) grads == first replay: {res}", flush=True)


def ac(fn):
    def run(x, w, b):
        with torch.autocast(device_type="cuda", cache_enabled=False):
            return fn(x, w, b)
    return run



def case_leaf16(name, fwd):
    """the bias as an fp16 LEAF (no fp32 -> fp16 cast in the graph)"""
    torch.manual_seed(0)
    w = torch.nn.Parameter(torch.randn(1536, 512, device="cuda").half() * 0.05)
    b = torch.nn.Parameter(torch.randn(1536, device="cuda").half() * 0.05)
    x = torch.randn(1088, 512, device="cuda").half()
    _run(name, w, b, lambda: fwd(x, w, b))


def _run(name, w, b, f):
    def body():
        w.grad = b.grad = None
        (f().float().pow(2).mean() * 256.0).backward()
    for _ in range(2):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            body()
        torch.cuda.current_stream().wait_stream(s)
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
    rb, rw = b.grad.clone(), w.grad.clone()
    res = []
    for _ in range(6):
        churn()
        g.replay()
        torch.cuda.synchronize()
        res.append((bool(torch.equal(b.grad, rb)), bool(torch.equal(w.grad, rw))))
    print(f"{name:44s} (bias, weight) grads == first replay: {res}", flush=True)



class Cast16(torch.autograd.Function):
    """b.half() with its backward as an explicit grad.float() (no ToCopyBackward0 node)"""
    @staticmethod
    def forward(ctx, t):
        return t.half()

    @staticmethod
    def backward(ctx, g):
        return g.float()


class Cast16Copy(torch.autograd.Function):
    """the same, backward into a preallocated-by-empty fp32 tensor with copy_"""
    @staticmethod
    def forward(ctx, t):
        return t.half()

    @staticmethod
    def backward(ctx, g):
        out = torch.empty(g.shape, dtype=torch.float32, device=g.device)
        out.copy_(g)
        return out


case("Cast16 Function: mm + cast(b)", lambda x, w, b: x.half() @ w.half().t() + Cast16.apply(b))
case("Cast16Copy Function: mm + cast(b)", lambda x, w, b: x.half() @ w.half().t() + Cast16Copy.apply(b))
case("b16 = b.half() (ToCopyBackward0)", lambda x, w, b: x.half() @ w.half().t() + b.half())
case_leaf16("fp16 leaves: linear(x16, w16, b16)", lambda x, w, b: F.linear(x, w, b))
case_leaf16("fp16 leaves: mm + b16", lambda x, w, b: x @ w.t() + b)
case_leaf16("fp16 leaves: b16 expand only", lambda x, w, b: (x @ w.t()) * 0 + b.expand(1088, -1))
case("fp32 b -> fp16 cast -> .float() sum", lambda x, w, b: (x.half() @ w.half().t()).float() * 0 + b.half().float())
case("F.linear fp32", lambda x, w, b: F.linear(x, w, b))
case("F.linear autocast", ac(lambda x, w, b: F.linear(x, w, b)))
case("autocast matmul + bias add", ac(lambda x, w, b: x @ w.t() + b))
case("fp16 by hand: linear(x16, w16, b16)", lambda x, w, b: F.linear(x.half(), w.half(), b.half()))
case("fp16 by hand: addmm(b16, x16, w16^T)", lambda x, w, b: torch.addmm(b.half(), x.half(), w.half().t()))
case("fp16 by hand: mm + b16", lambda x, w, b: x.half() @ w.half().t() + b.half())
case("fp32 param -> fp16 cast only", lambda x, w, b: (x.half() @ w.half().t()) * 0 + b.half().expand(1088, -1))
case("F.linear autocast 3-D input [64,17,512]", ac(lambda x, w, b: F.linear(x.view(64, 17, 512), w, b)))
