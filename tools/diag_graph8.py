"""The captured-update replay hazard, bisected further (diag_graph7: only a second model's FULL eager
update breaks the first model's replays -- its forward + backward alone do not).  Hypothesis: a
multi-tensor (foreach / fused-optimizer) kernel captured in the graph takes its tensor-list
metadata from memory that a later eager multi-tensor call over OTHER tensors overwrites, so the
replay then works on the other call's tensors.  Test: capture one op over list A, replay, run the
same op eagerly over list B, replay again; check which list the second replay changed."""
import torch


def lists(n, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return [torch.rand(257 + 13 * i, device="cuda", generator=g) + 0.5 for i in range(n)]


def op_mul(ts, _):
    torch._foreach_mul_(ts, 2.0)


def op_norm(ts, out):
    out.copy_(torch.stack(torch._foreach_norm(ts)).sum())


def op_unscale(ts, out):
    torch._amp_foreach_non_finite_check_and_unscale_(ts, out, torch.full((), 0.5, device="cuda"))


def make_adam(ts):
    ps = [torch.nn.Parameter(t) for t in ts]
    for p in ps:
        p.grad = torch.ones_like(p)
    return ps, torch.optim.Adam(ps, lr=0.1, fused=True, capturable=True)


for n in (8, 56, 200):
    for name, op in (("foreach_mul", op_mul), ("foreach_norm", op_norm), ("amp_unscale", op_unscale),
                     ("fused_adam", None)):
        A, B = lists(n, 1), lists(n, 2)
        outA, outB = torch.zeros((), device="cuda"), torch.zeros((), device="cuda")
        if op is None:
            pa, oa = make_adam(A)
            pb, ob = make_adam(B)
            run_a, run_b = oa.step, ob.step
            watch_a, watch_b = pa, pb
        else:
            run_a, run_b = (lambda: op(A, outA)), (lambda: op(B, outB))
            watch_a, watch_b = A, B
        if name == "foreach_norm":               # the output is what the replay writes
            watch_a, watch_b = [outA], [outB]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            run_a()                                   # warm-up
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            run_a()
        g.replay()
        torch.cuda.synchronize()
        a0 = [t.detach().clone() for t in watch_a]
        run_b()                                       # eager over B
        torch.cuda.synchronize()
        b0 = [t.detach().clone() for t in watch_b]
        g.replay()
        torch.cuda.synchronize()
        a_changed = sum(not torch.equal(x, y.detach()) for x, y in zip(a0, watch_a))
        if name == "foreach_norm":               # a norm replay must reproduce its value
            a_changed = 1 - a_changed
        b_changed = sum(not torch.equal(x, y.detach()) for x, y in zip(b0, watch_b))
        print(f"n={n:3d} {name:12s} replay after an eager call over B changed {a_changed}/{n} of A "
              f"and {b_changed}/{n} of B  ({'HAZARD' if b_changed else 'ok'})", flush=True)
