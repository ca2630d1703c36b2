"""The captured-update replay hazard: what does a second model's eager update
change that a later replay of the first model's graph reads?

For each variant: a graphed model m1 and an eager twin m2 (fresh, same weights).  m1 runs its two
eager warm-ups and its capture + first replay; then
  1. snapshot every tensor m1's update owns (parameters, .grad, Adam state, the update's static
     buffers, AMP scale / growth / found-inf),
  2. m2 runs one full eager update,
  3. diff m1's tensors against the snapshot (bitwise) -- which of them did m2's update write?
  4. replay m1 once more; report whether its stats are finite and which gradients are not.
Variants change one thing at a time: BLAS library, MIOpen on/off, where m2's update runs."""
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, "primal-ppo_amd")
from test_gpu_update_graph import _batch  # noqa: E402
from mapf_amd.model import Model  # noqa: E402

torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False


def fresh(graph):
    torch.manual_seed(0)
    m = Model(0, "cuda", global_model=True, numChannel=6, num_agents=8, fov=9)
    m.graph_update = graph
    m.network.eval()
    m.net_scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 8)
    return m


def owned(m):
    out = {}
    for n, p in m.network.named_parameters():
        out["param " + n] = p
        if p.grad is not None:
            out["grad " + n] = p.grad
        for k, v in m.net_optimizer.state.get(p, {}).items():
            if torch.is_tensor(v):
                out[f"adam {k} {n}"] = v
    for key, u in m._updates.items():
        for k in ("obs", "vec", "ret", "cret", "v", "cv", "action", "old_ps", "tv", "dyn", "scale", "growth",
                  "found_inf", "stats"):
            out[f"upd {k}"] = getattr(u, k)
    return out


def train(m, b):
    obs, vec, ret, cret, v, cv, act, ps, tv = b
    return m.train(obs, vec, ret, cret, v, cv, act, ps, None, tv, 1.0)


def run(name, setup=None, twin_stream=False):
    if setup:
        setup()
    g = torch.Generator(device="cuda").manual_seed(1)
    batches = [_batch(g) for _ in range(8)]
    m1, m2 = fresh(True), fresh(False)
    for k in range(3):
        train(m1, batches[k])          # warm-up x2, capture + replay
    torch.cuda.synchronize()
    upd = next(iter(m1._updates.values()))
    assert upd.graph is not None
    first_bad = None
    changed_all = set()
    for k in range(3, 8):
        snap = {n: t.detach().clone() for n, t in owned(m1).items()}
        torch.cuda.synchronize()
        if twin_stream:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                train(m2, batches[k])
            torch.cuda.current_stream().wait_stream(s)
        else:
            train(m2, batches[k])
        torch.cuda.synchronize()
        now = owned(m1)
        changed = [n for n, t in snap.items() if not torch.equal(t, now[n].detach())]
        changed_all.update(changed)
        s1 = train(m1, batches[k])
        torch.cuda.synchronize()
        finite = all(torch.isfinite(torch.tensor(float(x))) for x in s1[:9])
        bad_grads = [n for n, p in m1.network.named_parameters() if p.grad is not None and
                     not torch.isfinite(p.grad).all()]
        if not finite and first_bad is None:
            first_bad = k
        print(f"  [{name}] update {k}: twin changed {len(changed)} of m1's tensors {changed[:6]}; "
              f"replay finite {finite}; non-finite grads {len(bad_grads)} {bad_grads[:4]}; "
              f"scale {float(upd.scale):.1f}", flush=True)
    print(f"{name:40s} first non-finite replay: {first_bad}; twin wrote {sorted(changed_all)[:10]}", flush=True)


def blas(lib):
    return lambda: torch.backends.cuda.preferred_blas_library(lib)


if __name__ == "__main__":
    which = sys.argv[1:] or ["base", "twin_stream", "rocblas", "nomiopen"]
    print("preferred BLAS:", torch.backends.cuda.preferred_blas_library(), flush=True)
    for w in which:
        if w == "base":
            run("base")
        elif w == "twin_stream":
            run("twin on its own stream", twin_stream=True)
        elif w == "rocblas":
            run("rocBLAS (preferred_blas_library cublas)", setup=blas("cublas"))
        elif w == "nomiopen":
            torch.backends.cudnn.enabled = False
            run("MIOpen disabled")
            torch.backends.cudnn.enabled = True
