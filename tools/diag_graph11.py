"""The captured-update replay hazard: does the graphed model m1 share memory with the eager twin?
After m1's capture, list the address ranges of every tensor each model owns (parameters, .grad,
Adam state, the update's static buffers) and report overlaps after each twin update; then scale the
twin's parameters in place (no optimizer) and see whether m1's next replay notices."""
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, "primal-ppo_amd")
from test_gpu_update_graph import _batch  # noqa: E402
from mapf_amd.model import Model  # noqa: E402

torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False


def fresh(graph=True):
    torch.manual_seed(0)
    m = Model(0, "cuda", global_model=True, numChannel=6, num_agents=8, fov=9)
    m.graph_update = graph
    m.network.eval()
    m.net_scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 8)
    return m


def train(m, b):
    obs, vec, ret, cret, v, cv, act, ps, tv = b
    return m.train(obs, vec, ret, cret, v, cv, act, ps, None, tv, 1.0)


def finite(s):
    return all(torch.isfinite(torch.tensor(float(x))) for x in s[:9])


def ranges(m):
    out = {}
    for n, p in m.network.named_parameters():
        out["param " + n] = p
        if p.grad is not None:
            out["grad " + n] = p.grad
        for k, v in m.net_optimizer.state.get(p, {}).items():
            if torch.is_tensor(v) and v.is_cuda:
                out[f"adam.{k} {n}"] = v
    for u in m._updates.values():
        for k in ("obs", "vec", "ret", "cret", "v", "cv", "action", "old_ps", "tv", "dyn", "scale", "growth",
                  "found_inf", "stats"):
            out["upd " + k] = getattr(u, k)
    return {k: (t.data_ptr(), t.data_ptr() + t.untyped_storage().nbytes()) for k, t in out.items()}


def overlaps(a, b):
    hits = []
    for ka, (a0, a1) in a.items():
        for kb, (b0, b1) in b.items():
            if a0 < b1 and b0 < a1:
                hits.append((ka, kb))
    return hits


if __name__ == "__main__":
    g = torch.Generator(device="cuda").manual_seed(1)
    batches = [_batch(g) for _ in range(10)]
    m1, twin = fresh(), fresh(False)
    for k, b in enumerate(batches):
        if k >= 3:
            train(twin, b)
            torch.cuda.synchronize()
            hits = overlaps(ranges(m1), ranges(twin))
            print(f"after twin update {k}: {len(hits)} overlapping (m1, twin) tensor pairs {hits[:8]}", flush=True)
        ok = finite(train(m1, b))
        print(f"m1 update {k}: replay finite {ok}", flush=True)
    # the twin's parameters scaled in place: does m1's replay read them?
    with torch.no_grad():
        for p in twin.network.parameters():
            p.mul_(1000.0)
    torch.cuda.synchronize()
    print("after scaling the twin's parameters x1000: m1 replay finite", finite(train(m1, batches[0])), flush=True)
