"""Is the captured update's fused Adam the part another process-local optimizer step breaks, and
does pinned-host-memory churn between replays (what load() does) break it too?"""
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, "primal-ppo_amd")
from test_gpu_update_graph import _batch  # noqa: E402
from mapf_amd.model import Model  # noqa: E402

torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False


def fresh(graph, fused=True):
    torch.manual_seed(0)
    m = Model(0, "cuda", global_model=True, numChannel=6, num_agents=8, fov=9)
    if not fused:
        m.net_optimizer = torch.optim.Adam(m.network.parameters(), lr=m.net_optimizer.param_groups[0]["lr"],
                                           foreach=True, capturable=True)
    m.graph_update = graph
    m.network.eval()
    m.net_scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 8)
    return m


g = torch.Generator(device="cuda").manual_seed(1)
batches = [_batch(g) for _ in range(12)]


def full(m, b):
    obs, vec, ret, cret, v, cv, act, ps, tv = b
    m.train(obs, vec, ret, cret, v, cv, act, ps, None, tv, 1.0)


def pinned_churn(m, b):
    for n in (8, 64, 512, 4096, 1 << 14, 1 << 16):
        h = torch.full((n,), 1e30).pin_memory()
        torch.empty(n, device="cuda").copy_(h, non_blocking=True)
    torch.cuda.synchronize()


def twin_adam_only(m, b):
    for p in m.network.parameters():
        p.grad = torch.randn_like(p) * 1e-3
    m.net_optimizer.step()
    m.net_optimizer.zero_grad(set_to_none=True)


for name, fused, fn in (("fused Adam, pinned churn", True, pinned_churn),
                        ("fused Adam, twin's fused Adam step only", True, twin_adam_only),
                        ("fused Adam, eager twin updates", True, full)):
    m1 = fresh(True, fused)
    m2 = fresh(False)
    first = None
    for k, b in enumerate(batches):
        obs, vec, ret, cret, v, cv, act, ps, tv = b
        s1 = m1.train(obs, vec, ret, cret, v, cv, act, ps, None, tv, 1.0)
        if first is None and not torch.isfinite(torch.tensor(float(s1[8]))):
            first = k
        fn(m2, b)
    print(f"{name:45s} first non-finite replay: {first}", flush=True)
