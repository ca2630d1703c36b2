"""The captured-update replay hazard, pinned to the optimizer (diag_graph9: of a twin model's eager
update only its Adam step breaks the graphed model's later replays; diag_graph4: a twin's Adam step
on random gradients WITHOUT found_inf does not).  Variants (twin = eager model, m1 = graphed):
  rand_finf      twin: random grads, opt.found_inf = a zero tensor, fused Adam step
  rand_nofinf    twin: random grads, no found_inf, fused Adam step
  m1_foreach     m1's optimizer foreach + capturable (not fused); twin: full eager update
  twin_foreach   twin's optimizer foreach + capturable; twin: full eager update
  full           twin: full eager update (fused Adam both), the reference case
Each: 10 m1 updates, twin work before updates 3..9; m1's replay finiteness per update."""
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, "primal-ppo_amd")
from test_gpu_update_graph import _batch  # noqa: E402
from mapf_amd.model import Model  # noqa: E402

torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False


def fresh(graph=True, foreach=False):
    torch.manual_seed(0)
    m = Model(0, "cuda", global_model=True, numChannel=6, num_agents=8, fov=9)
    if foreach:
        m.net_optimizer = torch.optim.Adam(m.network.parameters(), lr=m.net_optimizer.param_groups[0]["lr"],
                                           foreach=True, capturable=True)
    m.graph_update = graph
    m.network.eval()
    m.net_scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 8)
    return m


def train(m, b):
    obs, vec, ret, cret, v, cv, act, ps, tv = b
    return m.train(obs, vec, ret, cret, v, cv, act, ps, None, tv, 1.0)


def finite(s):
    return all(torch.isfinite(torch.tensor(float(x))) for x in s[:9])


def rand_step(twin, finf):
    for p in twin.network.parameters():
        p.grad = torch.randn_like(p) * 1e-3
    opt = twin.net_optimizer
    opt.found_inf = torch.zeros((), device="cuda") if finf else None
    opt.step()
    opt.found_inf = None
    opt.zero_grad(set_to_none=True)


if __name__ == "__main__":
    kinds = sys.argv[1:] or ["rand_finf", "rand_nofinf", "m1_foreach", "twin_foreach", "full"]
    for kind in kinds:
        g = torch.Generator(device="cuda").manual_seed(1)
        batches = [_batch(g) for _ in range(10)]
        m1 = fresh(foreach=kind == "m1_foreach")
        twin = fresh(False, foreach=kind == "twin_foreach")
        res = []
        for k, b in enumerate(batches):
            if k >= 3:
                if kind == "rand_finf":
                    rand_step(twin, True)
                elif kind == "rand_nofinf":
                    rand_step(twin, False)
                else:
                    train(twin, b)
                torch.cuda.synchronize()
            res.append(finite(train(m1, b)))
        print(f"{kind:13s} m1 replay finite per update {res}", flush=True)
