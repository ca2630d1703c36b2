"""The captured-update replay hazard: WHEN does the graphed model's computation diverge?  Two runs of
the same m1 (same weights, same batches): one alone, one with an eager twin updating before m1's
updates 3..9.  Prints m1's 11 update stats side by side per update (bitwise equal or not) and the
max |difference| of m1's parameters after each update."""
import sys

import numpy as np
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
    return np.array([float(np.asarray(x)) for x in m.train(obs, vec, ret, cret, v, cv, act, ps, None, tv, 1.0)])


def run(with_twin):
    g = torch.Generator(device="cuda").manual_seed(1)
    batches = [_batch(g) for _ in range(10)]
    m1 = fresh()
    twin = fresh(False) if with_twin else None
    stats, params = [], []
    for k, b in enumerate(batches):
        if twin is not None and k >= 3:
            train(twin, b)
            torch.cuda.synchronize()
        stats.append(train(m1, b))
        params.append(torch.cat([p.detach().flatten() for p in m1.network.parameters()]).cpu().numpy())
    return stats, params


if __name__ == "__main__":
    s0, p0 = run(False)
    s1, p1 = run(True)
    np.set_printoptions(precision=6, linewidth=200)
    for k in range(len(s0)):
        same = np.array_equal(s0[k], s1[k])
        dp = np.nanmax(np.abs(p0[k] - p1[k]))
        print(f"update {k}: stats equal {same}; params max |diff| {dp:.3e}\n   alone {s0[k][[0, 1, 3, 8]]}\n   twin  "
              f"{s1[k][[0, 1, 3, 8]]}", flush=True)
