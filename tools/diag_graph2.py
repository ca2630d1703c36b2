"""Which of the captured update's persistent tensors changes while ANOTHER model's eager update runs
between two replays: checksums of params, grads, Adam state and AMP state of the graphed model
before and after the other model's update (they must not move)."""
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


def sums(m):
    out = {}
    for i, p in enumerate(m.network.parameters()):
        out[f"p{i}"] = p.detach().double().sum().item()
        if p.grad is not None:
            out[f"g{i}"] = p.grad.detach().double().sum().item()
            out[f"g{i}@"] = p.grad.data_ptr()
        st = m.net_optimizer.state.get(p, {})
        for k in ("exp_avg", "exp_avg_sq", "step"):
            if k in st:
                out[f"{k}{i}"] = st[k].detach().double().sum().item()
    for u in m._updates.values():
        for k in ("scale", "growth", "found_inf", "dyn", "obs", "stats"):
            out[f"u.{k}"] = getattr(u, k).detach().double().sum().item()
    return out


g = torch.Generator(device="cuda").manual_seed(1)
batches = [_batch(g) for _ in range(7)]
m1, m2 = fresh(True), fresh(False)
for k in range(7):
    obs, vec, ret, cret, v, cv, act, ps, tv = batches[k]
    s1 = m1.train(obs, vec, ret, cret, v, cv, act, ps, None, tv, 1.0)
    torch.cuda.synchronize()
    before = sums(m1)
    s2 = m2.train(obs, vec, ret, cret, v, cv, act, ps, None, tv, 1.0)
    torch.cuda.synchronize()
    after = sums(m1)
    moved = [key for key in before if before[key] != after.get(key)]
    print(k, "graph gnorm", float(s1[8]), "eager gnorm", float(s2[8]), "m1 tensors changed by m2's update:", moved[:12],
          len(moved), flush=True)
    ptrs1 = {v for key, v in before.items() if key.endswith("@")}
    ptrs2 = {p.grad.data_ptr() for p in m2.network.parameters() if p.grad is not None}
    print("   m1 grad buffers also used by m2:", len(ptrs1 & ptrs2), flush=True)
