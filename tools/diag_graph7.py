"""The captured-update replay hazard, bisected by the work run between replays (diag_graph5/6: the
second model's eager update changes none of the graphed model's tensors, and NaN-filled allocation
churn between replays does NOT break them -- so it is not a dangling allocator block).  Each
variant: a fresh graphed model m1 (two eager warm-ups, capture + replay), then before each of its
next updates ONE kind of work on the default stream:
  none        nothing
  matmul      fp16 GEMMs of the update's shapes (hipBLASLt on the default stream)
  conv        fp16 channels-last convolutions, forward + backward (MIOpen)
  twin_fwd    a twin model's training forward under autocast (grad enabled), no backward
  twin_bwd    ... + backward
  twin_full   a twin's whole eager update
  m1_fwd      m1's OWN training forward (grad enabled) + backward, no optimizer step
Prints each replay's finiteness."""
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


def fwd_bwd(m, b, backward=True):
    with torch.autocast(device_type="cuda"):
        out = m.network(b[0], b[1])
    if backward:
        (out[1].float().sum() + out[0].float().pow(2).sum()).backward()
    m.net_optimizer.zero_grad(set_to_none=True)


def work(kind, twin, m1, b):
    if kind == "matmul":
        for n in (512, 1536, 1024):
            a = torch.randn(512 * 17, 512, device="cuda").half()
            w = torch.randn(n, 512, device="cuda").half()
            torch.nn.functional.linear(a, w, torch.randn(n, device="cuda").half()).float().sum().item()
    elif kind == "conv":
        x = torch.randn(512, 128, 9, 9, device="cuda").half().contiguous(memory_format=torch.channels_last)
        x.requires_grad_(True)
        w = torch.randn(128, 128, 3, 3, device="cuda").half().requires_grad_(True)
        torch.nn.functional.conv2d(x, w, None, 1, 1).float().sum().backward()
    elif kind == "twin_fwd":
        fwd_bwd(twin, b, backward=False)
    elif kind == "twin_bwd":
        fwd_bwd(twin, b)
    elif kind == "twin_full":
        train(twin, b)
    elif kind == "m1_fwd":
        fwd_bwd(m1, b)
    torch.cuda.synchronize()


if __name__ == "__main__":
    kinds = sys.argv[1:] or ["none", "matmul", "conv", "twin_fwd", "twin_bwd", "twin_full", "m1_fwd"]
    for kind in kinds:
        g = torch.Generator(device="cuda").manual_seed(1)
        batches = [_batch(g) for _ in range(7)]
        m1 = fresh()
        twin = fresh(False) if kind.startswith("twin") else None
        res = []
        for k, b in enumerate(batches):
            if k >= 3:
                work(kind, twin, m1, b)
            res.append(finite(train(m1, b)))
        print(f"{kind:10s} replay finite per update {res}  scale {float(m1.net_scaler._scale):.0f}", flush=True)
