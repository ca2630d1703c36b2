"""Minimal reproducer hunt for the captured-backward hazard (diag_graph14/15: bias gradients of the
captured backward go non-finite after small-pool churn once the eager warm-ups' tensors are freed).
Each case: two eager warm-ups on a side stream (their tensors freed), capture fwd + backward on a side
stream, then [churn small NaN tensors, replay] x 10; prints the replay's non-finite parameter grads.
  linear    nn.Linear(512, 1536) on [1088, 512] fp16 under autocast
  conv      nn.Conv2d(128, 128, 3, padding 1) channels_last on [512, 128, 9, 9]
  net_sum   SCRIMPNet training forward, loss = sum of its outputs (no fused loss / normalisation)
  net_hipatt_off  the same with the training attention on SDPA instead of _HipAttention"""
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, "primal-ppo_amd")
from mapf_amd.net import SCRIMPNet, _SelfAttention  # noqa: E402

SMALL = [1 << (k % 17) for k in range(2000)]
torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False


def churn():
    ts = [torch.full((n,), float("nan"), device="cuda") for n in SMALL]
    torch.cuda.synchronize()
    del ts


def case(name):
    torch.manual_seed(0)
    if name == "linear":
        mod = torch.nn.Linear(512, 1536).cuda()
        x = torch.randn(1088, 512, device="cuda")
        fwd = lambda: mod(x).float().pow(2).mean()  # noqa: E731
    elif name == "conv":
        mod = torch.nn.Conv2d(128, 128, 3, padding=1).cuda().to(memory_format=torch.channels_last)
        x = torch.randn(512, 128, 9, 9, device="cuda").contiguous(memory_format=torch.channels_last)
        fwd = lambda: mod(x).float().pow(2).mean()  # noqa: E731
    else:
        _SelfAttention.hip_attention = name != "net_hipatt_off"
        mod = SCRIMPNet(numChannel=6, num_agents=8, fov=9).cuda().to(memory_format=torch.channels_last).eval()
        obs = (torch.rand(64, 8, 6, 9, 9, device="cuda") < 0.3).float()
        vec = torch.randn(64, 8, 4, device="cuda")

        def fwd():
            out = mod(obs, vec)
            return sum(o.float().sum() for o in (out[0], out[1], out[3], out[6]))
    params = list(mod.parameters())
    names = [n for n, _ in mod.named_parameters()]

    def body():
        for p in params:
            p.grad = None
        with torch.autocast(device_type="cuda", cache_enabled=False):
            loss = fwd()
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
    keep = [i for i, p in enumerate(params) if p.grad is not None]
    params, names = [params[i] for i in keep], [names[i] for i in keep]
    ref = [p.grad.clone() for p in params]
    res = []
    bad_names = set()
    for _ in range(10):
        churn()
        g.replay()
        torch.cuda.synchronize()
        bad = [n for n, p, r in zip(names, params, ref) if not torch.equal(p.grad, r)]
        res.append(len(bad))
        bad_names.update(bad)
    print(f"{name:15s} grads differing from the first replay, per churned replay {res} {sorted(bad_names)[:6]}",
          flush=True)


if __name__ == "__main__":
    for name in sys.argv[1:] or ["linear", "conv", "net_sum", "net_hipatt_off"]:
        case(name)
