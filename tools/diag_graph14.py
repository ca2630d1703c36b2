"""The captured-update replay hazard: which captured piece reads memory it does not own?  Small-pool
churn (NaN-filled tensors of 4 B .. 512 KiB allocated and freed between replays) turns the captured
update non-finite deterministically (diag_graph13).  Here the update body is captured only up to a
given piece; after each churn the replay's own outputs up to that piece are checked for NaN:
  norm      advantage normalisation (mapf_normalize_advantages_dlam)       -> adv, cadv
  fwd       + the training forward under autocast                           -> ps, v, sig, cv
  loss      + the fused PPO loss (mapf_ppo_loss_dcoef)                      -> loss
  bwd       + (loss * scale).backward()                                     -> every .grad
  clip      + unscale / found-inf + clip_grad_norm_                         -> grad norm
  adam      + fused Adam (found-inf skip)                                   -> every parameter"""
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, "primal-ppo_amd")
from test_gpu_update_graph import _batch  # noqa: E402
from mapf_amd.model import Model, _DeviceUpdate, _FusedPPOLoss  # noqa: E402
from mapf_amd.config import TrainingParameters as T  # noqa: E402
from mapf_amd.env import normalize_advantages_dlam  # noqa: E402

torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
SMALL = [1 << (k % 17) for k in range(2000)]


def churn():
    ts = [torch.full((n,), float("nan"), device="cuda") for n in SMALL]
    torch.cuda.synchronize()
    del ts


def body(m, u, stop, out):
    net, opt = m.network, m.net_optimizer
    opt.zero_grad(set_to_none=True)
    adv, cadv = normalize_advantages_dlam(u.ret.reshape(-1), u.v.reshape(-1), u.cret.reshape(-1), u.cv.reshape(-1),
                                          u.dyn[6:8], T.MINUS_ADV_WITH_CADV)
    out["norm"] = [adv, cadv]
    if stop == "norm":
        return
    adv, cadv = adv.view(u.ret.shape), cadv.view(u.ret.shape)
    with torch.autocast(device_type="cuda", cache_enabled=False):
        new_ps, new_v, block, policy_sig, _, _, new_cv = net(u.obs, u.vec, None)
    out["fwd"] = [new_ps, new_v, policy_sig, new_cv]
    if stop == "fwd":
        return
    all_loss, terms = _FusedPPOLoss.apply(new_ps, new_v, new_cv, policy_sig, u.old_ps, u.action.unsqueeze(-1),
                                          u.v, u.ret, u.cv, u.cret, adv, cadv, u.tv, u.dyn[:6])
    out["loss"] = [all_loss, terms]
    if stop == "loss":
        return
    (all_loss * u.scale).backward()
    params = [p for p in net.parameters() if p.grad is not None]
    out["bwd"] = [p.grad for p in params]
    out["bwd_names"] = [n for n, p in net.named_parameters() if p.grad is not None]
    if stop == "bwd":
        return
    u.found_inf.zero_()
    torch._amp_foreach_non_finite_check_and_unscale_([p.grad for p in params], u.found_inf,
                                                     u.scale.double().reciprocal().float())
    gn = torch.nn.utils.clip_grad_norm_(params, T.MAX_GRAD_NORM)
    out["clip"] = [gn, u.found_inf]
    if stop == "clip":
        return
    opt.grad_scale, opt.found_inf = None, u.found_inf
    opt.step()
    opt.grad_scale = opt.found_inf = None
    out["adam"] = list(net.parameters())


def bad(ts):
    return sum(int(not torch.isfinite(t.detach().float()).all()) for t in ts)


def run(stop):
    g = torch.Generator(device="cuda").manual_seed(1)
    batches = [_batch(g) for _ in range(14)]
    torch.manual_seed(0)
    m = Model(0, "cuda", global_model=True, numChannel=6, num_agents=8, fov=9)
    m.network.eval()
    m.net_scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 8)
    sc = m.net_scaler
    sc._lazy_init_scale_growth_tracker(m.device)
    obs, vec, ret, cret, v, cv, act, ps, tv = batches[0]
    u = _DeviceUpdate(m, obs, vec, ret, ps, tv, act.unsqueeze(-1))
    coef = (T.CLIP_RANGE, T.ENTROPY_COEF, T.VALUE_COEF, T.VALID_COEF, T.COST_VALUE_COEF, T.COST_COEF)
    out = {}
    graph = None
    res, names = [], []
    for k, b in enumerate(batches):
        obs, vec, ret, cret, v, cv, act, ps, tv = b
        u.load(obs, vec, ret, cret, v, cv, act.unsqueeze(-1), ps, tv, coef=coef, lam=0.0)
        if k < 2:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                body(m, u, stop, out)
            torch.cuda.current_stream().wait_stream(s)
            if not KEEP_WARMUP:
                out.clear()               # the warm-up's tensors (and autograd graph) die here
            continue
        if graph is None:
            graph = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                with torch.cuda.graph(graph, stream=s):
                    body(m, u, stop, out)
            torch.cuda.current_stream().wait_stream(s)
        if k >= 3:
            churn()
        graph.replay()
        torch.cuda.synchronize()
        res.append(bad(out[stop]))
        if stop == "bwd" and res[-1] and not names:
            names = [n for n, t in zip(out["bwd_names"], out["bwd"]) if not torch.isfinite(t.float()).all()]
    print(f"captured up to {stop:5s}: non-finite outputs per replay {res} {names}", flush=True)


KEEP_WARMUP = True


def full_qkv_forward_first(self, x):
    """forward_first with ONE linear over the whole to_qkv parameter (no w[:d] / w[d:] views)."""
    from mapf_amd.net import _HipAttention
    import torch.nn.functional as F
    b, n, d = x.shape
    qkv = self.to_qkv(x)
    q = qkv[:, 0, :d].contiguous()
    kv = qkv[:, :, d:].contiguous()
    if self._hip(x, q):
        return self.do1(self.nn1(_HipAttention.apply(q, kv, 1, 0, 0, d, self.scale)))
    raise RuntimeError("HIP attention expected")


if __name__ == "__main__":
    if "fullqkv" in sys.argv:
        sys.argv.remove("fullqkv")
        from mapf_amd.net import _SelfAttention
        _SelfAttention.forward_first = full_qkv_forward_first
        print("last block: one to_qkv linear (no parameter views)", flush=True)
    for keep in (False,):
        KEEP_WARMUP = keep
        print(f"warm-up outputs {'kept alive' if keep else 'freed'}:", flush=True)
        for stop in sys.argv[1:] or ["norm", "fwd", "loss", "bwd", "clip", "adam"]:
            run(stop)
