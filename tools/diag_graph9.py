"""The captured-update replay hazard, bisected inside a twin's eager update (diag_graph7: only the
twin's FULL update breaks the graphed model's replays; diag_graph8: foreach / fused-Adam metadata is
not it).  The twin runs one piece of _DeviceUpdate.body at a time between m1's updates (8 updates,
pieces repeated), and each piece's first non-finite m1 replay is printed."""
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, "primal-ppo_amd")
from test_gpu_update_graph import _batch  # noqa: E402
from mapf_amd.model import Model, _DeviceUpdate, _FusedPPOLoss  # noqa: E402
from mapf_amd.config import TrainingParameters as T  # noqa: E402

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


def twin_upd(twin, b):
    obs, vec, ret, cret, v, cv, act, ps, tv = b
    sc = twin.net_scaler
    if sc._scale is None:
        sc._lazy_init_scale_growth_tracker(twin.device)
    u = getattr(twin, "_diag_upd", None)
    if u is None:
        u = twin._diag_upd = _DeviceUpdate(twin, obs, vec, ret, ps, tv, act.unsqueeze(-1))
    u.load(obs, vec, ret, cret, v, cv, act.unsqueeze(-1), ps, tv,
           coef=(T.CLIP_RANGE, T.ENTROPY_COEF, T.VALUE_COEF, T.VALID_COEF, T.COST_VALUE_COEF, T.COST_COEF), lam=0.0)
    return u


def piece(kind, twin, b):
    u = twin_upd(twin, b)
    net, opt = twin.network, twin.net_optimizer
    opt.zero_grad(set_to_none=True)
    from mapf_amd.env import normalize_advantages_dlam
    adv, cadv = normalize_advantages_dlam(u.ret.reshape(-1), u.v.reshape(-1), u.cret.reshape(-1), u.cv.reshape(-1),
                                          u.dyn[6:8], T.MINUS_ADV_WITH_CADV)
    if kind == "load_norm":
        return
    adv, cadv = adv.view(u.ret.shape), cadv.view(u.ret.shape)
    with torch.autocast(device_type="cuda", cache_enabled=False):
        new_ps, new_v, block, policy_sig, _, _, new_cv = net(u.obs, u.vec, None)
    all_loss, terms = _FusedPPOLoss.apply(new_ps, new_v, new_cv, policy_sig, u.old_ps, u.action.unsqueeze(-1),
                                          u.v, u.ret, u.cv, u.cret, adv, cadv, u.tv, u.dyn[:6])
    if kind == "fused_loss":
        return
    (all_loss * u.scale).backward()
    if kind == "loss_backward":
        return
    params = [p for p in net.parameters() if p.grad is not None]
    u.found_inf.zero_()
    torch._amp_foreach_non_finite_check_and_unscale_([p.grad for p in params], u.found_inf,
                                                     u.scale.double().reciprocal().float())
    torch.nn.utils.clip_grad_norm_(params, T.MAX_GRAD_NORM)
    if kind == "unscale_clip":
        return
    opt.grad_scale, opt.found_inf = None, u.found_inf
    opt.step()
    opt.grad_scale = opt.found_inf = None
    if kind == "adam":
        return
    torch._amp_update_scale_(u.scale, u.growth, u.found_inf, *u.amp)


if __name__ == "__main__":
    kinds = sys.argv[1:] or ["load_norm", "fused_loss", "loss_backward", "unscale_clip", "adam", "scale_update"]
    for kind in kinds:
        g = torch.Generator(device="cuda").manual_seed(1)
        batches = [_batch(g) for _ in range(10)]
        m1, twin = fresh(), fresh(False)
        res = []
        for k, b in enumerate(batches):
            if k >= 3:
                piece(kind, twin, b)
                torch.cuda.synchronize()
            res.append(finite(train(m1, b)))
        print(f"{kind:14s} m1 replay finite per update {res}", flush=True)
