"""GPU tests of the fused PPO loss (csrc/mapf_ppo.hip): its value and
gradient against autograd through the reference's own expression (model.py:115-175,
restated in torch below), ties and clamp boundaries included, and a whole Model.train
update fused vs unfused from the same state."""
import copy

import numpy as np

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")


C = (0.2, 0.01, 0.08, 0.5, 0.3, 0.7)   # clip, entropy, value, valid, cost value, cost * lambda


def torch_loss(new_ps, new_v, new_cv, sig, old_ps, action, old_v, ret, old_cv, cret, adv, cadv, tv):
    clip, ent_c, vc, valid_c, cvc, costlam = C
    new_p, old_p = new_ps.gather(-1, action[..., None]), old_ps.gather(-1, action[..., None])
    ratio = torch.exp(torch.log(torch.clamp(new_p, 1e-6, 1.0)) - torch.log(torch.clamp(old_p, 1e-6, 1.0)))
    entropy = torch.mean(-torch.sum(new_ps * torch.log(torch.clamp(new_ps, 1e-6, 1.0)), dim=-1, keepdim=True))
    v, cv = new_v.squeeze(-1), new_cv.squeeze(-1)
    v_clip = old_v + torch.clamp(v - old_v, -clip, clip)
    critic = torch.mean(torch.maximum(torch.square(v - ret), torch.square(v_clip - ret)))
    cv_clip = old_cv + torch.clamp(cv - old_cv, -clip, clip)
    ccritic = torch.mean(torch.maximum(torch.square(cv - cret), torch.square(cv_clip - cret)))
    ratio = ratio.squeeze(-1)
    policy = torch.mean(torch.min(adv * ratio, adv * torch.clamp(ratio, 1.0 - clip, 1.0 + clip)))
    valid = -torch.mean(torch.log(torch.clamp(sig, 1e-6, 1.0 - 1e-6)) * tv +
                        torch.log(torch.clamp(1 - sig, 1e-6, 1.0 - 1e-6)) * (1 - tv))
    cost = torch.mean(ratio * cadv)
    all_loss = -policy - entropy * ent_c + vc * critic + valid_c * valid + cvc * ccritic + costlam * cost
    clip_frac = torch.mean(torch.greater(torch.abs(ratio - 1.0), clip).float())
    return all_loss, torch.stack([policy, entropy, critic, valid, ccritic, cost, clip_frac])


def _inputs(rows, n, seed, sig_dtype):
    g = torch.Generator(device="cuda").manual_seed(seed)
    r = lambda *s: torch.randn(*s, device="cuda", generator=g)
    new_ps = torch.softmax(r(rows, n, 5) * 2, -1)
    old_ps = torch.softmax(r(rows, n, 5) * 2, -1)
    old_ps[: rows // 4] = new_ps[: rows // 4]                     # ratio == 1: min() ties
    new_ps[0, 0] = torch.tensor([1.0, 0, 0, 0, 0])               # clamp boundaries / zeros
    action = torch.randint(0, 5, (rows, n), device="cuda", generator=g)
    new_v, old_v, ret = r(rows, n, 1), r(rows, n), r(rows, n)
    old_v[: rows // 4] = new_v[: rows // 4, :, 0]                 # max() ties
    new_cv, old_cv, cret = r(rows, n, 1), r(rows, n), r(rows, n)
    sig = torch.sigmoid(r(rows, n, 5) * 4).to(sig_dtype)
    sig[1, 1] = torch.tensor([0.0, 1.0, 0.5, 1e-7, 1 - 1e-7])
    tv = (r(rows, n, 5) > 0).float()
    return new_ps, new_v, new_cv, sig, old_ps, action, old_v, ret, old_cv, cret, r(rows, n), r(rows, n), tv


@pytest.mark.parametrize("rows,sig_dtype", [(256, torch.float32), (256, torch.float16), (3, torch.float32),
                                            (1500, torch.float16)])
def test_fused_loss_and_gradient_vs_autograd(rows, sig_dtype):
    from mapf_amd.model import _FusedPPOLoss
    x = _inputs(rows, 8, rows, sig_dtype)
    a = [t.clone().requires_grad_(True) if i < 4 else t for i, t in enumerate(x)]
    b = [t.clone().requires_grad_(True) if i < 4 else t for i, t in enumerate(x)]
    with torch.autocast(device_type="cuda"):   # as in Model.train: log/exp autocast to fp32
        ref_loss, ref_terms = torch_loss(*a)
    ref_loss.backward()
    loss, terms = _FusedPPOLoss.apply(*b, C)
    (loss * 3.0).backward()                                      # an upstream scale, like GradScaler's
    torch.testing.assert_close(loss, ref_loss.detach().float(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(terms, ref_terms.detach().float(), rtol=1e-5, atol=1e-6)
    for ta, tb in zip(a[:4], b[:4]):
        assert tb.grad.dtype == tb.dtype and tb.grad.shape == tb.shape
        tol = 2e-3 if tb.dtype == torch.float16 else 1e-5
        torch.testing.assert_close(tb.grad.float(), 3.0 * ta.grad.float(), rtol=tol, atol=tol * 1e-3)


def test_out_of_range_action_poisons_the_loss():
    from mapf_amd.model import _FusedPPOLoss
    x = list(_inputs(4, 2, 0, torch.float32))
    x[5] = x[5].clone()
    x[5][0, 0] = 7
    loss, _ = _FusedPPOLoss.apply(*x, C)
    assert torch.isnan(loss)


def test_model_update_fused_equals_unfused():
    from mapf_amd.model import Model
    torch.manual_seed(0)
    m1 = Model(0, "cuda", global_model=True, numChannel=6, num_agents=8, fov=9)
    m2 = copy.deepcopy(m1)
    m2.fused_loss = False
    g = torch.Generator(device="cuda").manual_seed(1)
    rows = 64
    obs = (torch.rand(rows, 8, 6, 9, 9, device="cuda", generator=g) < 0.3).float()
    vec = torch.randn(rows, 8, 4, device="cuda", generator=g)
    ret, v, cret, cv = (torch.randn(rows, 8, device="cuda", generator=g) for _ in range(4))
    act = torch.randint(0, 5, (rows, 8), device="cuda", generator=g)
    ps = torch.softmax(torch.randn(rows, 8, 5, device="cuda", generator=g), -1)
    tv = (torch.rand(rows, 8, 5, device="cuda", generator=g) < 0.7).float()
    for m in (m1, m2):                        # dropout off: both forwards see the same net
        m.network.eval()
        m.net_scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 8)   # no fp16 overflow: Adam steps
    s1 = m1.train(obs, vec, ret, cret, v, cv, act, ps, None, tv, 1.0)
    s2 = m2.train(obs, vec, ret, cret, v, cv, act, ps, None, tv, 1.0)
    assert all(torch.isfinite(torch.tensor(float(v))) for v in s1)
    for i, (a, b) in enumerate(zip(s1, s2)):
        assert abs(float(a) - float(b)) <= 1e-3 * max(1.0, abs(float(b))), (i, a, b)
    # the gradients both updates applied (left in .grad: unscaled and clipped by the same
    # norm).  Not the weights: Adam's first step is about lr * sign(grad), which flips
    # with the summation order wherever a gradient is ~0
    pairs = list(zip(m1.network.parameters(), m2.network.parameters()))
    assert all((p1.grad is None) == (p2.grad is None) for p1, p2 in pairs)   # heads the loss never reads
    pairs = [(p1, p2) for p1, p2 in pairs if p1.grad is not None]
    g1 = torch.cat([p1.grad.flatten() for p1, _ in pairs])
    g2 = torch.cat([p2.grad.flatten() for _, p2 in pairs])
    # the loss kernel itself is pinned to 1e-5 above; here the fp16 backward through the whole
    # net amplifies one-ulp differences of its gradient (1.01e-3 measured on one box, with the
    # gradient clipped to norm 10): a plumbing error would show as O(1)
    assert ((g1 - g2).norm() / g2.norm()).item() < 3e-3
    # per parameter: the first convolutions' gradients pass through every fp16 backward
    # layer of the net, so a one-ulp difference in the fp16 loss gradient grows to ~2 %
    # there (2.04 % measured on one box, MIOpen's backward algorithm varies per box)
    for p1, p2 in pairs:
        assert ((p1.grad - p2.grad).norm() / p2.grad.norm().clamp_min(1e-30)).item() < 5e-2


@pytest.mark.parametrize("inf", [False, True])
def test_fused_optimizer_tail_matches_torch(inf):
    """_DeviceUpdate._fused_tail (mapf_optim_unscale_clip_adam: unscale + found-inf, clip_grad_norm_(10),
    Adam) against torch's path (_amp_foreach_non_finite_check_and_unscale_, clip_grad_norm_, fused
    capturable Adam with found_inf) over three steps on the same tensors (a channels_last conv weight
    among them): parameters, moments and the unscaled clipped gradients within fp32 rounding of a
    different summation / contraction order, steps and the grad norm equal to fp32 rounding; with an inf
    gradient in the second step, that step is skipped by both (parameters, moments, step unchanged)"""
    import types
    from mapf_amd.config import TrainingParameters
    from mapf_amd.model import _DeviceUpdate
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    g = torch.Generator(device="cuda").manual_seed(5)
    shapes = [(128, 6, 3, 3), (128,), (512, 512), (5, 512), (5,), (1536, 512), (7,)]
    base = [torch.randn(s, device="cuda", generator=g) * 0.1 for s in shapes]
    base[0] = base[0].contiguous(memory_format=torch.channels_last)
    grads = [[torch.randn(s, device="cuda", generator=g).contiguous(memory_format=torch.channels_last
             if len(s) == 4 else torch.contiguous_format) * (2.0 ** 8) * 0.02 for s in shapes] for _ in range(3)]
    if inf:
        grads[1][2][3, 4] = float("inf")
    res = []
    for fused in (True, False):
        ps = [torch.nn.Parameter(b.clone()) for b in base]
        opt = torch.optim.Adam(ps, lr=TrainingParameters.lr, fused=True, capturable=True)
        scale = torch.full((1,), 2.0 ** 8, device="cuda")
        found = torch.zeros((), device="cuda")
        ns = types.SimpleNamespace(model=types.SimpleNamespace(fused_optim=True), scale=scale, found_inf=found)
        norms, founds = [], []
        for step in range(3):
            for p, gr in zip(ps, grads[step]):
                p.grad = gr.clone()
            found.zero_()
            if fused:
                assert _DeviceUpdate._fused_tail_ok(ns, opt, ps)
                norm = _DeviceUpdate._fused_tail(ns, opt, ps).clone()
            else:
                torch._amp_foreach_non_finite_check_and_unscale_([p.grad for p in ps], found,
                                                                 scale.double().reciprocal().float())
                norm = torch.nn.utils.clip_grad_norm_(ps, TrainingParameters.MAX_GRAD_NORM)
                opt.grad_scale, opt.found_inf = None, found
                opt.step()
                opt.grad_scale = opt.found_inf = None
            norms.append(norm.item())
            founds.append(found.item())
        st = [opt.state[p] for p in ps]
        res.append(([p.detach() for p in ps], [x["exp_avg"] for x in st], [x["exp_avg_sq"] for x in st],
                    [x["step"].item() for x in st], [p.grad for p in ps], norms, founds))
    (pf, mf, vf, sf, gf, nf, ff), (pt, mt, vt, stt, gt, nt, ft) = res
    assert ff == ft == ([0.0, 1.0, 0.0] if inf else [0.0, 0.0, 0.0])
    assert sf == stt == [2.0 if inf else 3.0] * len(shapes)
    np.testing.assert_allclose(nf, nt, rtol=1e-5)
    for a, b in zip(pf + mf + vf, pt + mt + vt):
        torch.testing.assert_close(a, b, rtol=2e-5, atol=1e-9)
    for a, b in zip(gf, gt):
        torch.testing.assert_close(a, b, rtol=2e-5, atol=1e-9, equal_nan=True)
