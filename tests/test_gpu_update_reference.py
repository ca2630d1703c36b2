"""The GPU PPO update pinned to the REFERENCE's update (tests/golden/g5_net.npz: one reference
Model.train, model.py:78-199, on CPU in fp32 with deterministic weights and dropout off).

Model.train's default GPU path -- HIP advantage normalisation, the training forward on the HIP
kernels (_CastParams, _BiasReLU / _BiasReLUPool conv epilogues, _HipLayerNorm, _HipAttention,
optionally _SplitKLinear), the fused loss, backward, AMP unscale / found-inf / clip, fused Adam,
the loss-scale update -- runs once eagerly and once as the captured hipGraph replay, from the same
start (weights, Adam state, loss scale and multiplier reset in place after the capture's two
warm-up updates).  Tolerances come from fp16 autocast (the reference runs fp32 on the CPU):
  * the 12 returned stats within 2e-2 relative (the loss terms, grad norm, multiplier); the means
    of the normalised advantages (~1e-8 in fp32) within 1e-5; clip_frac within one element of the
    32 (a ratio within fp16 rounding of 1 +- clip may flip);
  * the weights: Adam's first step moves every element by lr * g / (|g| + eps) -- +-lr wherever
    |g| >> eps -- so each probed element of after_* is within 2 lr of the reference's (the bound of
    tests/test_gpu_distributed_update.py), and the DIRECTION of the step agrees with the
    reference's on >= 99 % of the elements the reference moved by more than lr / 2 (those whose
    fp32 gradient is not within fp16 noise of 0).
The NaN tests: the training epilogues keep torch's NaN semantics, so a NaN in a conv
output reaches the loss and GradScaler's found-inf skips the step, as with F.relu / max_pool2d."""
import numpy as np
import pytest
import torch

from golden_io import load

pytestmark = pytest.mark.gpu

FIELDS = ["observation", "vector", "returns", "cost_returns", "old_v", "old_cv", "action", "old_ps", "train_valid"]
PROBES = ["conv1.weight", "fully_connected_2.bias", "transformer.layers.1.0.fn.fn.to_qkv.weight", "policy_layer.weight"]
LR = 1e-5                                  # TrainingParameters.lr (alg_parameters.py:52)


@pytest.fixture
def two_agents():
    from mapf_amd.config import EnvParameters
    old = EnvParameters.N_AGENTS
    EnvParameters.N_AGENTS = 2             # make_golden.py g5_net: set_params(2, 9)
    yield
    EnvParameters.N_AGENTS = old


def _model():
    from mapf_amd.model import Model
    from test_net import det_weights
    m = Model(0, "cuda", global_model=True, numChannel=6, num_agents=2, fov=9)
    w = det_weights(m.network.state_dict())
    m.network.load_state_dict(w)
    m.network.eval()                       # dropout off, as the reference update was made
    return m, w


def _reset(m, w):
    """the state before the first update, in place (the captured graph keeps these tensors)"""
    from mapf_amd.config import LagrangianParameters, TrainingParameters
    from mapf_amd.model import get_lagrangian
    with torch.no_grad():
        sd = m.network.state_dict()
        for k, v in w.items():
            sd[k].copy_(v)
        for st in m.net_optimizer.state.values():
            for key in ("exp_avg", "exp_avg_sq", "step"):
                st[key].zero_()
        m.net_scaler._scale.fill_(m.net_scaler._init_scale)
        m.net_scaler._growth_tracker.zero_()
    m.lagrange = get_lagrangian(LagrangianParameters.LAGRANGIAN_TYPE, TrainingParameters.COST_LIMIT_PER_AGENT)
    m.network.weights_updated()


def _train(m, z):
    g = lambda k: z["train_" + k]  # noqa: E731
    hidden = np.zeros((len(g("returns")), 2, 2, 512), np.float32)
    stats = m.train(g("observation"), g("vector"), g("returns"), g("cost_returns"), g("old_v"), g("old_cv"),
                    g("action"), g("old_ps"), hidden, g("train_valid"), 3.0)
    return np.array([float(np.asarray(x)) for x in stats])


@pytest.mark.parametrize("split_k", [False, True])
@pytest.mark.parametrize("graph", [False, True])
def test_device_update_matches_reference_update(two_agents, graph, split_k, monkeypatch):
    from mapf_amd.net import _SplitKLinear
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    if split_k:        # the 17-token layers' split weight gradient (34,816+ rows in real minibatches)
        monkeypatch.setattr(_SplitKLinear, "MIN_ROWS", 8)
    calls = []
    orig = _SplitKLinear.backward
    monkeypatch.setattr(_SplitKLinear, "backward", staticmethod(lambda ctx, gy: calls.append(1) or orig(ctx, gy)))
    z = load("g5_net")
    torch.manual_seed(0)
    m, w = _model()
    assert m.fused_loss
    m.graph_update = graph
    if graph:
        from mapf_amd.model import _DeviceUpdate
        for _ in range(_DeviceUpdate.WARMUP):      # the eager warm-ups before the capture
            _train(m, z)
        _reset(m, w)
    calls.clear()
    got = _train(m, z)
    upd = next(iter(m._updates.values()))
    assert (upd.graph is not None) == graph
    assert (len(calls) > 0) == split_k, calls      # (graph: the capture traced the backward once)
    assert upd.found_inf.item() == 0, "the first AMP step overflowed"
    ref = z["train_stats"]
    print(f"graph={graph} split_k={split_k}\n  gpu {np.array2string(got, precision=6)}\n"
          f"  ref {np.array2string(ref, precision=6)}")
    idx = [0, 1, 2, 3, 4, 5, 6, 8, 11]
    np.testing.assert_allclose(got[idx], ref[idx], rtol=2e-2, atol=1e-4)
    np.testing.assert_allclose(got[[9, 10]], ref[[9, 10]], atol=1e-5)
    assert abs(got[7] - ref[7]) <= 1 / 32 + 1e-6, (got[7], ref[7])
    sd = m.network.state_dict()
    moved_total = 0
    for k in PROBES:
        before = w[k].numpy().reshape(-1)[:2048]
        after_ref = z["after_" + k.replace(".", "_")]
        after = sd[k].detach().float().cpu().numpy().reshape(-1)[:2048]
        d_ref, d = after_ref - before, after - before
        assert np.abs(after - after_ref).max() <= 2 * LR * 1.001, k
        # the deep layers' reference gradients are ~eps-sized for these weights (conv1's step <= 2e-8,
        # layer 1's to_qkv 7e-12): their direction is below fp16 autocast's resolution and not compared
        moved = np.abs(d_ref) > LR / 2
        agree = np.mean(np.sign(d[moved]) == np.sign(d_ref[moved])) if moved.any() else float("nan")
        print(f"  {k}: |step| ref max {np.abs(d_ref).max():.2e} gpu max {np.abs(d).max():.2e}; "
              f"{moved.sum()} elements moved > lr/2, step direction agrees on {agree:.4f}")
        if moved.any():
            assert agree >= 0.99, (k, agree)
        moved_total += moved.sum()
    assert moved_total >= 1024               # policy_layer.weight: every element moved by ~lr


def test_relu_epilogues_keep_nan_like_torch():
    """_BiasReLU / _BiasReLUPool with NaNs in the conv output: forward and gradient equal torch's
    F.relu / max_pool2d on the same fp16 arithmetic, NaNs included (max_pool2d's argmax takes the
    window's NaN; threshold_backward passes the gradient where the output is NaN)."""
    from mapf_amd.net import _BiasReLU, _BiasReLUPool
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    g = torch.Generator(device="cuda").manual_seed(5)
    for pooled in (False, True):
        r0 = torch.randn(8, 128, 6, 6, device="cuda", generator=g).half().contiguous(memory_format=torch.channels_last)
        r0[0, 3, 2, 2] = float("nan")
        r0[1, 7, 0, 1] = float("nan")
        r0[2, 9, 4, 4] = float("inf")
        b0 = (0.1 * torch.randn(128, device="cuda", generator=g)).half()
        gp = torch.randn(8, 128, 3 if pooled else 6, 3 if pooled else 6, device="cuda", generator=g).half()
        out = []
        for hip in (True, False):
            r, b = r0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
            if hip:
                y = _BiasReLUPool.apply(r, b) if pooled else _BiasReLU.apply(r.clone(), b)
            else:
                a = torch.relu((r.float() + b.float().view(-1, 1, 1)).half())
                y = torch.nn.functional.max_pool2d(a, 2) if pooled else a
            y.backward(gp.contiguous(memory_format=torch.channels_last))
            out.append((y.detach().float(), r.grad.float(), b.grad.float()))
        (yh, grh, gbh), (yt, grt, gbt) = out
        assert torch.isnan(yh).sum() == torch.isnan(yt).sum() > 0
        torch.testing.assert_close(yh, yt, rtol=0, atol=0, equal_nan=True)
        torch.testing.assert_close(grh, grt, rtol=0, atol=0, equal_nan=True)
        torch.testing.assert_close(gbh, gbt, rtol=2e-3, atol=2e-3, equal_nan=True)


def test_nan_in_a_conv_output_skips_the_step(two_agents):
    """A NaN observation element makes conv1's outputs around it NaN: the loss is NaN, GradScaler's
    found-inf is set, the step is skipped (weights unchanged) and the loss scale halves -- what the
    reference's torch ops do; with fmaxf-style ReLUs the NaN was zeroed and Adam stepped."""
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    z = load("g5_net")
    torch.manual_seed(0)
    m, w = _model()
    m.graph_update = False
    z = {k: (v.copy() if k.startswith("train_") else v) for k, v in z.items()}
    z["train_observation"][3, 1, 2, 4, 4] = float("nan")
    scale0 = float(m.net_scaler._init_scale)
    stats = _train(m, z)
    upd = next(iter(m._updates.values()))
    assert upd.found_inf.item() == 1
    assert np.isnan(stats[0])
    assert m.net_scaler._scale.item() == scale0 * 0.5
    sd = m.network.state_dict()
    for k in PROBES:
        np.testing.assert_array_equal(sd[k].detach().cpu().numpy(), w[k].numpy(), err_msg=k)
