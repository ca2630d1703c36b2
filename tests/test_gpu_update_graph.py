"""The PPO update on the device (Model._train_device, model.py:78-199 of the reference): the
whole AMP update -- HIP normalisation, forward, fused loss, backward, unscale + found-inf,
clip, fused Adam, loss-scale update -- captured once per minibatch shape and replayed.  With
MIOpen's deterministic algorithms the replays must apply the same updates as the eager body (same
kernels: bitwise in practice), change the weights, keep the AMP state on the device, and leave the
acting path on the new weights.

The graphed model and its eager twins train INTERLEAVED, with small tensors allocated and freed
between updates: before round 5 that made a later replay non-finite.  The cause was the HIP
runtime's packet capture replaying a captured memset only once, so every captured multi-block
reduction (bias gradients, grad norm) summed stale partials (DESIGN.md 6a,
test_gpu_graph_capture_mode.py); mapf_amd switches that capture mode off."""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _batch(g, rows=64, n=8):
    obs = (torch.rand(rows, n, 6, 9, 9, device="cuda", generator=g) < 0.3).float()
    vec = torch.randn(rows, n, 4, device="cuda", generator=g)
    ret, v, cret, cv = (torch.randn(rows, n, device="cuda", generator=g) for _ in range(4))
    act = torch.randint(0, 5, (rows, n), device="cuda", generator=g)
    ps = torch.softmax(torch.randn(rows, n, 5, device="cuda", generator=g), -1)
    tv = (torch.rand(rows, n, 5, device="cuda", generator=g) < 0.7).float()
    return obs, vec, ret, cret, v, cv, act, ps, tv


def _churn():
    """small tensors of 4 B .. 256 KiB allocated, NaN-filled and freed (the small-pool traffic the
    host side of an update or a second model makes)"""
    ts = [torch.full((1 << (k % 17),), float("nan"), device="cuda") for k in range(600)]
    torch.cuda.synchronize()
    del ts


@pytest.fixture
def deterministic_convs():
    """MIOpen's deterministic convolution algorithms for the test (its default backward reduces in a
    run-dependent order, which Adam's first steps amplify)"""
    old = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    yield
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = old


@pytest.mark.parametrize("hip_attention", [True, False])
def test_graphed_updates_equal_eager_updates(deterministic_convs, hip_attention, monkeypatch):
    from mapf_amd.model import Model
    from mapf_amd.net import _SelfAttention
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    monkeypatch.setattr(_SelfAttention, "hip_attention", hip_attention)
    torch.manual_seed(0)
    m1 = Model(0, "cuda", global_model=True, numChannel=6, num_agents=8, fov=9)
    m2 = copy.deepcopy(m1)
    m2.graph_update = False
    m4 = copy.deepcopy(m2)                      # a second eager twin: the backward's own run-to-run spread
    for m in (m1, m2, m4):
        m.network.eval()                        # no dropout: both see the same net
        m.net_scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 8)
    g = torch.Generator(device="cuda").manual_seed(1)
    batches = [_batch(g) for _ in range(6)]
    w0 = m1.network.conv1.weight.detach().clone()
    init = [p.detach().clone() for p in m1.network.parameters()]
    runs = {id(m): [] for m in (m1, m2, m4)}
    for (obs, vec, ret, cret, v, cv, act, ps, tv) in batches:
        for m in (m1, m2, m4):               # a second model's eager update between two replays
            runs[id(m)].append(m.train(obs, vec, ret, cret, v, cv, act, ps, None, tv, 1.0))
            _churn()
    for k in range(len(batches)):
        s1, s2, s4 = runs[id(m1)][k], runs[id(m2)][k], runs[id(m4)][k]
        # (grad_norm, stats[8], is inf when the fp16 backward overflowed: the AMP step is then
        # skipped on the device and the scale halved -- in both models alike)
        assert all(np.isfinite(float(x)) for i, x in enumerate(s1) if i != 8), (k, s1)
        for i, (a, b) in enumerate(zip(s1, s2)):
            a, b = float(a), float(b)
            if i == 8:                          # a non-finite norm only where the eager one is too
                assert np.isfinite(a) == np.isfinite(b) and not np.isnan(a), (k, a, b)
                if not np.isfinite(b):
                    continue
            assert abs(a - b) <= max(1e-5 * max(1.0, abs(b)), 3 * abs(float(s4[i]) - b)), (k, i, a, b, float(s4[i]))
    assert len(m1.network._h16) == 0            # the acting path's fp16 weights are re-read
    upd = next(iter(m1._updates.values()))
    assert upd.graph is not None and upd.eager_runs == upd.WARMUP   # updates 3..6 were replays
    assert not torch.equal(m1.network.conv1.weight, w0)            # ... which moved the weights
    # the weights after six updates: equal to the eager twins' (or within their own spread, should
    # MIOpen's deterministic algorithms still differ between runs)
    delta = lambda m: torch.cat([(p.detach() - p0).flatten() for p, p0 in zip(m.network.parameters(), init)])  # noqa
    d1, d2, d4 = delta(m1), delta(m2), delta(m4)
    r_ge = ((d1 - d2).norm() / d2.norm()).item()
    r_ee = ((d4 - d2).norm() / d2.norm()).item()
    print(f"relative delta difference: graph vs eager {r_ge:.4f}, eager vs eager {r_ee:.4f}")
    assert d2.norm() > 0 and r_ge <= max(2.5 * r_ee, 1e-4), (r_ge, r_ee)
    torch.testing.assert_close(m1._updates[next(iter(m1._updates))].scale,
                               m2._updates[next(iter(m2._updates))].scale)
    # acting after graphed updates == acting of a model holding the same weights
    saved, m1._updates = m1._updates, {}         # (captured graphs are not copyable)
    m3 = copy.deepcopy(m1)
    m1._updates = saved
    obs, vec = batches[0][0], batches[0][1]
    torch.manual_seed(5)
    a1 = m1.network(obs, vec)
    torch.manual_seed(5)
    a3 = m3.network(obs, vec)
    with torch.no_grad():
        torch.manual_seed(5)
        f1 = m1.network(obs, vec)
        torch.manual_seed(5)
        f3 = m3.network(obs, vec)
    with torch.no_grad():
        torch.manual_seed(5)
        f1b = m1.network(obs, vec)
    torch.testing.assert_close(a1[0], a3[0], atol=5e-3, rtol=1e-2)   # MIOpen: last-bit run-to-run spread
    assert all(torch.equal(x, y) for x, y in zip(f1, f3))           # the acting path: bit-identical
    assert all(torch.equal(x, y) for x, y in zip(f1, f1b))


def test_update_shapes_get_their_own_graphs():
    from mapf_amd.model import Model
    torch.manual_seed(0)
    m = Model(0, "cuda", global_model=True, numChannel=6, num_agents=8, fov=9)
    m.net_scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 8)
    g = torch.Generator(device="cuda").manual_seed(2)
    for rows in (32, 48, 32, 48, 32, 48, 32):
        b = _batch(g, rows)
        s = m.train(*b[:8], None, b[8], 0.5)
        assert all(np.isfinite(float(x)) or (k == 8 and np.isinf(float(x))) for k, x in enumerate(s))
    assert len(m._updates) == 2 and all(u.graph is not None for u in m._updates.values())


def test_graphed_updates_draw_dropout_masks_like_eager(deterministic_convs):
    """Dropout ON (train mode) at the fused training sites (_DropResLN, _GeluDropout: the counter-hash
    masks seeded from SCRIMPNet._train_seed in device memory, incremented by every forward -- a captured
    increment in the graph): the graphed updates equal an eager twin's, update by update, so every replay
    drew the mask the eager forward drew; and consecutive updates draw different masks (the same
    minibatch twice gives different losses).  torch's own dropout sites (the tokens' and the last
    residual's, torch's RNG) are set to 0 so only the fused ones draw."""
    from mapf_amd.model import Model
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    torch.manual_seed(0)
    m1 = Model(0, "cuda", global_model=True, numChannel=6, num_agents=8, fov=9)
    with torch.no_grad():
        m1.network.dropout.p = 0.0
        m1.network.transformer.layers[-1][1].fn.fn.do2.p = 0.0
    m1.net_scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 8)
    m2 = copy.deepcopy(m1)
    m2.graph_update = False
    m2.net_scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 8)
    for m in (m1, m2):                                       # the same starting count (each its own tensor)
        m.network.__dict__["_train_seed"] = torch.tensor([42], dtype=torch.int64, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(3)
    b = _batch(g)
    s1 = [m1.train(*b[:8], None, b[8], 1.0) for _ in range(6)]
    s2 = [m2.train(*b[:8], None, b[8], 1.0) for _ in range(6)]
    upd = next(iter(m1._updates.values()))
    assert upd.graph is not None and upd.eager_runs == upd.WARMUP
    for k in range(6):
        for i, (a, c) in enumerate(zip(s1[k], s2[k])):
            assert float(a) == float(c) or (np.isnan(float(a)) and np.isnan(float(c))), (k, i, float(a), float(c))
    # the same minibatch, new masks: the loss terms move from update to update (the weights move by ~lr only)
    assert len({round(float(s[0]), 6) for s in s1}) == 6, [float(s[0]) for s in s1]
    for p1, p2 in zip(m1.network.parameters(), m2.network.parameters()):
        assert torch.equal(p1, p2)
