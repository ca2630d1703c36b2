"""GPU tests of the acting forward's fused epilogues (csrc/mapf_policy.hip):
SCRIMPNet._forward_fused against the same network's PyTorch path (autocast fp16,
dropout off in both: the paths draw different dropout masks), and the dropout
kernels' keep rate and scaling.  The reference outputs themselves pin the PyTorch
path (tests/test_net.py, fp32 CPU)."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")


def _net(n_agents=8):
    from mapf_amd.model import Model
    torch.manual_seed(3)
    return Model(0, "cuda", numChannel=6, num_agents=n_agents, fov=9).network


@pytest.mark.parametrize("B,own", [(5, True), (256, True), (256, False)])
def test_fused_acting_forward_matches_torch_path(B, own):
    net = _net().eval()                        # dropout off: both paths deterministic
    net.fused_attention = net.fused_residual_ln = net.own_conv = net.fused_linear = own
    g = torch.Generator(device="cuda").manual_seed(B)
    obs = (torch.rand(B, 8, 6, 9, 9, device="cuda", generator=g) < 0.25).float()
    vec = torch.randn(B, 8, 4, device="cuda", generator=g)
    with torch.no_grad():
        net.fused_acting = False
        ref = net(obs, vec)
        net.fused_acting = True
        got = net(obs, vec)
    names = ["policy", "value", "blocking", "policy_sig", "x", "logits", "cost_value"]
    for name, r, o in zip(names, ref, got):
        assert o.shape == r.shape, name
        # fp16 autocast on both sides; the fused LayerNorm / epilogues round like torch's
        # ops but reduce in a different order
        torch.testing.assert_close(o.float(), r.float(), rtol=3e-2, atol=3e-2, msg=name)


@pytest.mark.parametrize("own_conv,fused_linear,training", [(True, True, False), (True, False, False),
                                                              (True, True, True)])
def test_fused_acting_forward_is_deterministic(own_conv, fused_linear, training):
    """the acting forward is a function of weights and inputs: bit-identical over repeated
    calls and on a deep copy of the network (a kernel that reads memory it did not write, or
    races on LDS, shows up here first)"""
    import copy
    net = _net().train(training)               # training: dropout on, masks from the seeded hash stream
    net.own_conv, net.fused_linear = own_conv, fused_linear
    g = torch.Generator(device="cuda").manual_seed(9)
    obs = (torch.rand(300, 8, 6, 9, 9, device="cuda", generator=g) < 0.25).float()
    vec = torch.randn(300, 8, 4, device="cuda", generator=g)
    twin = copy.deepcopy(net)
    with torch.no_grad():
        call = lambda m: (torch.manual_seed(4), m(obs, vec))[1]    # noqa
        runs = [call(net) for _ in range(3)] + [call(twin)]
        junk = torch.full((1 << 26,), float("nan"), device="cuda")   # recycle the freed blocks as NaN
        del junk
        runs.append(call(net))
    names = ["policy", "value", "blocking", "policy_sig", "x", "logits", "cost_value"]
    for j, r in enumerate(runs[1:], 1):
        bad = [n for n, a, b in zip(names, runs[0], r) if not torch.equal(a, b)]
        assert not bad, (j, bad, [(a.float() - b.float()).abs().max().item() for a, b in zip(runs[0], r)])


def test_training_forward_keeps_torch_ops():
    net = _net()
    obs = (torch.rand(4, 8, 6, 9, 9, device="cuda") < 0.25).float()
    vec = torch.randn(4, 8, 4, device="cuda")
    out = net(obs, vec)                        # grad enabled: the autograd path
    out[1].sum().backward()
    assert net.conv1.weight.grad is not None and torch.isfinite(net.conv1.weight.grad).all()


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def test_dropout_kernels_keep_rate_and_scale():
    from mapf_amd import _lib
    lib = _lib.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    n = 1 << 22
    x = torch.zeros(n, device="cuda")
    y = torch.ones(n, dtype=torch.float16, device="cuda")
    _lib.check(lib.mapf_dropout_residual(_p(x), _p(y), n, 0.2, 1234, st))
    kept = (x == 1.25).float().mean().item()
    assert abs(kept - 0.8) < 3e-3 and bool(((x == 0) | (x == 1.25)).all())
    # a different seed draws a different mask
    x2 = torch.zeros(n, device="cuda")
    _lib.check(lib.mapf_dropout_residual(_p(x2), _p(y), n, 0.2, 1235, st))
    assert (x != x2).float().mean().item() > 0.2
    # the counter hash's masks: every lane of a float4 at the keep rate, neighbours (in a float4,
    # across float4s, a row apart) and the two seeds' masks uncorrelated
    m = (x == 1.25).float()
    assert all(abs(m[k::4].mean().item() - 0.8) < 5e-3 for k in range(4))
    for lag in (1, 3, 4, 5, 512):
        c = torch.corrcoef(torch.stack([m[:-lag], m[lag:]]))[0, 1].item()
        assert abs(c) < 5e-3, (lag, c)
    c = torch.corrcoef(torch.stack([m, (x2 == 1.25).float()]))[0, 1].item()
    assert abs(c) < 5e-3, c
    # GELU + dropout: kept entries equal fp16(gelu(v) * 1.25)
    v = torch.linspace(-4, 4, n, device="cuda").half()
    h = v.clone()
    _lib.check(lib.mapf_gelu_dropout_f16(_p(h), n, 0.2, 99, st))
    ref = (torch.nn.functional.gelu(v.float()).half().float() * 1.25).half()
    keep = h != 0
    assert abs(keep.float().mean().item() - 0.8) < 5e-3
    torch.testing.assert_close(h[keep], ref[keep], rtol=0, atol=2e-3)
    # p = 0 is the identity
    h0 = v.clone()
    _lib.check(lib.mapf_gelu_dropout_f16(_p(h0), n, 0.0, 99, st))
    torch.testing.assert_close(h0, torch.nn.functional.gelu(v.float()).half(), rtol=0, atol=2e-3)


def test_layernorm_and_conv_epilogues_vs_torch():
    from mapf_amd import _lib
    lib = _lib.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rows = 1000
    x = torch.randn(rows, 512, device="cuda") * 3 + 1
    ln = torch.nn.LayerNorm(512).cuda()
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.5, 0.5)
    y = torch.empty(rows, 512, dtype=torch.float16, device="cuda")
    _lib.check(lib.mapf_layernorm_f16(_p(x), 512, _p(ln.weight), _p(ln.bias), _p(y), rows, 512, 1e-5, st))
    torch.testing.assert_close(y.float(), ln(x).detach().half().float(), rtol=0, atol=4e-3)
    # conv epilogue: NHWC [B, C, H, W] channels_last fp16
    B, C, H, W = 7, 128, 9, 9
    c = torch.randn(B, C, H, W, device="cuda").half().contiguous(memory_format=torch.channels_last)
    bias = torch.randn(C, device="cuda").half()
    ref = torch.relu(c + bias.view(1, C, 1, 1))
    pooled = torch.empty(B, C, H // 2, W // 2, dtype=torch.float16, device="cuda",
                         memory_format=torch.channels_last)
    _lib.check(lib.mapf_nhwc_bias_relu_pool2(_p(c), _p(bias), _p(pooled), B, H, W, C, st))
    assert torch.equal(pooled, torch.nn.functional.max_pool2d(ref, 2))
    _lib.check(lib.mapf_nhwc_bias_relu(_p(c), _p(bias), B * H * W, C, st))
    assert torch.equal(c, ref)


@pytest.mark.parametrize("n,rows", [(17, 17), (17, 1), (17, 16), (5, 5), (1, 1), (32, 32), (32, 3)])
def test_attention_kernel_vs_sdpa(n, rows):
    from mapf_amd import _lib
    lib = _lib.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    B, d, hh = 300, 512, 16
    g = torch.Generator(device="cuda").manual_seed(n * 100 + rows)
    qkv = (torch.randn(B, n, 3 * d, device="cuda", generator=g) * 2).half()
    scale = d ** -0.5
    out = torch.empty(B, rows, d, dtype=torch.float16, device="cuda")
    q = qkv[:, :rows, :d]
    _lib.check(lib.mapf_attention_f16(_p(qkv), _p(qkv[..., d:]), _p(qkv[..., 2 * d:]), _p(out), B, n, rows,
                                      3 * d, n * 3 * d, 3 * d, n * 3 * d, hh, d // hh, scale, st))
    heads = lambda t: t.reshape(B, t.shape[1], hh, d // hh).transpose(1, 2).float()
    ref = torch.nn.functional.scaled_dot_product_attention(heads(q), heads(qkv[..., d:2 * d]),
                                                           heads(qkv[..., 2 * d:]), scale=scale)
    ref = ref.transpose(1, 2).reshape(B, rows, d)
    # fp32 scores and softmax on fp16 inputs; P is rounded to fp16 before P.V (as flash
    # SDPA does) and the output to fp16
    torch.testing.assert_close(out.float(), ref, rtol=4e-3, atol=4e-3)
    # argument checks fail without launching: too many tokens, unaligned strides
    assert lib.mapf_attention_f16(_p(qkv), _p(qkv), _p(qkv), _p(out), B, 33, 1, 3 * d, 0, 3 * d, 0, hh, 32, scale,
                                  st) != 0
    assert lib.mapf_attention_f16(_p(qkv), _p(qkv), _p(qkv), _p(out), B, n, 1, 3 * d + 4, 0, 3 * d, 0, hh, 32,
                                  scale, st) != 0


def test_residual_layernorm_equals_two_launches():
    from mapf_amd import _lib
    lib = _lib.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rows = 777
    x = torch.randn(rows, 512, device="cuda") * 2
    y = torch.randn(rows, 512, device="cuda").half()
    g = torch.rand(512, device="cuda") + 0.5
    e = torch.randn(512, device="cuda")
    x1, x2 = x.clone(), x.clone()
    z1 = torch.empty(rows, 512, dtype=torch.float16, device="cuda")
    z2 = torch.empty_like(z1)
    for p in (0.0, 0.2):
        _lib.check(lib.mapf_dropout_residual(_p(x1), _p(y), x1.numel(), p, 77, st))
        _lib.check(lib.mapf_layernorm_f16(_p(x1), 512, _p(g), _p(e), _p(z1), rows, 512, 1e-5, st))
        _lib.check(lib.mapf_dropout_residual_layernorm(_p(x2), _p(y), _p(g), _p(e), _p(z2), rows, 512, 1e-5, p, 77,
                                                       st))
        assert torch.equal(x1, x2) and torch.equal(z1, z2)


def test_tokens_layernorm_equals_two_launches():
    from mapf_amd import _lib
    lib = _lib.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    B, L, D = 333, 16, 512
    A = torch.rand(B, L, device="cuda")
    VV = torch.randn(B, D, device="cuda").half()
    cls, pos = torch.randn(D, device="cuda"), torch.randn(L + 1, D, device="cuda")
    g, e = torch.rand(D, device="cuda") + 0.5, torch.randn(D, device="cuda")
    for p in (0.0, 0.1):
        x1 = torch.empty(B, L + 1, D, device="cuda")
        x2 = torch.empty_like(x1)
        z1 = torch.empty(B, L + 1, D, dtype=torch.float16, device="cuda")
        z2 = torch.empty_like(z1)
        _lib.check(lib.mapf_tokens(_p(x1), _p(A), _p(VV), _p(cls), _p(pos), B, L, D, p, 5, st))
        _lib.check(lib.mapf_layernorm_f16(_p(x1), D, _p(g), _p(e), _p(z1), B * (L + 1), D, 1e-5, st))
        _lib.check(lib.mapf_tokens_layernorm(_p(x2), _p(A), _p(VV), _p(cls), _p(pos), B, L, D, p, 5, _p(g), _p(e),
                                             1e-5, _p(z2), st))
        assert torch.equal(x1, x2) and torch.equal(z1, z2)
        if p == 0:                             # the token formula itself (net.py:124-131)
            ref = torch.cat([cls.expand(B, 1, D), A[..., None] * VV.float()[:, None]], 1) + pos
            torch.testing.assert_close(x1, ref, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("B", [1, 7, 333])
def test_linear512_tokens_variant_equals_tokens_then_linear512(B):
    """mapf_tokens_layernorm(x = NULL) + mapf_linear512_tokens_residual_layernorm (the tokens
    recomputed in the epilogue) == mapf_tokens_layernorm(x) + mapf_linear512_residual_layernorm:
    bit-identical LayerNorm input, residual stream and LayerNorm output, dropout on and off."""
    from mapf_amd import _lib
    lib = _lib.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    L, D = 16, 512
    gen = torch.Generator(device="cuda").manual_seed(B)
    A = torch.rand(B, L, device="cuda", generator=gen)
    VV = torch.randn(B, D, device="cuda", generator=gen).half()
    cls, pos = torch.randn(D, device="cuda", generator=gen), torch.randn(L + 1, D, device="cuda", generator=gen)
    g0, e0 = torch.rand(D, device="cuda", generator=gen) + 0.5, torch.randn(D, device="cuda", generator=gen)
    g1, e1 = torch.rand(D, device="cuda", generator=gen) + 0.5, torch.randn(D, device="cuda", generator=gen)
    a = torch.randn(B * (L + 1), D, device="cuda", generator=gen).half()
    w = (torch.randn(D, D, device="cuda", generator=gen) / D ** 0.5).half()
    bias = (torch.randn(D, device="cuda", generator=gen) * 0.1).half()
    for p_tok, p in ((0.0, 0.0), (0.1, 0.2)):
        x1 = torch.empty(B, L + 1, D, device="cuda")
        y1, y2 = (torch.empty(B, L + 1, D, dtype=torch.float16, device="cuda") for _ in range(2))
        _lib.check(lib.mapf_tokens_layernorm(_p(x1), _p(A), _p(VV), _p(cls), _p(pos), B, L, D, p_tok, 11, _p(g0),
                                             _p(e0), 1e-5, _p(y1), st))
        _lib.check(lib.mapf_tokens_layernorm(None, _p(A), _p(VV), _p(cls), _p(pos), B, L, D, p_tok, 11, _p(g0), _p(e0),
                                             1e-5, _p(y2), st))
        z1, z2 = (torch.empty(B, L + 1, D, dtype=torch.float16, device="cuda") for _ in range(2))
        x2 = torch.full_like(x1, float("nan"))
        _lib.check(lib.mapf_linear512_residual_layernorm(_p(a), _p(w), _p(bias), _p(x1), _p(g1), _p(e1), _p(z1),
                                                         B * (L + 1), 1e-5, p, 22, st))
        _lib.check(lib.mapf_linear512_tokens_residual_layernorm(_p(a), _p(w), _p(bias), _p(x2), _p(g1), _p(e1), _p(z2),
                                                                B, L, 1e-5, p, 22, _p(A), _p(VV), _p(cls), _p(pos),
                                                                p_tok, 11, st))
        torch.cuda.synchronize()
        assert torch.equal(y1, y2) and torch.equal(x1, x2) and torch.equal(z1, z2), (p_tok, p)


def test_linear512_rows_variant_writes_back_every_kth_row():
    """mapf_linear512_residual_layernorm_rows(x_every = 17): z as the full launch for every row, the
    residual written back for rows 0, 17, 34, ... only (the rest untouched)"""
    from mapf_amd import _lib
    lib = _lib.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    gen = torch.Generator(device="cuda").manual_seed(5)
    rows, k = 17 * 41, 17
    a = torch.randn(rows, 512, device="cuda", generator=gen).half()
    w = (torch.randn(512, 512, device="cuda", generator=gen) / 512 ** 0.5).half()
    bias = (torch.randn(512, device="cuda", generator=gen) * 0.1).half()
    g1, e1 = torch.rand(512, device="cuda", generator=gen) + 0.5, torch.randn(512, device="cuda", generator=gen)
    x0 = torch.randn(rows, 512, device="cuda", generator=gen)
    x1, x2 = x0.clone(), x0.clone()
    z1, z2 = (torch.empty(rows, 512, dtype=torch.float16, device="cuda") for _ in range(2))
    _lib.check(lib.mapf_linear512_residual_layernorm(_p(a), _p(w), _p(bias), _p(x1), _p(g1), _p(e1), _p(z1), rows,
                                                     1e-5, 0.1, 3, st))
    _lib.check(lib.mapf_linear512_residual_layernorm_rows(_p(a), _p(w), _p(bias), _p(x2), _p(g1), _p(e1), _p(z2), rows,
                                                          1e-5, 0.1, 3, k, st))
    torch.cuda.synchronize()
    keep = torch.arange(rows, device="cuda") % k == 0
    assert torch.equal(z1, z2) and torch.equal(x2[keep], x1[keep]) and torch.equal(x2[~keep], x0[~keep])


def test_fp16_weight_cache_follows_in_place_updates():
    net = _net().eval()
    obs = (torch.rand(16, 8, 6, 9, 9, device="cuda") < 0.25).float()
    vec = torch.randn(16, 8, 4, device="cuda")
    with torch.no_grad():
        net(obs, vec)                          # fills the cache
        for prm in (net.conv1a.weight, net.transformer.layers[0][0].fn.fn.to_qkv.weight,
                    net.transformer.layers[1][0].fn.fn.to_qkv.bias, net.token_wV):
            prm.mul_(0.5)                      # an optimizer-style in-place update
        got = net(obs, vec)
        net.fused_acting = False
        ref = net(obs, vec)
    torch.testing.assert_close(got[1].float(), ref[1].float(), rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(got[5].float(), ref[5].float(), rtol=3e-2, atol=3e-2)


@pytest.fixture(params=[2, 0], ids=["image_resident", "per_tap"])
def conv_impl(request):
    """Both implicit-GEMM forms (mapf_conv_select: 2 image-resident, 0 per-tap staged; the default 1
    picks one of them per layer)."""
    from mapf_amd import _lib
    _lib.check(_lib.lib().mapf_conv_select(request.param))
    yield request.param
    _lib.check(_lib.lib().mapf_conv_select(1))


@pytest.mark.parametrize("ci,co,ks,H,B", [(128, 128, 3, 9, 37), (128, 128, 3, 11, 3), (128, 256, 2, 4, 50),
                                         (256, 256, 2, 5, 33), (256, 256, 2, 6, 7), (128, 128, 3, 9, 1),
                                         (128, 128, 3, 9, 1001), (128, 256, 2, 4, 2111), (256, 256, 2, 6, 1003)])
@pytest.mark.parametrize("relu", [0, 1])
def test_conv_kernel_vs_torch(ci, co, ks, H, B, relu, conv_impl):
    """mapf_conv_nhwc_f16 (MFMA implicit GEMM, csrc/mapf_conv.hip) == the autocast conv (fp16
    operands, fp32 accumulation, fp16 output; + fp16 bias, ReLU) to fp16 rounding -- ragged
    pixel counts (the last tile's rows past M), every padding tap, 3x3 and 2x2, and grids with
    more tiles than CUs (a persistent workgroup's K pipeline running on into its next tile)."""
    from mapf_amd import _lib
    g = torch.Generator(device="cuda").manual_seed(ci + co + H + B)
    cl = torch.channels_last
    x = torch.randn(B, ci, H, H, device="cuda", generator=g).half().contiguous(memory_format=cl)
    w = (torch.randn(co, ci, ks, ks, device="cuda", generator=g) / (ci * ks * ks) ** 0.5).half()
    b = torch.randn(co, device="cuda", generator=g).half()
    ref = torch.nn.functional.conv2d(x.float(), w.float(), None, 1, 1).half()
    if relu:
        ref = torch.relu((ref.float() + b.float().view(1, -1, 1, 1)).half().float()).half()
    Ho = H + 2 - ks + 1
    y = torch.full((B, co, Ho, Ho), float("nan"), dtype=torch.float16, device="cuda").contiguous(memory_format=cl)
    wp = w.permute(0, 2, 3, 1).contiguous()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(_lib.lib().mapf_conv_nhwc_f16(_p(x), _p(wp), _p(b), _p(y), B, H, H, ci, co, ks, 1, relu, st))
    torch.cuda.synchronize()
    assert torch.isfinite(y).all()
    torch.testing.assert_close(y.float(), ref.float(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("ci,co,ks,H,B", [(128, 128, 3, 9, 37), (128, 128, 3, 9, 1), (128, 128, 3, 11, 5),
                                         (256, 256, 2, 6, 1003), (256, 256, 2, 6, 7)])
def test_conv_pool_kernel_equals_conv_then_pool(ci, co, ks, H, B, conv_impl):
    """mapf_conv_nhwc_pool_f16 (whole-image tiles, pooled epilogue) == mapf_conv_nhwc_f16(relu=0) then
    mapf_nhwc_bias_relu_pool2, bit-identical; and == torch's relu(conv + b) then MaxPool2d(2) to
    fp16 rounding"""
    from mapf_amd import _lib
    L = _lib.lib()
    g = torch.Generator(device="cuda").manual_seed(ci + co + H + B)
    cl = torch.channels_last
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    x = torch.randn(B, ci, H, H, device="cuda", generator=g).half().contiguous(memory_format=cl)
    w = (torch.randn(co, ci, ks, ks, device="cuda", generator=g) / (ci * ks * ks) ** 0.5).half()
    b = torch.randn(co, device="cuda", generator=g).half()
    wp = w.permute(0, 2, 3, 1).contiguous()
    Ho = H + 2 - ks + 1
    raw = torch.empty(B, co, Ho, Ho, dtype=torch.float16, device="cuda").contiguous(memory_format=cl)
    _lib.check(L.mapf_conv_nhwc_f16(_p(x), _p(wp), _p(b), _p(raw), B, H, H, ci, co, ks, 1, 0, st))
    want = torch.empty(B, co, Ho // 2, Ho // 2, dtype=torch.float16, device="cuda").contiguous(memory_format=cl)
    _lib.check(L.mapf_nhwc_bias_relu_pool2(_p(raw), _p(b), _p(want), B, Ho, Ho, co, st))
    got = torch.full_like(want, float("nan"))
    _lib.check(L.mapf_conv_nhwc_pool_f16(_p(x), _p(wp), _p(b), _p(got), B, H, H, ci, co, ks, 1, st))
    torch.cuda.synchronize()
    assert torch.equal(got, want)
    ref = torch.nn.functional.max_pool2d(torch.relu(
        (torch.nn.functional.conv2d(x.float(), w.float(), None, 1, 1).half().float() + b.float().view(1, -1, 1, 1))
        .half().float()), 2)
    torch.testing.assert_close(got.float(), ref, rtol=1e-2, atol=1e-2)


def test_conv_kernel_rejects_other_shapes():
    from mapf_amd import _lib
    x = torch.zeros(1, dtype=torch.float16, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert _lib.lib().mapf_conv_nhwc_f16(_p(x), _p(x), _p(x), _p(x), 1, 9, 9, 6, 128, 3, 1, 1, st) == -1
    assert _lib.lib().mapf_conv_nhwc_f16(_p(x), _p(x), _p(x), _p(x), 1, 9, 9, 128, 128, 3, 3, 1, st) == -1


@pytest.mark.parametrize("rows", [1, 63, 64, 1000])
@pytest.mark.parametrize("p", [0.0, 0.2])
def test_linear512_epilogues_equal_linear_then_epilogue(rows, p):
    """mapf_linear512_gelu_dropout / _residual_layernorm (MFMA GEMM + epilogue, one launch) == torch's
    fp16 Linear followed by mapf_gelu_dropout_f16 / mapf_dropout_residual_layernorm with the same
    seed: the same dropout masks (every dropped element dropped in both), values to fp16 rounding of
    the GEMM's other summation order; ragged row counts (the last workgroup's rows past M)."""
    from mapf_amd import _lib
    L = _lib.lib()
    g = torch.Generator(device="cuda").manual_seed(rows)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    a = torch.randn(rows, 512, device="cuda", generator=g).half()
    w = (torch.randn(512, 512, device="cuda", generator=g) / 512 ** 0.5).half()
    b = (torch.randn(512, device="cuda", generator=g) * 0.1).half()
    seed = 1234 + rows
    # GELU + dropout
    ref = torch.nn.functional.linear(a, w, b).contiguous()
    _lib.check(L.mapf_gelu_dropout_f16(_p(ref), ref.numel(), p, seed, st))
    out = torch.full_like(ref, float("nan"))
    _lib.check(L.mapf_linear512_gelu_dropout(_p(a), _p(w), _p(b), _p(out), rows, p, seed, st))
    torch.cuda.synchronize()
    assert torch.equal(out == 0, ref == 0) or p == 0.0
    torch.testing.assert_close(out.float(), ref.float(), rtol=1e-2, atol=1e-2)
    # dropout + residual + LayerNorm
    gamma = 1 + 0.1 * torch.randn(512, device="cuda", generator=g)
    beta = 0.1 * torch.randn(512, device="cuda", generator=g)
    x0 = torch.randn(rows, 512, device="cuda", generator=g)
    x1, z1 = x0.clone(), torch.empty(rows, 512, dtype=torch.float16, device="cuda")
    y = torch.nn.functional.linear(a, w, b).contiguous()
    _lib.check(L.mapf_dropout_residual_layernorm(_p(x1), _p(y), _p(gamma), _p(beta), _p(z1), rows, 512, 1e-5, p,
                                                 seed, st))
    x2, z2 = x0.clone(), torch.full((rows, 512), float("nan"), dtype=torch.float16, device="cuda")
    _lib.check(L.mapf_linear512_residual_layernorm(_p(a), _p(w), _p(b), _p(x2), _p(gamma), _p(beta), _p(z2), rows,
                                                   1e-5, p, seed, st))
    torch.cuda.synchronize()
    assert torch.equal(x2 == x0, x1 == x0)            # the same elements dropped
    torch.testing.assert_close(x2, x1, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(z2.float(), z1.float(), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("C,H,B", [(6, 9, 37), (6, 11, 5), (7, 9, 130), (5, 9, 1)])
def test_conv_first_kernel_vs_torch(C, H, B):
    """mapf_conv_first_f32 (conv1 from the fp32 NCHW observation, one MFMA chunk) == autocast conv1
    + bias + ReLU to fp16 rounding; 0/1 observations as the env writes them and general values."""
    from mapf_amd import _lib
    g = torch.Generator(device="cuda").manual_seed(C * 100 + B)
    for obs in ((torch.rand(B, C, H, H, device="cuda", generator=g) < 0.3).float(),
                torch.randn(B, C, H, H, device="cuda", generator=g)):
        w = (torch.randn(128, C, 3, 3, device="cuda", generator=g) / (C * 9) ** 0.5).half()
        b = (torch.randn(128, device="cuda", generator=g) * 0.1).half()
        ref = torch.nn.functional.conv2d(obs.half().float(), w.float(), None, 1, 1).half()
        ref = torch.relu((ref.float() + b.float().view(1, -1, 1, 1)).half().float()).half()
        y = torch.full((B, 128, H, H), float("nan"), dtype=torch.float16, device="cuda").contiguous(
            memory_format=torch.channels_last)
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        w64 = torch.nn.functional.pad(w.reshape(128, -1), (0, 64 - C * 9)).contiguous()
        _lib.check(_lib.lib().mapf_conv_first_f32(_p(obs), _p(w64), _p(b), _p(y), B, C, H, H, 128, st))
        torch.cuda.synchronize()
        torch.testing.assert_close(y.float(), ref.float(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("bwd_form", [1, 0])
@pytest.mark.parametrize("n,first", [(17, False), (17, True), (5, False), (32, False), (9, True)])
def test_hip_attention_autograd_vs_sdpa(n, first, bwd_form):
    """_HipAttention (mapf_attention_f16 + mapf_attention_bwd_f16) == SDPA on the same fp16 q, k, v
    in fp32: output and dq / dk / dv, for the fused qkv tensor (one gradient) and for token 0's
    query against separate k / v (forward_first); both backward forms (mapf_attention_bwd_select:
    1 MFMA, the default; 0 VALU)."""
    from mapf_amd import _lib
    _lib.check(_lib.lib().mapf_attention_bwd_select(bwd_form))
    try:
        _attention_vs_sdpa(n, first)
    finally:
        _lib.check(_lib.lib().mapf_attention_bwd_select(1))


def _attention_vs_sdpa(n, first):
    from mapf_amd.net import _HipAttention
    g = torch.Generator(device="cuda").manual_seed(n + 100 * first)
    b, d, scale = 37, 512, 512 ** -0.5
    gout = torch.randn(b, 1 if first else n, d, device="cuda", generator=g).half()
    if first:
        qsrc = (torch.randn(b, d, device="cuda", generator=g) * 2).half().requires_grad_()
        kvsrc = (torch.randn(b, n, 2 * d, device="cuda", generator=g) * 2).half().requires_grad_()
        out = _HipAttention.apply(qsrc, kvsrc, 1, 0, 0, d, scale)
        out.backward(gout)
        q32 = qsrc.detach().float().view(b, 1, 16, 32).transpose(1, 2).requires_grad_()
        kv32 = kvsrc.detach().float().view(b, n, 2, 16, 32).permute(2, 0, 3, 1, 4)
        k32, v32 = kv32[0].clone().requires_grad_(), kv32[1].clone().requires_grad_()
    else:
        qsrc = (torch.randn(b, n, 3 * d, device="cuda", generator=g) * 2).half().requires_grad_()
        kvsrc = qsrc
        out = _HipAttention.apply(qsrc, qsrc, n, 0, d, 2 * d, scale)
        out.backward(gout)
        qkv32 = qsrc.detach().float().view(b, n, 3, 16, 32).permute(2, 0, 3, 1, 4)
        q32, k32, v32 = (t.clone().requires_grad_() for t in qkv32)
    ref = torch.nn.functional.scaled_dot_product_attention(q32, k32, v32, scale=scale)
    ref.backward(gout.float().view(b, -1, 16, 32).transpose(1, 2))
    torch.testing.assert_close(out.float(), ref.transpose(1, 2).reshape(b, -1, d), rtol=2e-2, atol=2e-2)
    gq = q32.grad.transpose(1, 2).reshape(b, -1, d)
    gk = k32.grad.transpose(1, 2).reshape(b, n, d)
    gv = v32.grad.transpose(1, 2).reshape(b, n, d)
    if first:
        got_q, got_k, got_v = qsrc.grad.view(b, 1, d), kvsrc.grad[..., :d], kvsrc.grad[..., d:]
    else:
        got_q, got_k, got_v = qsrc.grad[..., :d], qsrc.grad[..., d:2 * d], qsrc.grad[..., 2 * d:]
    for name, got, want in (("dq", got_q, gq), ("dk", got_k, gk), ("dv", got_v, gv)):
        assert torch.isfinite(got).all(), name
        torch.testing.assert_close(got.float(), want, rtol=3e-2, atol=3e-2, msg=name)


def test_training_forward_uses_hip_attention_and_matches_sdpa():
    """the training forward (autograd) with _HipAttention == with SDPA: each parameter's gradient
    within 2 % (relative norm) or 3x the spread of two SDPA runs (MIOpen's backward reduces in a
    run-dependent order)"""
    net = _net().eval()
    obs = (torch.rand(16, 8, 6, 9, 9, device="cuda") < 0.25).float()
    vec = torch.randn(16, 8, 4, device="cuda")
    grads = []
    for hip in (True, False, False):
        for m in net.modules():
            if hasattr(m, "hip_attention"):
                m.hip_attention = hip
        net.zero_grad()
        out = net(obs, vec)
        (out[1].float().sum() + out[0].float().pow(2).sum()).backward()
        grads.append([p.grad.detach().float().clone() for p in net.parameters() if p.grad is not None])
    for a, b, c in zip(*grads):
        nb = b.norm().item()
        if nb == 0:
            continue
        r_hip, r_spread = (a - b).norm().item() / nb, (c - b).norm().item() / nb
        assert r_hip <= max(2e-2, 3 * r_spread), (a.shape, r_hip, r_spread)


@pytest.mark.parametrize("rows", [1, 64, 127, 129, 1000, 17 * 97])
def test_linear512_row_tiles_are_bit_identical(rows):
    """mapf_linear512_select / _stages / _kdepth: 128-row workgroups (two 64-row tiles sharing each staged
    weight chunk), 2-, 3- and 4-stage K rings and 64-deep full-line K chunks give bit-identical outputs to
    64-row, 2-stage, 32-deep workgroups -- the same MFMA sequence per
    element, the same epilogues -- for the GELU, residual + LayerNorm, rows and tokens variants,
    ragged row counts included (the last workgroup's second tile partly or wholly past M)."""
    from mapf_amd import _lib
    L = _lib.lib()
    g = torch.Generator(device="cuda").manual_seed(rows)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    a = torch.randn(rows, 512, device="cuda", generator=g).half()
    w = (torch.randn(512, 512, device="cuda", generator=g) / 512 ** 0.5).half()
    b = (torch.randn(512, device="cuda", generator=g) * 0.1).half()
    gamma = 1 + 0.1 * torch.randn(512, device="cuda", generator=g)
    beta = 0.1 * torch.randn(512, device="cuda", generator=g)
    x0 = torch.randn(rows, 512, device="cuda", generator=g)
    Bt = max(1, rows // 17)
    A = torch.rand(Bt, 16, device="cuda", generator=g)
    VV = torch.randn(Bt, 512, device="cuda", generator=g).half()
    cls, pos = torch.randn(512, device="cuda", generator=g), torch.randn(17, 512, device="cuda", generator=g)
    at = torch.randn(Bt * 17, 512, device="cuda", generator=g).half()

    def run():
        out = torch.full((rows, 512), float("nan"), dtype=torch.float16, device="cuda")
        _lib.check(L.mapf_linear512_gelu_dropout(_p(a), _p(w), _p(b), _p(out), rows, 0.2, 7, st))
        x1, z1 = x0.clone(), torch.full((rows, 512), float("nan"), dtype=torch.float16, device="cuda")
        _lib.check(L.mapf_linear512_residual_layernorm(_p(a), _p(w), _p(b), _p(x1), _p(gamma), _p(beta), _p(z1), rows,
                                                       1e-5, 0.2, 8, st))
        x2, z2 = x0.clone(), torch.full((rows, 512), float("nan"), dtype=torch.float16, device="cuda")
        _lib.check(L.mapf_linear512_residual_layernorm_rows(_p(a), _p(w), _p(b), _p(x2), _p(gamma), _p(beta), _p(z2),
                                                            rows, 1e-5, 0.2, 9, 17, st))
        x3 = torch.full((Bt * 17, 512), float("nan"), device="cuda")
        z3 = torch.full((Bt * 17, 512), float("nan"), dtype=torch.float16, device="cuda")
        _lib.check(L.mapf_linear512_tokens_residual_layernorm(_p(at), _p(w), _p(b), _p(x3), _p(gamma), _p(beta), _p(z3),
                                                              Bt, 16, 1e-5, 0.2, 10, _p(A), _p(VV), _p(cls), _p(pos),
                                                              0.1, 11, st))
        torch.cuda.synchronize()
        return out, x1, z1, x2, z2, x3, z3

    forms = {}
    try:
        for mt in (1, 2):
            for stages in (2, 3, 4):              # mapf_linear512_stages: the K ring's depth
                _lib.check(L.mapf_linear512_select(mt))
                _lib.check(L.mapf_linear512_stages(stages))
                forms[(mt, stages)] = run()
            _lib.check(L.mapf_linear512_kdepth(64))   # full-line 64-deep K chunks (two stages)
            forms[(mt, "k64")] = run()
            _lib.check(L.mapf_linear512_kdepth(0))
    finally:
        _lib.check(L.mapf_linear512_select(0))
        _lib.check(L.mapf_linear512_stages(0))
        _lib.check(L.mapf_linear512_kdepth(0))
    ref = forms[(1, 2)]
    for form, outs in forms.items():
        for k, (u, v) in enumerate(zip(outs, ref)):
            assert torch.isfinite(u.float()).all(), (form, k)
            assert torch.equal(u, v), (form, k)
