"""The training forward's split weight-gradient linear (net._SplitKLinear, used by _train_linear for
the 17-token layers): under fp16 autocast its output, input gradient and bias gradient equal plain
F.linear's (the same GEMMs), and its weight gradient -- SPLIT (16) row chunks, fp32 partial products
summed in fp32, rounded to fp16 -- matches autograd's one-GEMM fp16 weight gradient to fp16
rounding (relative 2e-3 in norm, elementwise within a few fp16 ulps of the gradient's scale)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,n_in,n_out", [(34816, 512, 1536), (34816, 512, 512), (8192, 512, 1024)])
def test_split_weight_gradient_matches_autocast_linear(rows, n_in, n_out):
    from mapf_amd.net import _SplitKLinear, _train_linear
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    g = torch.Generator(device="cuda").manual_seed(rows + n_out)
    x0 = torch.randn(rows, n_in, device="cuda", generator=g)
    w0 = torch.randn(n_out, n_in, device="cuda", generator=g) / n_in ** 0.5
    b0 = torch.randn(n_out, device="cuda", generator=g) * 0.1
    gy = torch.randn(rows, n_out, device="cuda", generator=g).half()
    res = []
    for split in (True, False):
        x, w, b = (t.clone().requires_grad_(True) for t in (x0, w0, b0))
        with torch.autocast(device_type="cuda"):
            y = _train_linear(x, w, b) if split else F.linear(x, w, b)
        assert y.dtype == torch.float16
        y.backward(gy)
        res.append((y.detach(), x.grad, w.grad, b.grad))
    (ys, gxs, gws, gbs), (yp, gxp, gwp, gbp) = res
    assert torch.equal(ys, yp)
    torch.testing.assert_close(gxs, gxp, rtol=0, atol=0)
    torch.testing.assert_close(gbs, gbp, rtol=1e-3, atol=1e-3)
    assert gws.dtype == torch.float32 and torch.isfinite(gws).all()
    rel = ((gws - gwp).norm() / gwp.norm()).item()
    assert rel < 2e-3, rel
    scale = gwp.abs().max().item()
    assert (gws - gwp).abs().max().item() <= 4 * 2 ** -10 * scale
    print(f"rows {rows} {n_out}x{n_in}: weight-gradient rel diff {rel:.2e}; fp32 partials: "
          f"{_SplitKLinear.out_dtype_ok}")


@pytest.mark.parametrize("rows,strided", [(2048, False), (2048, True), (4095, False), (77, True), (1, False)])
def test_short_linear_matches_autocast_linear(rows, strided):
    """net._LinearBG (the training forward's short 2-D fp16 linears via _train_linear: torch's addmm and
    backward GEMMs, the bias gradient from mapf_colsum_f16's one-launch column sum) against autocast
    F.linear: output bit-identical, input / weight gradients equal (the same GEMMs), the bias gradient
    within fp16 rounding of another fp32 summation order.  strided: x is token 0 of a [rows, 17, 512]."""
    from mapf_amd.net import _LinearBG, _train_linear
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    g = torch.Generator(device="cuda").manual_seed(rows + strided)
    xs = torch.randn(rows, 17 if strided else 1, 512, device="cuda", generator=g).half()
    w0 = (torch.randn(512, 512, device="cuda", generator=g) / 512 ** 0.5).half()
    b0 = (torch.randn(512, device="cuda", generator=g) * 0.1).half()
    gy = torch.randn(rows, 512, device="cuda", generator=g).half()
    res, calls = [], []
    orig = _LinearBG.forward
    try:
        _LinearBG.forward = staticmethod(lambda ctx, *a: calls.append(1) or orig(ctx, *a))
        for own in (True, False):
            x3, w, b = (t.clone().requires_grad_(True) for t in (xs, w0, b0))
            x = x3[:, 0]
            with torch.autocast(device_type="cuda"):
                y = _train_linear(x, w, b) if own else F.linear(x, w, b)
            y.backward(gy)
            res.append((y.detach(), x3.grad, w.grad, b.grad))
    finally:
        _LinearBG.forward = orig
    assert calls == [1]
    assert torch.equal(res[0][0], res[1][0])
    torch.testing.assert_close(res[0][1], res[1][1], rtol=0, atol=0)
    torch.testing.assert_close(res[0][2], res[1][2], rtol=1e-3, atol=1e-3)
    ref = gy.double().sum(0)
    err_own = (res[0][3].double() - ref).abs().max().item()
    err_torch = (res[1][3].double() - ref).abs().max().item()
    ulp = 2 ** -10 * ref.abs().max().item()
    assert err_own <= max(err_torch, ulp), (err_own, err_torch, ulp)


@pytest.mark.parametrize("b", [512, 2048])
def test_qkv_first_matches_two_linears(b):
    """net._QKVFirst (the last block's token-0 query and all-token keys / values from one to_qkv weight, one
    backward) against the two _train_linear calls it replaces (a _LinearBG on x[:, 0] and a _SplitKLinear on
    x): q and kv bit-identical; kv's weight and both bias gradients equal (the same kernels); x's gradient and
    q's weight gradient within fp16 rounding (token 0's rows: one fused accumulate instead of an fp16 add)"""
    from mapf_amd.net import _QKVFirst, _train_linear
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    n, d = 17, 512
    g = torch.Generator(device="cuda").manual_seed(b)
    x0 = torch.randn(b, n, d, device="cuda", generator=g).half()
    w0 = (torch.randn(3 * d, d, device="cuda", generator=g) / d ** 0.5).half()
    b0 = (torch.randn(3 * d, device="cuda", generator=g) * 0.1).half()
    dq = torch.randn(b, d, device="cuda", generator=g).half()
    dkv = torch.randn(b, n, 2 * d, device="cuda", generator=g).half()
    res = []
    for fused in (True, False):
        x, w, bb = (t.clone().requires_grad_(True) for t in (x0, w0, b0))
        with torch.autocast(device_type="cuda"):
            if fused:
                q, kv = _QKVFirst.apply(x, w, bb)
            else:
                q, kv = _train_linear(x[:, 0], w[:d], bb[:d]), _train_linear(x, w[d:], bb[d:])
        torch.autograd.backward([q, kv], [dq, dkv])
        res.append((q.detach(), kv.detach(), x.grad, w.grad, bb.grad))
    (qf, kvf, gxf, gwf, gbf), (qr, kvr, gxr, gwr, gbr) = res
    assert torch.equal(qf, qr) and torch.equal(kvf, kvr)
    assert torch.equal(gwf[d:], gwr[d:]) and torch.equal(gbf, gbr)
    for a, r in ((gxf, gxr), (gwf[:d], gwr[:d])):
        rel = ((a.float() - r.float()).norm() / r.float().norm()).item()
        assert rel < 2e-3, rel
    assert torch.equal(gxf[:, 1:], gxr[:, 1:])


@pytest.mark.parametrize("rows,C", [(0, 512), (1, 512), (63, 8), (2048, 512), (8192, 1536), (8193, 512), (300, 12)])
def test_colsum_f16_matches_fp64(rows, C):
    """mapf_colsum_f16 (one launch for rows <= 8192 with C % 8 == 0, partials + sum otherwise) against an
    fp64 column sum: within one fp16 rounding of the fp32 sum"""
    import ctypes
    from mapf_amd import _lib
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    g = torch.Generator(device="cuda").manual_seed(rows + C)
    x = torch.randn(max(rows, 1), C, device="cuda", generator=g).half()[:rows]
    out = torch.full((C,), 7.0, dtype=torch.float16, device="cuda")
    work = torch.empty(512 * C, dtype=torch.float32, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(_lib.lib().mapf_colsum_f16(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                          ctypes.c_void_p(work.data_ptr()), rows, C, st))
    torch.cuda.synchronize()
    ref = x.double().sum(0)
    tol = 2 ** -10 * ref.abs().clamp_min(1.0) + 1e-6 * rows
    assert ((out.double() - ref).abs() <= tol).all(), (out.double() - ref).abs().max().item()


@pytest.mark.parametrize("rows", [34816, 2048, 35, 1])
def test_hip_layernorm_matches_autocast_layernorm(rows):
    """net._HipLayerNorm (mapf_layernorm_f16 forward, mapf_layernorm_bwd_f16 backward) against torch's
    LayerNorm under autocast followed by the fp16 cast the next linear makes: z within one fp16 ulp,
    dx / dgamma / dbeta to fp32 rounding of the reductions."""
    from mapf_amd.net import _HipLayerNorm
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    g = torch.Generator(device="cuda").manual_seed(rows)
    x0 = torch.randn(rows, 512, device="cuda", generator=g) * 2 + 0.5
    w0 = 1 + 0.1 * torch.randn(512, device="cuda", generator=g)
    b0 = 0.1 * torch.randn(512, device="cuda", generator=g)
    dz = torch.randn(rows, 512, device="cuda", generator=g).half()
    dres = torch.randn(rows, 512, device="cuda", generator=g)
    out = []
    for hip in (True, False):
        x, w, b = (t.clone().requires_grad_(True) for t in (x0, w0, b0))
        with torch.autocast(device_type="cuda"):
            if hip:
                z, res = _HipLayerNorm.apply(x, w, b, 1e-5)
            else:
                z, res = F.layer_norm(x, (512,), w, b, 1e-5).half(), x
        assert z.dtype == torch.float16
        # the PreNorm's residual: its gradient (dres) reaches x beside the LayerNorm's
        torch.autograd.backward([z, res], [dz, dres])
        out.append((z.detach(), x.grad, w.grad, b.grad))
    (zh, dxh, dwh, dbh), (zt, dxt, dwt, dbt) = out
    torch.testing.assert_close(zh.float(), zt.float(), rtol=2e-3, atol=2e-3)
    torch.testing.assert_close(dxh, dxt, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dwh, dwt, rtol=1e-4, atol=1e-3 * max(1.0, rows ** 0.5 / 10))
    torch.testing.assert_close(dbh, dbt, rtol=1e-4, atol=1e-3 * max(1.0, rows ** 0.5 / 10))


@pytest.mark.parametrize("cin,cout,ks,pad,hw", [(128, 128, 3, 1, 9), (128, 256, 2, 1, 4), (256, 500, 3, 0, 3)])
def test_conv_bias_relu_matches_autocast_conv_relu(cin, cout, ks, pad, hw):
    """SCRIMPNet._conv_relu's GPU training form (conv without bias, then net._BiasReLU: in-place bias +
    ReLU, mapf_relu_bias_bwd_f16 backward) against (a) the same arithmetic in torch ops -- fp16 conv,
    fp32 bias add rounded to fp16, ReLU -- to fp16 tolerance, and (b) the reference form F.relu(conv(x))
    under autocast: its forward is checked elementwise against the double-rounding bound below (round 6,
    measured: bit-identical -- torch adds the bias to MIOpen's fp16 output the same way); its gradients
    within 2e-2 (MIOpen's backward of the biased convolution reduces in another order)."""
    import torch.nn.functional as F_
    from mapf_amd.net import SCRIMPNet
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    torch.manual_seed(cout + ks)
    conv = torch.nn.Conv2d(cin, cout, ks, 1, pad).cuda().to(memory_format=torch.channels_last)
    with torch.no_grad():
        conv.bias.normal_(0, 0.1)
    x0 = torch.randn(64, cin, hw, hw, device="cuda").contiguous(memory_format=torch.channels_last)
    net = SCRIMPNet(numChannel=6, num_agents=8, fov=9)
    forms = {
        "hip": lambda x: net._conv_relu(x, conv),
        "same": lambda x: torch.relu((F_.conv2d(x, conv.weight, None, 1, pad).float() +
                                      conv.bias.half().float().view(-1, 1, 1)).half()),
        "torch": lambda x: torch.relu(conv(x)),
    }
    res = {}
    old = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False   # one MIOpen algorithm
    try:
        for name, fn in forms.items():
            res[name] = _run_form(fn, conv, x0)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = old
    torch.testing.assert_close(res["hip"][0], res["same"][0], rtol=0, atol=0)
    for ref, tol in (("same", 2e-3), ("torch", 2e-2)):
        for k, (a, b) in enumerate(zip(res["hip"][1:], res[ref][1:])):
            rel = ((a - b).norm() / b.norm()).item()
            assert rel < tol, (ref, k, rel)
    # the forward against the reference form F.relu(conv(x)) with the conv's own bias:
    # the two differ only in where the bias meets the fp16 rounding -- fp16(fp16(acc) + b) here -- so
    # elementwise |hip - torch| <= 1 ulp of the pre-bias output + 1 ulp of the result (fp16 ulps;
    # 2^-24 below the normal range), which also covers a last-bit difference between MIOpen's
    # solvers for the biased and the unbiased convolution
    with torch.no_grad(), torch.autocast(device_type="cuda"):
        pre = F_.conv2d(x0, conv.weight, None, 1, pad).float()
    hip, ref_y = res["hip"][0], res["torch"][0]
    bound = _ulp16(pre.abs()) + _ulp16(torch.maximum(hip.abs(), ref_y.abs()))
    excess = ((hip - ref_y).abs() - bound).max().item()
    same = (hip == ref_y).float().mean().item()
    print(f"conv {cin}->{cout} k{ks}: forward vs F.relu(conv(x)): {same:.4%} bit-identical, "
          f"max |diff| {(hip - ref_y).abs().max().item():.3e}")
    assert excess <= 0, excess


def _ulp16(v):
    """the fp16 unit in the last place at magnitude v (fp32 tensor)"""
    _, e = torch.frexp(v)
    return torch.where(v >= 2.0 ** -14, torch.ldexp(torch.ones_like(v), e - 11), torch.full_like(v, 2.0 ** -24))


def _run_form(fn, conv, x0):
    conv.zero_grad()
    x = x0.clone().requires_grad_(True)
    with torch.autocast(device_type="cuda"):
        y = fn(x)
    gy = torch.randn(y.shape, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1)).half()
    y.backward(gy.contiguous(memory_format=torch.channels_last))
    return y.detach().float(), x.grad.float(), conv.weight.grad.clone(), conv.bias.grad.clone()


@pytest.mark.parametrize("cin,cout,ks,pad,hw", [(128, 128, 3, 1, 9), (256, 256, 2, 1, 6), (128, 128, 3, 1, 8)])
def test_conv_bias_relu_pool_matches_autocast(cin, cout, ks, pad, hw):
    """SCRIMPNet._conv_relu_pool's GPU training form (net._BiasReLUPool: mapf_nhwc_bias_relu_pool2 +
    mapf_relu_bias_pool_bwd_f16) against the same arithmetic in torch ops (fp16 conv, fp32 bias add
    rounded to fp16, ReLU, MaxPool2d(2): torch's argmax routing) -- outputs bit-identical, gradients to
    fp16 tolerance -- and against pool(relu(conv(x))) under autocast (2e-2, see the unpooled test).
    Odd sizes (9x9, 7x7) leave a row and a column no window covers: their gradient must be 0."""
    import torch.nn.functional as F_
    from mapf_amd.net import SCRIMPNet
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    torch.manual_seed(cout + ks + hw)
    conv = torch.nn.Conv2d(cin, cout, ks, 1, pad).cuda().to(memory_format=torch.channels_last)
    pool = torch.nn.MaxPool2d(2)
    with torch.no_grad():
        conv.bias.normal_(0, 0.1)
    x0 = torch.randn(64, cin, hw, hw, device="cuda").contiguous(memory_format=torch.channels_last)
    net = SCRIMPNet(numChannel=6, num_agents=8, fov=9)
    forms = {
        "hip": lambda x: net._conv_relu_pool(x, conv, pool),
        "same": lambda x: pool(torch.relu((F_.conv2d(x, conv.weight, None, 1, pad).float() +
                                           conv.bias.half().float().view(-1, 1, 1)).half())),
        "torch": lambda x: pool(torch.relu(conv(x))),
    }
    res = {}
    old = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        for name, fn in forms.items():
            res[name] = _run_form(fn, conv, x0)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = old
    torch.testing.assert_close(res["hip"][0], res["same"][0], rtol=0, atol=0)
    for ref, tol in (("same", 2e-3), ("torch", 2e-2)):
        for k, (a, b) in enumerate(zip(res["hip"][1:], res[ref][1:])):
            rel = ((a - b).norm() / b.norm()).item()
            assert rel < tol, (ref, k, rel)


@pytest.mark.parametrize("cin,cout,ks,pad,hw,b", [(128, 128, 3, 1, 9, 96), (128, 256, 2, 1, 4, 64),
                                                  (256, 128, 2, 0, 5, 40), (256, 256, 2, 1, 5, 64),
                                                  (256, 256, 2, 1, 6, 33)])
def test_hip_conv_matches_miopen_conv(cin, cout, ks, pad, hw, b):
    """net._HipConv (the training forward's conv on mapf_conv_nhwc_f16; data gradient by the same kernel
    over the flipped, transposed weight -- conv2's is the 256 -> 128 2x2 form, also run forward here --
    weight gradient MIOpen's) against F.conv2d on the same fp16 NHWC tensors, MIOpen's
    deterministic algorithms: output and data gradient to fp16 rounding of another fp32 summation order
    (2e-3 relative in norm, elementwise 1e-2 of the tensor's scale), weight gradient equal (the same call)."""
    from mapf_amd.net import SCRIMPNet, _HipConv
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    g = torch.Generator(device="cuda").manual_seed(cin + cout + hw)
    cl = torch.channels_last
    x0 = torch.randn(b, cin, hw, hw, device="cuda", generator=g).half().contiguous(memory_format=cl)
    w0 = (torch.randn(cout, cin, ks, ks, device="cuda", generator=g) / (cin * ks * ks) ** 0.5).half().contiguous(
        memory_format=cl)
    ho = hw + 2 * pad - ks + 1
    gy = torch.randn(b, cout, ho, ho, device="cuda", generator=g).half().contiguous(memory_format=cl)
    old = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    res = []
    try:
        for hip in (True, False):
            x, w = x0.clone().requires_grad_(True), w0.clone().requires_grad_(True)
            y = _HipConv.apply(x, w, pad) if hip else torch.nn.functional.conv2d(x, w, None, 1, pad)
            y.backward(gy)
            res.append((y.detach().float(), x.grad.float(), w.grad.float()))
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = old
    for k, (a, r) in enumerate(zip(*res)):
        rel = ((a - r).norm() / r.norm()).item()
        err = (a - r).abs().max().item() / r.abs().max().item()
        print(f"conv {cin}->{cout} k{ks} {hw}x{hw}: {('y', 'dx', 'dw')[k]} relative {rel:.2e}, max {err:.2e}"
              f"{'' if k != 1 else (' (own kernel)' if (cout, cin, ks) in SCRIMPNet._OWN_CONV else ' (MIOpen)')}")
        assert rel < 2e-3 and err < 1e-2, (k, rel, err)


def test_training_forward_convs_take_hip_conv():
    """SCRIMPNet's training forward (GPU, autocast, grad) runs conv1a .. conv2b through _HipConv
    (conv1 from the 6-channel observation and conv3 stay MIOpen's: shapes the kernel does not have)"""
    from mapf_amd.net import SCRIMPNet, _HipConv
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    net = SCRIMPNet(numChannel=6, num_agents=8, fov=9).cuda().to(memory_format=torch.channels_last)
    calls, flipped = [], []
    orig = _HipConv.forward
    try:
        _HipConv.forward = staticmethod(
            lambda ctx, x, w, pad, b=None, wt=None: calls.append((tuple(w.shape), b is not None))
            or flipped.append(wt is not None and torch.equal(wt, w.flip(2, 3).transpose(0, 1)))
            or orig(ctx, x, w, pad, b, wt))
        obs = (torch.rand(4, 8, 6, 9, 9, device="cuda") < 0.3).float()
        out = net(obs, torch.randn(4, 8, 4, device="cuda"))
        out[1].float().sum().backward()
    finally:
        _HipConv.forward = orig
    # the un-pooled layers take the bias + ReLU in the conv's epilogue (SCRIMPNet.conv_bias_relu)
    assert calls == [((128, 128, 3, 3), True), ((128, 128, 3, 3), False), ((256, 128, 2, 2), True),
                     ((256, 256, 2, 2), True), ((256, 256, 2, 2), False)], calls
    # each carries its flipped, transposed weight from _CastParams' launch (mapf_cast_f32_to_f16_multi_flip)
    assert flipped == [True] * 5, flipped


@pytest.mark.parametrize("cin,cout,ks,pad,hw,b", [(128, 128, 3, 1, 9, 96), (128, 256, 2, 1, 4, 64),
                                                  (256, 256, 2, 1, 5, 64)])
def test_hip_conv_bias_relu_epilogue_equals_two_passes(cin, cout, ks, pad, hw, b):
    """_HipConv with the bias (bias + ReLU in the conv kernel's epilogue; backward: mapf_relu_bias_bwd_f16
    then the conv's own gradients) == _BiasReLU over _HipConv's raw output: output, data, weight and bias
    gradients bit-identical (the same roundings: fp16(fp16(acc) + b), the same backward kernels)"""
    from mapf_amd.net import _BiasReLU, _HipConv
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    g = torch.Generator(device="cuda").manual_seed(3 * cin + cout)
    cl = torch.channels_last
    x0 = torch.randn(b, cin, hw, hw, device="cuda", generator=g).half().contiguous(memory_format=cl)
    w0 = (torch.randn(cout, cin, ks, ks, device="cuda", generator=g) / (cin * ks * ks) ** 0.5).half().contiguous(
        memory_format=cl)
    b0 = (torch.randn(cout, device="cuda", generator=g) * 0.3).half()
    ho = hw + 2 * pad - ks + 1
    gy = torch.randn(b, cout, ho, ho, device="cuda", generator=g).half().contiguous(memory_format=cl)
    old = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    res = []
    try:
        for fused in (True, False):
            x, w, bb = (t.clone().requires_grad_(True) for t in (x0, w0, b0))
            y = _HipConv.apply(x, w, pad, bb) if fused else _BiasReLU.apply(_HipConv.apply(x, w, pad), bb)
            y.backward(gy)
            res.append((y.detach(), x.grad, w.grad, bb.grad))
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = old
    assert (res[0][0] == 0).float().mean().item() > 0.2          # the ReLU clamps a good share
    for k, (a, r) in enumerate(zip(*res)):
        assert torch.equal(a, r), ("y", "dx", "dw", "db")[k]


def test_conv3_as_gemm_matches_conv():
    """SCRIMPNet._conv_nobias on conv3 (3x3 over a 3x3 input, no padding: one output pixel) is a GEMM over
    the channels_last views, K ordered (ky, kx, c): output, data and weight gradients match F.conv2d's
    to fp16 rounding of another summation order"""
    from mapf_amd.net import SCRIMPNet
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    g = torch.Generator(device="cuda").manual_seed(9)
    cl = torch.channels_last
    net = SCRIMPNet(numChannel=6, num_agents=8, fov=9)
    x0 = torch.randn(96, 256, 3, 3, device="cuda", generator=g).half().contiguous(memory_format=cl)
    w0 = (torch.randn(500, 256, 3, 3, device="cuda", generator=g) / 48).half().contiguous(memory_format=cl)
    gy = torch.randn(96, 500, 1, 1, device="cuda", generator=g).half()
    res = []
    for gemm in (True, False):
        x, w = x0.clone().requires_grad_(True), w0.clone().requires_grad_(True)
        mm = type("M", (), {"weight": w, "padding": (0, 0), "stride": (1, 1), "dilation": (1, 1), "groups": 1})()
        y = net._conv_nobias(x, mm) if gemm else torch.nn.functional.conv2d(x, w, None, 1, 0)
        y.backward(gy)
        res.append((y.detach().float().reshape(96, 500), x.grad.float(), w.grad.float()))
    for k, (a, r) in enumerate(zip(*res)):
        rel = ((a - r).norm() / r.norm()).item()
        print(f"conv3 as GEMM: {('y', 'dx', 'dw')[k]} relative {rel:.2e}")
        assert rel < 2e-3, (k, rel)


def _seed(v=12345):
    return torch.tensor([v], dtype=torch.int64, device="cuda")


@pytest.mark.parametrize("p", [0.0, 0.2])
@pytest.mark.parametrize("strided", [False, True])
def test_drop_res_ln_matches_torch_chain(p, strided):
    """net._DropResLN (x = res + dropout(y), z = fp16(LN(x)); backward: LN's with the residual gradient and
    the dropped branch's fp16 gradient) against the unfused chain -- torch add of the (masked, scaled)
    fp16 branch, then _HipLayerNorm -- given the SAME mask: p = 0 bit-identical forward and gradients;
    p = 0.2: the mask the kernel drew is read back from its output (x - res == 0 exactly where dropped)
    and fed to the chain; keep rate 0.8 +- 0.01.  strided: res is token 0 of a [b, 17, 512] stream."""
    from mapf_amd.net import _DropResLN, _HipLayerNorm
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    g = torch.Generator(device="cuda").manual_seed(3)
    b = 640
    base = torch.randn(b, 17, 512, device="cuda", generator=g) * 2
    res0 = base[:, :1] if strided else base[:, :5]
    y0 = torch.randn(res0.shape, device="cuda", generator=g).half()
    w0, b0 = 1 + 0.1 * torch.randn(512, device="cuda", generator=g), 0.1 * torch.randn(512, device="cuda", generator=g)
    dz = torch.randn(res0.shape, device="cuda", generator=g).half()
    dx_down = torch.randn(res0.shape, device="cuda", generator=g)
    out = {}
    for fused in (True, False):
        res, y, w, bb = (t.detach().clone().requires_grad_(True) for t in (res0, y0, w0, b0))
        if fused:
            z, x = _DropResLN.apply(res, y, w, bb, 1e-5, p, _seed(), 3)
            keep = (x.detach() - res0) != 0
            keep |= y0.float() == 0
            out["keep"] = keep
        else:
            k = out["keep"]
            ydrop = torch.where(k, y * (1.0 / (1.0 - p)), torch.zeros_like(y)) if p > 0 else y
            x = res + ydrop
            z, x = _HipLayerNorm.apply(x, w, bb, 1e-5)
        torch.autograd.backward([z, x], [dz, dx_down])
        out[fused] = (z.detach().float(), x.detach(), res.grad, y.grad.float(), w.grad, bb.grad)
    if p > 0:
        rate = out["keep"].float().mean().item()
        assert abs(rate - (1 - p)) < 0.01, rate
    for k, (a, r) in enumerate(zip(out[True], out[False])):
        if p == 0:
            assert torch.equal(a, r), k
        else:
            torch.testing.assert_close(a, r, rtol=2e-3, atol=2e-3, msg=str(k))
    assert torch.equal(out[True][3] == 0, out[False][3] == 0) or p == 0     # the gradient dropped where the forward did


@pytest.mark.parametrize("p", [0.0, 0.2])
@pytest.mark.parametrize("B", [96, 2048, 301])
def test_tokens_ln_matches_torch_chain(p, B):
    """net._TokensLN (tokens + dropout + the first PreNorm, mapf_tokens_layernorm_train; backward
    mapf_layernorm_bwd_f16 + mapf_tokens_train_bwd) against SCRIMPNet.forward's torch chain -- A * VV, cat
    with cls, + pos, dropout, then _HipLayerNorm -- given the SAME mask (read back from the kernel's x:
    exactly 0 where dropped): x and z bit-identical; gradients of A, VV, cls, pos, gamma, beta within fp32
    summation order (1e-5 relative in norm; dVV, fp16, within 1e-3); keep rate 1 - p +- 0.01.  B = 301: a
    ragged last block of the backward's per-block sums."""
    from mapf_amd.net import _HipLayerNorm, _TokensLN
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    g = torch.Generator(device="cuda").manual_seed(B + int(10 * p))
    A0 = torch.rand(B, 16, device="cuda", generator=g) + 0.5
    VV0 = torch.randn(B, 512, device="cuda", generator=g).half()
    cls0 = torch.randn(1, 1, 512, device="cuda", generator=g)
    pos0 = torch.randn(1, 17, 512, device="cuda", generator=g)
    w0 = 1 + 0.1 * torch.randn(512, device="cuda", generator=g)
    b0 = 0.1 * torch.randn(512, device="cuda", generator=g)
    dz = torch.randn(B, 17, 512, device="cuda", generator=g).half()
    dres = torch.randn(B, 17, 512, device="cuda", generator=g)
    res = []
    for fused in (True, False):
        A, VV, cls, pos, w, b = (t.clone().requires_grad_(True) for t in (A0, VV0, cls0, pos0, w0, b0))
        if fused:
            z, x = _TokensLN.apply(A, VV, cls, pos, w, b, 1e-5, p, _seed(7), 32)
            keep = x != 0
        else:
            T = A.unsqueeze(2) * VV.unsqueeze(1)
            xt = torch.cat((cls.expand(B, -1, -1), T), dim=1) + pos
            xt = xt * keep * (1.0 / (1.0 - p)) if p > 0 else xt
            z, x = _HipLayerNorm.apply(xt, w, b, 1e-5)
        (z.float() * dz.float()).sum().add_((x * dres).sum()).backward()
        res.append((x.detach(), z.detach(), A.grad, VV.grad, cls.grad, pos.grad, w.grad, b.grad))
    if p > 0:
        assert abs(keep.float().mean().item() - (1 - p)) < 0.01
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    for k, (a, r) in enumerate(zip(res[0][2:], res[1][2:])):
        rel = ((a.float() - r.float()).norm() / r.float().norm()).item()
        assert rel < (1e-3 if k == 1 else 1e-5), (("A", "VV", "cls", "pos", "gamma", "beta")[k], rel)


def test_training_forward_takes_tokens_ln():
    """SCRIMPNet's training forward (GPU, autocast, grad) builds the tokens through _TokensLN, and with
    SCRIMPNet.fused_tokens off through torch's chain: outputs within fp16 rounding, every gradient within
    2e-2 (relative norm) -- dropout off (eval), deterministic convolutions"""
    from mapf_amd.net import SCRIMPNet, _TokensLN
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    torch.manual_seed(1)
    net = SCRIMPNet(numChannel=6, num_agents=8, fov=9).cuda().to(memory_format=torch.channels_last)
    net.eval()
    obs = (torch.rand(16, 8, 6, 9, 9, device="cuda") < 0.3).float()
    vec = torch.randn(16, 8, 4, device="cuda")
    calls, res = [], []
    orig = _TokensLN.forward
    old = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        _TokensLN.forward = staticmethod(lambda ctx, *a: calls.append(a[0].shape) or orig(ctx, *a))
        for fused in (True, False):
            SCRIMPNet.fused_tokens = fused
            net.zero_grad()
            out = net(obs, vec)
            (out[1].float().sum() + out[0].float().pow(2).sum()).backward()
            res.append(([o.detach().float() for o in out], [p.grad.detach().clone() for p in net.parameters()
                                                              if p.grad is not None]))
    finally:
        SCRIMPNet.fused_tokens = True
        _TokensLN.forward = orig
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = old
    assert calls == [torch.Size([128, 16])], calls
    for a, r in zip(res[0][0], res[1][0]):
        torch.testing.assert_close(a, r, rtol=1e-2, atol=4e-3)
    assert len(res[0][1]) == len(res[1][1])
    for a, r in zip(res[0][1], res[1][1]):
        rel = ((a - r).norm() / r.norm().clamp_min(1e-30)).item()
        assert rel < 2e-2, rel


@pytest.mark.parametrize("p", [0.0, 0.2])
def test_gelu_dropout_matches_torch(p):
    """net._GeluDropout against F.gelu then the same mask (read back from the output) on fp16: p = 0
    bit-identical forward and gradient (torch's fp16 GELU and GeluBackward compute in fp32); p = 0.2
    to fp16 rounding (torch scales after the GELU's rounding the same way), keep rate 0.8 +- 0.01."""
    from mapf_amd.net import _GeluDropout
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    g = torch.Generator(device="cuda").manual_seed(4)
    h0 = (torch.randn(4096, 512, device="cuda", generator=g) * 2).half()
    gy = torch.randn(4096, 512, device="cuda", generator=g).half()
    h = h0.clone().requires_grad_(True)
    y = _GeluDropout.apply(h, p, _seed(77), 5)
    y.backward(gy)
    h2 = h0.clone().requires_grad_(True)
    ref = torch.nn.functional.gelu(h2)
    keep = (y.detach() != 0) | (ref.detach() == 0)
    if p > 0:
        assert abs(keep.float().mean().item() - (1 - p)) < 0.01
        ref = torch.where(keep, ref * (1.0 / (1.0 - p)), torch.zeros_like(ref))
    ref.backward(gy)
    if p == 0:
        same_y = (y == ref.detach()).float().mean().item()
        same_g = (h.grad == h2.grad).float().mean().item()
        print(f"gelu: forward {same_y:.5%} bit-identical to torch's, gradient {same_g:.5%}")
        # torch's exp / erf builds may round differently in the last bit: within one fp16 ulp
        torch.testing.assert_close(y.float(), ref.detach().float(), rtol=1e-3, atol=1e-5)
        torch.testing.assert_close(h.grad.float(), h2.grad.float(), rtol=1e-3, atol=1e-5)
    else:
        torch.testing.assert_close(y.float(), ref.detach().float(), rtol=2e-3, atol=2e-3)
        torch.testing.assert_close(h.grad.float(), h2.grad.float(), rtol=2e-3, atol=2e-3)


def test_training_forward_fused_residuals_equal_unfused():
    """SCRIMPNet's training forward with _Encoder.fused_train (every LayerNorm-feeding residual a
    _DropResLN, the MLP's GELU + dropout a _GeluDropout) == the unfused forward, dropout off: outputs
    within fp16 rounding (1e-2 relative) and every parameter's gradient within 2e-2 (relative norm); and with
    dropout on, two forwards draw different masks (the device seed counter moves)."""
    from mapf_amd.net import SCRIMPNet, _Encoder
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    torch.manual_seed(0)
    net = SCRIMPNet(numChannel=6, num_agents=8, fov=9).cuda().to(memory_format=torch.channels_last)
    obs = (torch.rand(16, 8, 6, 9, 9, device="cuda") < 0.3).float()
    vec = torch.randn(16, 8, 4, device="cuda")
    net.eval()
    res = []
    old = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False   # conv1 / conv3: MIOpen's
    try:
        for fused in (True, False):
            _Encoder.fused_train = fused
            net.zero_grad()
            out = net(obs, vec)
            (out[1].float().sum() + out[0].float().pow(2).sum()).backward()
            res.append(([o.detach().float() for o in out], [p.grad.detach().clone() for p in net.parameters()
                                                              if p.grad is not None]))
    finally:
        _Encoder.fused_train = True
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = old
    # the same operations and rounding points; torch's GELU kernels may round their exp / erf in the last
    # bit differently (test_gelu_dropout_matches_torch), which moves the outputs by fp16 ulps; those ulps pass
    # through two transformer layers and the LSTM, so a near-zero output can sit 2-4 ulps (of 1.0) away:
    # elementwise 4e-3 absolute, and the whole output within 5e-3 relative norm
    for a, r in zip(res[0][0], res[1][0]):
        rel = ((a - r).norm() / r.norm().clamp_min(1e-30)).item()
        print(f"output: max |diff| {(a - r).abs().max().item():.3e}, bit-identical {(a == r).float().mean().item():.4%}, "
              f"rel norm {rel:.2e}")
        torch.testing.assert_close(a, r, rtol=1e-2, atol=4e-3)
        assert rel < 5e-3, rel
    assert len(res[0][1]) == len(res[1][1])
    for a, r in zip(res[0][1], res[1][1]):
        rel = ((a - r).norm() / r.norm().clamp_min(1e-30)).item()
        assert rel < 2e-2, rel
    net.train()
    with torch.no_grad():
        net.dropout.p = 0.0                                  # torch's own dropout sites off: only the fused ones draw
        net.transformer.layers[-1][1].fn.fn.do2.p = 0.0
    outs = [net(obs, vec)[1].detach() for _ in range(2)]
    assert not torch.equal(outs[0], outs[1])
