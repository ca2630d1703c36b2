"""SCRIMPNet policy/value network, state_dict-compatible with the reference.

Architecture and parameter names follow net.py:38-155 and transformer.py:1-100
of the reference so that a reference checkpoint (`torch.save({"model": ...})`,
driver.py:182-193) loads with `load_state_dict` unchanged:

  obs [.., C, F, F] -> 3x conv3x3(128) -> maxpool -> 3x conv2x2(256) -> maxpool
  -> conv3x3(500) -> flatten ++ fc(vector 4 -> 12) -> 512 -> residual MLP
  -> 16-token tokeniser + cls token + positional embedding
  -> 2 pre-norm transformer blocks (16 heads, MLP 512, GELU, dropout 0.2)
  -> cls -> nn_same applied twice -> policy(5) / value / cost value / blocking

The tokeniser keeps the reference's exact arithmetic: its einsum
'bij,zjk->bik' SUMS over the 8 token matrices and its softmax runs over a
length-1 axis, so every token equals the summed-V projection (kept literally).
Runs under torch autocast like the reference (net.py:101).
"""
import ctypes
import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .config import EnvParameters, NetParameters


def _xavier_like(module):
    """weights_init (net.py:18-35): uniform(+-sqrt(6/(fan_in+fan_out))), zero bias."""
    name = module.__class__.__name__
    if name.find("Conv") != -1:
        shape = list(module.weight.data.size())
        fan_in = np.prod(shape[1:4])
        fan_out = np.prod(shape[2:4]) * shape[0]
        bound = math.sqrt(6.0 / (fan_in + fan_out))
        module.weight.data.uniform_(-bound, bound)
        module.bias.data.fill_(0)
    elif name.find("Linear") != -1:
        fan_out, fan_in = module.weight.data.size()
        bound = math.sqrt(6.0 / (fan_in + fan_out))
        module.weight.data.uniform_(-bound, bound)
        if module.bias is not None:
            module.bias.data.fill_(0)


class _HipLayerNorm(torch.autograd.Function):
    """fp16(LayerNorm(x)) of the TRAINING forward under autocast -- what the next fp16 linear reads
    (autocast runs layer_norm in fp32 and casts at the linear): the forward is mapf_layernorm_f16
    (the acting path's kernel), the backward mapf_layernorm_bwd_f16 (dx in fp32, dgamma / dbeta
    summed over the rows).  Replaces torch's LayerNorm forward, its two backward kernels and the
    fp32 <-> fp16 casts on either side (tools/profile_update.py).  x: fp32 [.., 512]."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        """returns (z, x viewed): the PreNorm adds the second output back as its residual, so the
        residual path's gradient arrives in backward and is added to dx by the kernel"""
        from . import _lib
        ctx.set_materialize_grads(False)
        x2 = x.reshape(-1, 512)
        if x2.stride(0) % 4 or x2.stride(1) != 1:
            x2 = x2.contiguous()
        rows = x2.shape[0]
        z = torch.empty(rows, 512, dtype=torch.float16, device=x.device)
        st = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
        _lib.check(_lib.lib().mapf_layernorm_f16(ctypes.c_void_p(x2.data_ptr()), x2.stride(0),
                                                 ctypes.c_void_p(weight.data_ptr()), ctypes.c_void_p(bias.data_ptr()),
                                                 ctypes.c_void_p(z.data_ptr()), rows, 512, float(eps), st))
        ctx.save_for_backward(x2, weight)
        ctx.eps, ctx.shape = float(eps), x.shape
        return z.view(*x.shape[:-1], 512), x.view_as(x)

    @staticmethod
    def backward(ctx, dz, dres):
        from . import _lib
        x2, weight = ctx.saved_tensors
        rows = x2.shape[0]
        if dz is None:
            dz = torch.zeros(rows, 512, dtype=torch.float16, device=x2.device)
        dz = dz.reshape(rows, 512).to(torch.float16).contiguous()
        if dres is not None:
            dres = dres.reshape(rows, 512).to(torch.float32).contiguous()
        dx = torch.empty(rows, 512, dtype=torch.float32, device=dz.device)
        dg = torch.empty(512, dtype=torch.float32, device=dz.device)
        db = torch.empty(512, dtype=torch.float32, device=dz.device)
        work = torch.empty(2 * 512 * 512, dtype=torch.float32, device=dz.device)
        st = ctypes.c_void_p(torch.cuda.current_stream(dz.device).cuda_stream)
        p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        _lib.check(_lib.lib().mapf_layernorm_bwd_f16(p(x2), x2.stride(0), p(weight), p(dz),
                                                     None if dres is None else p(dres), p(dx), p(dg), p(db),
                                                     p(work), rows, 512, ctx.eps, st))
        return dx.view(ctx.shape), dg, db, None


def _cast_multi(fn, srcs, dsts, stream):
    from . import _lib
    k = len(srcs)
    arr = lambda ts: (ctypes.c_void_p * k)(*[t.data_ptr() for t in ts])  # noqa: E731
    _lib.check(fn(arr(srcs), arr(dsts), (ctypes.c_int64 * k)(*[t.numel() for t in srcs]), k, stream))


class _CastParams(torch.autograd.Function):
    """fp16 copies of fp32 parameters in ONE launch (mapf_cast_f32_to_f16_multi), their gradients back
    to fp32 in one (mapf_cast_f16_to_f32_multi): what autocast's per-weight casts and their
    ToCopyBackward nodes compute (round to nearest even; exact), in 2 launches instead of ~90 per
    update (tools/profile_update.py)."""

    @staticmethod
    def dense(t):
        """storage is exactly the tensor's numel elements (any dense layout: contiguous, channels_last)"""
        return t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last))

    @staticmethod
    def forward(ctx, flips, *params):
        """flips: indices of channels_last conv weights whose flipped, transposed fp16 copy ([Cin][Cout][ks][ks],
        channels_last: _HipConv's data-gradient weight) is returned too, after the plain copies, from the
        same launch (mapf_cast_f32_to_f16_multi_flip); those copies carry no gradient"""
        from . import _lib
        ctx.set_materialize_grads(False)
        assert all(_CastParams.dense(p) for p in params)
        ctx.layouts = [(p.shape, p.stride()) for p in params]
        outs = [torch.empty_strided(p.shape, p.stride(), dtype=torch.float16, device=p.device) for p in params]
        st = ctypes.c_void_p(torch.cuda.current_stream(params[0].device).cuda_stream)
        if not flips:
            _cast_multi(_lib.lib().mapf_cast_f32_to_f16_multi, params, outs, st)
            return tuple(outs)
        fl = [params[i] for i in flips]
        assert all(w.dim() == 4 and w.shape[2] == w.shape[3] and w.is_contiguous(memory_format=torch.channels_last)
                   for w in fl)
        wts = [torch.empty((w.shape[1], w.shape[0], w.shape[2], w.shape[3]), dtype=torch.float16, device=w.device,
                           memory_format=torch.channels_last) for w in fl]
        src, dst = list(params) + fl, outs + wts
        k = len(src)
        arr = lambda ts: (ctypes.c_void_p * k)(*[t.data_ptr() for t in ts])  # noqa: E731
        co = (ctypes.c_int32 * k)(*([0] * len(params) + [w.shape[0] for w in fl]))
        kk = (ctypes.c_int32 * k)(*([0] * len(params) + [w.shape[2] for w in fl]))
        _lib.check(_lib.lib().mapf_cast_f32_to_f16_multi_flip(arr(src), arr(dst),
                                                              (ctypes.c_int64 * k)(*[t.numel() for t in src]),
                                                              co, kk, k, st))
        ctx.mark_non_differentiable(*wts)
        return tuple(outs + wts)

    @staticmethod
    def backward(ctx, *grads):
        from . import _lib
        grads = grads[:len(ctx.layouts)]                 # the flipped copies carry none
        live = [i for i, g in enumerate(grads) if g is not None]
        outs = [None] * len(grads)
        if live:
            src, dst = [], []
            for i in live:
                shape, stride = ctx.layouts[i]
                g = grads[i]
                if g.stride() != stride:        # the parameter's own layout (AccumulateGrad keeps it)
                    g = torch.empty_strided(shape, stride, dtype=g.dtype, device=g.device).copy_(g)
                src.append(g)
                dst.append(torch.empty_strided(shape, stride, dtype=torch.float32, device=g.device))
            st = ctypes.c_void_p(torch.cuda.current_stream(src[0].device).cuda_stream)
            _cast_multi(_lib.lib().mapf_cast_f16_to_f32_multi, src, dst, st)
            for i, d in zip(live, dst):
                outs[i] = d
        return (None,) + tuple(outs)


class _BiasReLU(torch.autograd.Function):
    """relu(y + b) in place on a convolution's NHWC fp16 output (mapf_nhwc_bias_relu, the acting
    path's epilogue), for the TRAINING forward's conv layers run without MIOpen's bias; backward
    mapf_relu_bias_bwd_f16: the ReLU mask and the bias gradient (fp32 sums rounded to fp16, as
    torch's fp16 sum) in one pass -- in place of MIOpen's bias add, torch's ReLU and threshold
    backward and its bias-gradient reduction.  y: fp16 channels_last, b: fp16 [C]."""

    @staticmethod
    def forward(ctx, y, b):
        from . import _lib
        C = y.shape[1]
        rows = y.numel() // C
        st = ctypes.c_void_p(torch.cuda.current_stream(y.device).cuda_stream)
        _lib.check(_lib.lib().mapf_nhwc_bias_relu(ctypes.c_void_p(y.data_ptr()), ctypes.c_void_p(b.data_ptr()), rows,
                                                  C, st))
        ctx.mark_dirty(y)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import _lib
        y, = ctx.saved_tensors
        C = y.shape[1]
        rows = y.numel() // C
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = torch.empty_like(y)
        db = torch.empty(C, dtype=torch.float16, device=y.device)
        work = torch.empty(512 * C, dtype=torch.float32, device=y.device)
        st = ctypes.c_void_p(torch.cuda.current_stream(y.device).cuda_stream)
        p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        _lib.check(_lib.lib().mapf_relu_bias_bwd_f16(p(y), p(dy), p(dx), p(db), p(work), rows, C, st))
        return dx, db


class _BiasReLUPool(torch.autograd.Function):
    """maxpool2x2(relu(r + b)) from a convolution's raw NHWC fp16 output r in one pass
    (mapf_nhwc_bias_relu_pool2, the acting path's epilogue) for the TRAINING forward's pooled layers
    (conv1b, conv2b; net.py:106-111); backward mapf_relu_bias_pool_bwd_f16: torch's max_pool2d argmax
    routing, the ReLU mask and the bias gradient in one pass -- in place of the bias + ReLU pass, torch's
    max-pool forward / backward and the masked-gradient pass."""

    @staticmethod
    def forward(ctx, r, b):
        from . import _lib
        B, C, H, W = r.shape
        p = torch.empty((B, C, H // 2, W // 2), dtype=torch.float16, device=r.device,
                        memory_format=torch.channels_last)
        st = ctypes.c_void_p(torch.cuda.current_stream(r.device).cuda_stream)
        _lib.check(_lib.lib().mapf_nhwc_bias_relu_pool2(ctypes.c_void_p(r.data_ptr()), ctypes.c_void_p(b.data_ptr()),
                                                        ctypes.c_void_p(p.data_ptr()), B, H, W, C, st))
        ctx.save_for_backward(r, b)
        return p

    @staticmethod
    def backward(ctx, dp):
        from . import _lib
        r, b = ctx.saved_tensors
        B, C, H, W = r.shape
        dp = dp.contiguous(memory_format=torch.channels_last)
        dr = torch.empty_like(r)
        db = torch.empty(C, dtype=torch.float16, device=r.device)
        work = torch.empty(512 * C, dtype=torch.float32, device=r.device)
        st = ctypes.c_void_p(torch.cuda.current_stream(r.device).cuda_stream)
        p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        _lib.check(_lib.lib().mapf_relu_bias_pool_bwd_f16(p(r), p(b), p(dp), p(dr), p(db), p(work), B, H, W, C, st))
        return dr, db


class _HipConv(torch.autograd.Function):
    """conv2d(x, w) without bias (stride 1, fp16 NHWC, net.py:104-112) for the TRAINING forward's
    128- / 256-channel layers on the acting path's MFMA implicit GEMM (mapf_conv_nhwc_f16, raw fp16
    output: fp32 accumulation, one rounding, as MIOpen's); the bias + ReLU (+ pool) follow in _BiasReLU /
    _BiasReLUPool.  Backward: the data gradient is the same kernel run over dy with the flipped,
    transposed weight (dx = conv(dy, w[:, :, ::-1, ::-1]^T), padding ks - 1 - pad) wherever that
    shape is one the kernel has (SCRIMPNet._OWN_CONV: every layer from conv1a to conv2b), else MIOpen's;
    the weight gradient is MIOpen's (aten.convolution_backward).  In place of MIOpen's forward and data
    gradient (0.28 + 0.48 ms of a 256 x 8-row update, profiles/r06_update_profile_c3.txt)."""

    @staticmethod
    def forward(ctx, x, w, pad, b=None, wt=None):
        from . import _lib
        B, Cin, H, W = x.shape
        Cout, _, ks, _ = w.shape
        y = torch.empty((B, Cout, H + 2 * pad - ks + 1, W + 2 * pad - ks + 1), dtype=torch.float16, device=x.device,
                        memory_format=torch.channels_last)
        st = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
        # a channels_last [Cout][Cin][ks][ks] weight is [Cout][ks][ks][Cin] in memory: the kernel's packed form;
        # with b: relu(fp16(fp16(acc) + b)) in the epilogue, what _BiasReLU's pass writes
        bp = None if b is None else ctypes.c_void_p(b.data_ptr())
        _lib.check(_lib.lib().mapf_conv_nhwc_f16(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(w.data_ptr()), bp,
                                                 ctypes.c_void_p(y.data_ptr()), B, H, W, Cin, Cout, ks, pad,
                                                 0 if b is None else 1, st))
        ctx.save_for_backward(x, w, None if b is None else y, wt)
        ctx.pad = pad
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import _lib
        x, w, y, wt = ctx.saved_tensors
        pad = ctx.pad
        B, Cin, H, W = x.shape
        Cout, _, ks, _ = w.shape
        dy = dy.contiguous(memory_format=torch.channels_last)
        db = None
        if y is not None:                       # the fused bias + ReLU: _BiasReLU's backward first
            rows = y.numel() // Cout
            dyr = torch.empty_like(y)
            db = torch.empty(Cout, dtype=torch.float16, device=y.device)
            work = torch.empty(512 * Cout, dtype=torch.float32, device=y.device)
            st = ctypes.c_void_p(torch.cuda.current_stream(y.device).cuda_stream)
            p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
            _lib.check(_lib.lib().mapf_relu_bias_bwd_f16(p(y), p(dy), p(dyr), p(db), p(work), rows, Cout, st))
            dy = dyr
        own_dx = ctx.needs_input_grad[0] and (Cout, Cin, ks) in SCRIMPNet._OWN_CONV
        mask = [ctx.needs_input_grad[0] and not own_dx, ctx.needs_input_grad[1], False]
        dx = dw = None
        if any(mask):
            gx, gw, _ = torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [pad, pad], [1, 1], False, [0, 0], 1,
                                                            mask)
            dx = gx if mask[0] else None
            dw = gw if mask[1] else None
        if own_dx:
            if wt is None:                      # else _CastParams made it (SCRIMPNet._flip_names)
                wt = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)  # [Cin][ks][ks][Cout]
            dx = torch.empty(x.shape, dtype=torch.float16, device=x.device, memory_format=torch.channels_last)
            st = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
            _lib.check(_lib.lib().mapf_conv_nhwc_f16(ctypes.c_void_p(dy.data_ptr()), ctypes.c_void_p(wt.data_ptr()), None,
                                                     ctypes.c_void_p(dx.data_ptr()), B, dy.shape[2], dy.shape[3], Cout,
                                                     Cin, ks, ks - 1 - pad, 0, st))
        return dx, dw, None, db, None


class _TokensLN(torch.autograd.Function):
    """The TRAINING forward's tokeniser tail and the first PreNorm in one pass (round 6):
    x = dropout(cat(cls, A * VV) + pos) fp32, z = fp16(LayerNorm(x)) -- mapf_tokens_layernorm_train, the
    ops and roundings of SCRIMPNet.forward's torch chain (net.py:124-130, transformer.py:7-24; the mask is
    the kernels' counter hash from the device seed, salt 32).  Backward: LayerNorm's with the residual's
    gradient (mapf_layernorm_bwd_f16), then mapf_tokens_train_bwd: the dropout mask, dA, dVV (fp16) and the
    sums over the batch for pos and cls.  In place of torch's mul, cat, add, dropout, LayerNorm launches and
    their backward's mul / sum / masked-scale passes (~0.29 ms of a 256 x 8-row update,
    profiles/r06n_update_shapes.txt).  A: fp32 [B, 16]; VV: fp16 [B, 512]; returns (z [B, 17, 512] fp16,
    x [B, 17, 512] fp32: the first block's residual)."""

    @staticmethod
    def forward(ctx, A, VV, cls, pos, weight, bias, eps, p, seed, salt):
        from . import _lib
        ctx.set_materialize_grads(False)
        B = A.shape[0]
        x = torch.empty(B, 17, 512, dtype=torch.float32, device=A.device)
        z = torch.empty(B, 17, 512, dtype=torch.float16, device=A.device)
        st = ctypes.c_void_p(torch.cuda.current_stream(A.device).cuda_stream)
        ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        _lib.check(_lib.lib().mapf_tokens_layernorm_train(ptr(x), ptr(A), ptr(VV), ptr(cls), ptr(pos), B, 16, float(p),
                                                          ptr(seed), int(salt), ptr(weight), ptr(bias), float(eps),
                                                          ptr(z), st))
        ctx.save_for_backward(x, A, VV, weight, seed)
        ctx.eps, ctx.p, ctx.salt, ctx.shapes = float(eps), float(p), int(salt), (cls.shape, pos.shape)
        return z, x

    @staticmethod
    def backward(ctx, dz, dres):
        from . import _lib
        x, A, VV, weight, seed = ctx.saved_tensors
        B = A.shape[0]
        rows = B * 17
        dev = x.device
        if dz is None:
            dz = torch.zeros(rows, 512, dtype=torch.float16, device=dev)
        dz = dz.reshape(rows, 512).to(torch.float16).contiguous()
        if dres is not None:
            dres = dres.reshape(rows, 512).to(torch.float32).contiguous()
        dx = torch.empty(rows, 512, dtype=torch.float32, device=dev)
        dg = torch.empty(512, dtype=torch.float32, device=dev)
        db = torch.empty(512, dtype=torch.float32, device=dev)
        work = torch.empty(512 * 17 * 512, dtype=torch.float32, device=dev)   # mapf_tokens_train_bwd's partials
        st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        _lib.check(_lib.lib().mapf_layernorm_bwd_f16(ptr(x), 512, ptr(weight), ptr(dz),
                                                     None if dres is None else ptr(dres), ptr(dx), ptr(dg), ptr(db),
                                                     ptr(work), rows, 512, ctx.eps, st))
        dA = torch.empty(B, 16, dtype=torch.float32, device=dev)
        dVV = torch.empty(B, 512, dtype=torch.float16, device=dev)
        dpos = torch.empty(17, 512, dtype=torch.float32, device=dev)
        dcls = torch.empty(512, dtype=torch.float32, device=dev)
        _lib.check(_lib.lib().mapf_tokens_train_bwd(ptr(dx), ptr(A), ptr(VV), ptr(dA), ptr(dVV), ptr(dpos), ptr(dcls),
                                                    ptr(work), B, 16, ctx.p, ptr(seed), ctx.salt, st))
        cs, ps = ctx.shapes
        return dA, dVV, dcls.view(cs), dpos.view(ps), dg, db, None, None, None, None


def _drop_p(m):
    """a Dropout module's probability as the forward applies it (0 in eval mode)"""
    return float(m.p) if m.training else 0.0


class _DropResLN(torch.autograd.Function):
    """The TRAINING forward's residual + next PreNorm in one pass (round 6): x_out = res + dropout(y),
    z = fp16(LayerNorm(x_out)) -- mapf_dropout_residual_layernorm_train; backward
    mapf_layernorm_dropout_bwd_f16: LayerNorm's backward with the residual gradient (as _HipLayerNorm),
    the dropped branch's fp16 gradient and dgamma / dbeta in one pass.  In place of torch's dropout
    forward / backward, the fp32 add and a separate LayerNorm launch at every residual that feeds a
    LayerNorm (transformer.py:7-24, 64-85).  The dropout mask is the kernels' counter hash seeded from
    `seed` (SCRIMPNet._train_seed, int64 [1] in device memory, incremented by every training forward --
    also inside a captured update) and the site's salt.  res: fp32 [.., 512] (a strided view allowed),
    y: fp16 [.., 512]."""

    @staticmethod
    def forward(ctx, res, y, weight, bias, eps, p, seed, salt):
        from . import _lib
        ctx.set_materialize_grads(False)
        rows = res.numel() // 512
        r2 = res.reshape(rows, 512)
        if r2.stride(1) != 1 or r2.stride(0) % 4:
            r2 = r2.contiguous()
        y2 = y.reshape(rows, 512).contiguous()
        xo = torch.empty(rows, 512, dtype=torch.float32, device=res.device)
        z = torch.empty(rows, 512, dtype=torch.float16, device=res.device)
        st = ctypes.c_void_p(torch.cuda.current_stream(res.device).cuda_stream)
        q = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        _lib.check(_lib.lib().mapf_dropout_residual_layernorm_train(q(r2), r2.stride(0), q(y2), q(xo), q(weight), q(bias),
                                                                     q(z), rows, 512, float(eps), float(p), q(seed),
                                                                     int(salt), st))
        ctx.save_for_backward(xo, weight, seed)
        ctx.meta = (float(eps), float(p), int(salt), res.shape, y.shape)
        out_shape = tuple(res.shape[:-1]) + (512,)
        return z.view(out_shape), xo.view(out_shape)

    @staticmethod
    def backward(ctx, dz, dxo):
        from . import _lib
        xo, weight, seed = ctx.saved_tensors
        eps, p, salt, res_shape, y_shape = ctx.meta
        rows = xo.shape[0]
        dz = (torch.zeros(rows, 512, dtype=torch.float16, device=xo.device) if dz is None else
              dz.reshape(rows, 512).to(torch.float16).contiguous())
        if dxo is not None:
            dxo = dxo.reshape(rows, 512).to(torch.float32).contiguous()
        dx = torch.empty(rows, 512, dtype=torch.float32, device=xo.device)
        dy = torch.empty(rows, 512, dtype=torch.float16, device=xo.device)
        dg = torch.empty(512, dtype=torch.float32, device=xo.device)
        db = torch.empty(512, dtype=torch.float32, device=xo.device)
        work = torch.empty(2 * 512 * 512, dtype=torch.float32, device=xo.device)
        st = ctypes.c_void_p(torch.cuda.current_stream(xo.device).cuda_stream)
        q = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        _lib.check(_lib.lib().mapf_layernorm_dropout_bwd_f16(q(xo), q(weight), q(dz), None if dxo is None else q(dxo),
                                                             q(dx), q(dy), q(dg), q(db), q(work), rows, 512, eps, p,
                                                             q(seed), salt, st))
        return dx.view(res_shape), dy.view(y_shape), dg, db, None, None, None, None


class _GeluDropout(torch.autograd.Function):
    """dropout(gelu(h)) of the TRAINING forward's MLP (transformer.py:27-45, af1 + do1) in one pass each
    way (round 6): mapf_gelu_dropout_train_f16 / mapf_gelu_dropout_bwd_f16 -- torch's fp16 GELU, dropout,
    masked_scale and GeluBackward kernels in two launches; the mask as _DropResLN's.  h: fp16."""

    @staticmethod
    def forward(ctx, h, p, seed, salt):
        from . import _lib
        h = h.contiguous()
        out = torch.empty_like(h)
        st = ctypes.c_void_p(torch.cuda.current_stream(h.device).cuda_stream)
        _lib.check(_lib.lib().mapf_gelu_dropout_train_f16(ctypes.c_void_p(h.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                                          h.numel(), float(p), ctypes.c_void_p(seed.data_ptr()),
                                                          int(salt), st))
        ctx.save_for_backward(h, seed)
        ctx.meta = (float(p), int(salt))
        return out

    @staticmethod
    def backward(ctx, dout):
        from . import _lib
        h, seed = ctx.saved_tensors
        p, salt = ctx.meta
        dout = dout.to(torch.float16).contiguous()
        dh = torch.empty_like(h)
        st = ctypes.c_void_p(torch.cuda.current_stream(h.device).cuda_stream)
        q = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        _lib.check(_lib.lib().mapf_gelu_dropout_bwd_f16(q(h), q(dout), q(dh), h.numel(), p, q(seed), salt, st))
        return dh, None, None, None


class _PreNorm(nn.Module):
    """Residual(LayerNormalize(dim, fn)) of transformer.py:7-24 (state_dict path `.fn.norm` / `.fn.fn`)."""

    hip_layernorm = True               # the training forward's LayerNorm on _HipLayerNorm (GPU, autocast)

    def __init__(self, dim, fn):
        super().__init__()
        self.fn = nn.Module()
        self.fn.norm = nn.LayerNorm(dim)
        self.fn.fn = fn

    def _norm(self, x):
        """(LayerNorm(x), the residual x): on the GPU training path one _HipLayerNorm whose backward
        also takes the residual's gradient"""
        n = self.fn.norm
        if (self.hip_layernorm and x.is_cuda and x.dtype == torch.float32 and x.shape[-1] == 512 and
                torch.is_grad_enabled() and torch.is_autocast_enabled("cuda") and n.elementwise_affine):
            return _HipLayerNorm.apply(x, n.weight, n.bias, n.eps)
        return n(x), x

    def forward(self, x):
        z, res = self._norm(x)
        return self.fn.fn(z) + res

    def forward_first(self, x):
        """Token 0 of forward(x) only (x: [b, n, d] -> [b, 1, d])."""
        z, res = self._norm(x)
        return self.fn.fn.forward_first(z) + res[:, :1]


class _HipAttention(torch.autograd.Function):
    """softmax(q k^T * scale) v over <= 32 tokens, 16 heads of 32, for the TRAINING forward:
    mapf_attention_f16 forward, mapf_attention_bwd_f16 backward (csrc/mapf_policy.hip) in place of
    SDPA's flash kernels, which are tiled for long sequences.  q: `rows` tokens at column q_off of
    qsrc [b, t, wq] (or [b, wq]); k, v at columns k_off, v_off of kvsrc [b, n, wkv]; both fp16
    and contiguous -- qsrc may be kvsrc (the fused qkv projection), then one gradient comes back.
    Returns [b, rows, 512] fp16."""

    @staticmethod
    def _meta(qsrc, kvsrc):
        b, n, wkv = kvsrc.shape
        wq = qsrc.shape[-1]
        q_ss = wq * (qsrc.shape[1] if qsrc.dim() == 3 else 1)
        return b, n, wq, q_ss, wkv, n * wkv

    @staticmethod
    def forward(ctx, qsrc, kvsrc, rows, q_off, k_off, v_off, scale):
        from . import _lib
        b, n, wq, q_ss, kv_ts, kv_ss = _HipAttention._meta(qsrc, kvsrc)
        out = torch.empty(b, rows, 512, dtype=torch.float16, device=qsrc.device)
        st = ctypes.c_void_p(torch.cuda.current_stream(qsrc.device).cuda_stream)
        e = 2                                                      # bytes per fp16 element
        _lib.check(_lib.lib().mapf_attention_f16(
            ctypes.c_void_p(qsrc.data_ptr() + e * q_off), ctypes.c_void_p(kvsrc.data_ptr() + e * k_off),
            ctypes.c_void_p(kvsrc.data_ptr() + e * v_off), ctypes.c_void_p(out.data_ptr()), b, n, rows, wq, q_ss,
            kv_ts, kv_ss, 16, 32, float(scale), st))
        ctx.save_for_backward(qsrc, kvsrc, out)
        ctx.args = (rows, q_off, k_off, v_off, scale, qsrc.data_ptr() == kvsrc.data_ptr())
        return out

    @staticmethod
    def backward(ctx, dout):
        from . import _lib
        qsrc, kvsrc, out = ctx.saved_tensors
        rows, q_off, k_off, v_off, scale, same = ctx.args
        b, n, wq, q_ss, kv_ts, kv_ss = _HipAttention._meta(qsrc, kvsrc)
        dout = dout.contiguous()
        gq = torch.empty_like(qsrc)
        gkv = gq if same else torch.empty_like(kvsrc)
        st = ctypes.c_void_p(torch.cuda.current_stream(qsrc.device).cuda_stream)
        e = 2
        p = lambda t, off=0: ctypes.c_void_p(t.data_ptr() + e * off)  # noqa
        _lib.check(_lib.lib().mapf_attention_bwd_f16(
            p(qsrc, q_off), p(kvsrc, k_off), p(kvsrc, v_off), p(out), p(dout), p(gq, q_off), p(gkv, k_off),
            p(gkv, v_off), b, n, rows, wq, q_ss, kv_ts, kv_ss, 512, rows * 512, 16, 32, float(scale), st))
        return gq, (None if same else gkv), None, None, None, None, None


class _SplitKLinear(torch.autograd.Function):
    """F.linear under fp16 autocast for the TRAINING forward's 17-token layers (34,816 rows at 2,048
    agents): the forward is autocast's (fp16 operands, one GEMM with the bias), the input gradient
    one GEMM; the WEIGHT gradient is split over SPLIT row chunks, one batched GEMM with fp32 partial
    products summed in fp32, then rounded to fp16 as autograd's one-GEMM fp16 weight gradient is
    (so an fp16 overflow still reaches GradScaler's found-inf).  hipBLASLt's one GEMM has only
    (out / 64) x (in / 128) output tiles for the 34,816-deep reduction -- 32 tiles on 256 CUs for a
    512 x 512 weight (tools/profile_update.py)."""

    SPLIT = 16                      # 8 -> 16: -0.06 / -0.11 ms per 256 x 8 / 256 x 16 update (profiles/r06ze_ab_split*)
    MIN_ROWS = 8192                 # _train_linear takes this form from this many rows on
    out_dtype_ok = None             # torch.bmm(..., out_dtype=float32) on this build (decided once, _fp32_bmm)

    @staticmethod
    def _fp32_bmm(a, c):
        """torch.bmm(a, c, out_dtype=float32), or None when this torch build has no such overload --
        decided once, by the call's signature error (TypeError / NotImplementedError) only: any other
        error (an OOM, a launch failure) propagates instead of switching every later gradient to fp16
        partial products"""
        if _SplitKLinear.out_dtype_ok is False:
            return None
        try:
            parts = torch.bmm(a, c, out_dtype=torch.float32)
        except (TypeError, NotImplementedError) as e:
            import warnings
            warnings.warn(f"torch.bmm(..., out_dtype=float32) unavailable ({e}): split weight gradients use fp16 "
                          f"partial products", RuntimeWarning)
            _SplitKLinear.out_dtype_ok = False
            return None
        _SplitKLinear.out_dtype_ok = True
        return parts

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.float16)
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.bias_dtype = b.dtype if b is not None else None
        return F.linear(x, w, b)

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        n_out, n_in = w.shape
        gy2 = gy.reshape(-1, n_out)
        x2 = x.reshape(-1, n_in)
        gx = (gy2 @ w).view(x.shape) if ctx.needs_input_grad[0] else None
        S = _SplitKLinear.SPLIT
        r = gy2.shape[0] // S
        a = gy2.view(S, r, n_out).transpose(1, 2)
        c = x2.view(S, r, n_in)
        parts = _SplitKLinear._fp32_bmm(a, c)
        if parts is None:
            parts = torch.bmm(a, c).float()
        gw = parts.sum(0).to(torch.float16).to(w.dtype)
        gb = None
        if ctx.needs_input_grad[2] and n_out % 4:
            gb = gy2.sum(0).to(ctx.bias_dtype)
        elif ctx.needs_input_grad[2]:   # bias gradient: the column sums of gy (mapf_colsum_f16, fp32 sums -> fp16)
            from . import _lib
            gy2 = gy2.contiguous()
            gb = torch.empty(n_out, dtype=torch.float16, device=gy.device)
            work = torch.empty(512 * n_out, dtype=torch.float32, device=gy.device)
            st = ctypes.c_void_p(torch.cuda.current_stream(gy.device).cuda_stream)
            _lib.check(_lib.lib().mapf_colsum_f16(ctypes.c_void_p(gy2.data_ptr()), ctypes.c_void_p(gb.data_ptr()),
                                                  ctypes.c_void_p(work.data_ptr()), gy2.shape[0], n_out, st))
            gb = gb.to(ctx.bias_dtype)
        return gx, gw, gb


class _QKVFirst(torch.autograd.Function):
    """The last encoder block's projections (forward_first_core) from ONE to_qkv weight [3d, d]: token 0's
    query q = x[:, 0] W_q^T + b_q and every token's keys / values kv = x W_kv^T + b_kv, with one backward:
    the input gradient is kv's GEMM with token 0's query gradient accumulated into its rows (addmm_), so no
    zero-filled [b, n, d] select gradient and no add; the weight and bias gradients are written into one
    [3d, d] / [3d] tensor, so no zero-filled slice gradients and adds either.  kv's weight gradient is
    _SplitKLinear's (split-K, fp32 partials, rounded to fp16), q's one GEMM; the bias gradients
    mapf_colsum_f16.  x: fp16 [b, n, d] contiguous; w, b fp16 (the training forward's _CastParams copies)."""

    @staticmethod
    def forward(ctx, x, w, b):
        d = x.shape[-1]
        ctx.save_for_backward(x, w)
        return torch.addmm(b[:d], x[:, 0], w[:d].t()), F.linear(x, w[d:], b[d:])

    @staticmethod
    def backward(ctx, dq, dkv):
        from . import _lib
        x, w = ctx.saved_tensors
        B, n, d = x.shape
        dev = x.device
        x2 = x.reshape(-1, d)
        dq = torch.zeros(B, d, dtype=x.dtype, device=dev) if dq is None else dq.contiguous()
        dkv2 = (torch.zeros(B * n, 2 * d, dtype=x.dtype, device=dev) if dkv is None else dkv.reshape(-1, 2 * d)
                .contiguous())
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = (dkv2 @ w[d:]).view(B, n, d)
            gx[:, 0].addmm_(dq, w[:d])
        if ctx.needs_input_grad[1]:
            gw = torch.empty(3 * d, d, dtype=torch.float16, device=dev)
            torch.mm(dq.t(), x[:, 0], out=gw[:d])
            S = _SplitKLinear.SPLIT
            R = dkv2.shape[0]
            parts = None
            if R % S == 0:
                a, c = dkv2.view(S, R // S, 2 * d).transpose(1, 2), x2.view(S, R // S, d)
                parts = _SplitKLinear._fp32_bmm(a, c)
                if parts is None:
                    parts = torch.bmm(a, c).float()
            if parts is not None:
                gw[d:].copy_(parts.sum(0))
            else:
                torch.mm(dkv2.t(), x2, out=gw[d:])
            gw = gw.to(w.dtype)
        if ctx.needs_input_grad[2]:
            gb = torch.empty(3 * d, dtype=torch.float16, device=dev)
            work = torch.empty(512 * 2 * d, dtype=torch.float32, device=dev)
            st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            for g2, lo, C in ((dq, 0, d), (dkv2, d, 2 * d)):
                _lib.check(_lib.lib().mapf_colsum_f16(ctypes.c_void_p(g2.data_ptr()),
                                                      ctypes.c_void_p(gb.data_ptr() + 2 * lo),
                                                      ctypes.c_void_p(work.data_ptr()), g2.shape[0], C, st))
        return gx, gw, gb


class _LinearBG(torch.autograd.Function):
    """F.linear(x, w, b) on fp16 operands for the training forward's short linears (token 0's and the
    fully connected layers: 2-D, rows < _SplitKLinear.MIN_ROWS): the same addmm forward and the same
    two GEMMs backward as torch's AddmmBackward, the bias gradient from mapf_colsum_f16's one-launch
    column sum (fp32, fixed order, rounded to fp16) in place of torch's fp16 reduction (~15 us per layer,
    8 layers per update: profiles/r06n_update_shapes.txt).  x: fp16 [rows, in] (strided rows allowed)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return torch.addmm(b, x, w.t())

    @staticmethod
    def backward(ctx, gy):
        from . import _lib
        x, w = ctx.saved_tensors
        gy = gy.contiguous()
        gx = gy.mm(w) if ctx.needs_input_grad[0] else None
        gw = x.t().mm(gy).t() if ctx.needs_input_grad[1] else None
        gb = None
        if ctx.needs_input_grad[2]:
            n_out = gy.shape[1]
            gb = torch.empty(n_out, dtype=torch.float16, device=gy.device)
            work = torch.empty(1 if gy.shape[0] <= 8192 else 512 * n_out, dtype=torch.float32, device=gy.device)
            st = ctypes.c_void_p(torch.cuda.current_stream(gy.device).cuda_stream)
            _lib.check(_lib.lib().mapf_colsum_f16(ctypes.c_void_p(gy.data_ptr()), ctypes.c_void_p(gb.data_ptr()),
                                                  ctypes.c_void_p(work.data_ptr()), gy.shape[0], n_out, st))
        return gx, gw, gb


def _train_linear(x, w, b):
    """F.linear(x, w, b) of the training forward: the split weight gradient (_SplitKLinear) when x
    has many rows (grad enabled, on the GPU), _LinearBG for short 2-D fp16 ones, plain autocast F.linear
    otherwise."""
    rows = x.numel() // x.shape[-1]
    if torch.is_grad_enabled() and x.is_cuda and torch.is_autocast_enabled("cuda"):
        if rows >= _SplitKLinear.MIN_ROWS and rows % _SplitKLinear.SPLIT == 0 and w.requires_grad:
            return _SplitKLinear.apply(x, w, b)
        if (_LinearBG.enabled and x.dim() == 2 and x.dtype == w.dtype == torch.float16 and b is not None and
                b.dtype == torch.float16 and w.shape[0] % 8 == 0 and 0 < rows <= 8192 and x.stride(1) == 1):
            return _LinearBG.apply(x, w, b)
    return F.linear(x, w, b)


_LinearBG.enabled = True


class _SelfAttention(nn.Module):
    """transformer.py:48-85: fused qkv projection, softmax(q k^T / sqrt(dim)) v, output projection.
    Note the reference scales by dim ** -0.5 (the model width), not the head width.
    The attention itself is one fused scaled_dot_product_attention call (no dropout on
    the attention weights, as in the reference): 17 tokens x 16 heads x 32 per agent
    as batched GEMMs would be ~500k tiny matrix products per layer."""

    def __init__(self, dim, heads, dropout):
        super().__init__()
        self.heads = heads
        self.scale = dim ** -0.5
        self.to_qkv = nn.Linear(dim, dim * 3, bias=True)
        nn.init.xavier_uniform_(self.to_qkv.weight)
        nn.init.zeros_(self.to_qkv.bias)
        self.nn1 = nn.Linear(dim, dim)
        nn.init.xavier_uniform_(self.nn1.weight)
        nn.init.zeros_(self.nn1.bias)
        self.do1 = nn.Dropout(dropout)

    hip_attention = True               # the training forward's attention on _HipAttention (GPU, fp16)
    qkv_first = True                   # the last block's q / kv projections and their backward as _QKVFirst

    def _hip(self, x, t):
        return (self.hip_attention and x.is_cuda and t.dtype == torch.float16 and self.heads == 16 and
                x.shape[-1] == 512 and x.shape[1] <= 32 and torch.is_grad_enabled())

    def forward(self, x):
        return self.do1(self.forward_core(x))

    def forward_core(self, x):
        """forward(x) before its dropout (the fused training residual applies it)"""
        b, n, d = x.shape
        h = self.heads
        qkv = _train_linear(x, self.to_qkv.weight, self.to_qkv.bias)
        if self._hip(x, qkv):
            att = _HipAttention.apply(qkv.contiguous(), qkv.contiguous(), n, 0, d, 2 * d, self.scale)
            return _train_linear(att, self.nn1.weight, self.nn1.bias)
        qkv = qkv.view(b, n, 3, h, d // h).permute(2, 0, 3, 1, 4)   # 3, b, h, n, dh
        q, k, v = qkv[0], qkv[1], qkv[2]
        out = F.scaled_dot_product_attention(q, k, v, scale=self.scale).transpose(1, 2).reshape(b, n, d)
        return self.nn1(out)

    def forward_first(self, x):
        """Token 0 of forward(x) only: keys and values of every token, the query of token 0."""
        return self.do1(self.forward_first_core(x))

    def forward_first_core(self, x):
        b, n, d = x.shape
        h = self.heads
        w, bias = self.to_qkv.weight, self.to_qkv.bias
        # x[:, 0] is a 2-D strided view: one GEMM with lda = n*d ([b, 1, d] would run as a slow bmm)
        if (self.qkv_first and torch.is_grad_enabled() and x.is_cuda and torch.is_autocast_enabled("cuda") and
                x.dtype == w.dtype == bias.dtype == torch.float16 and x.is_contiguous() and d % 8 == 0 and
                w.requires_grad and b * n >= _SplitKLinear.MIN_ROWS):
            q, kv = _QKVFirst.apply(x, w, bias)
        else:
            q = _train_linear(x[:, 0], w[:d], bias[:d])
            kv = _train_linear(x, w[d:], bias[d:])
        if self._hip(x, q):
            att = _HipAttention.apply(q.contiguous(), kv.contiguous(), 1, 0, 0, d, self.scale)
            return _train_linear(att.reshape(b, d), self.nn1.weight, self.nn1.bias).view(b, 1, d)
        q = q.view(b, 1, h, d // h).transpose(1, 2)                                             # b, h, 1, dh
        kv = kv.view(b, n, 2, h, d // h).permute(2, 0, 3, 1, 4)                                 # 2, b, h, n, dh
        out = F.scaled_dot_product_attention(q, kv[0], kv[1], scale=self.scale).transpose(1, 2).reshape(b, 1, d)
        return self.nn1(out)


class _FeedForward(nn.Module):
    """MLP_Block (transformer.py:27-45)."""

    def __init__(self, dim, hidden, dropout):
        super().__init__()
        self.nn1 = nn.Linear(dim, hidden)
        nn.init.xavier_uniform_(self.nn1.weight)
        nn.init.normal_(self.nn1.bias, std=1e-6)
        self.af1 = nn.GELU()
        self.do1 = nn.Dropout(dropout)
        self.nn2 = nn.Linear(hidden, dim)
        nn.init.xavier_uniform_(self.nn2.weight)
        nn.init.normal_(self.nn2.bias, std=1e-6)
        self.do2 = nn.Dropout(dropout)

    def forward(self, x):
        return self.do2(self.forward_core(x))

    def forward_core(self, x, seed=None, salt=0):
        """forward(x) before its last dropout; with the training seed, GELU + dropout as _GeluDropout"""
        h = _train_linear(x, self.nn1.weight, self.nn1.bias)
        if (seed is not None and h.is_cuda and h.dtype == torch.float16 and h.numel() % 4 == 0 and
                getattr(self.af1, "approximate", None) == "none"):
            h = _GeluDropout.apply(h, _drop_p(self.do1), seed, salt)
        else:
            h = self.do1(self.af1(h))
        return _train_linear(h, self.nn2.weight, self.nn2.bias)


class _Encoder(nn.Module):
    def __init__(self, dim, depth, heads, mlp_dim, dropout):
        super().__init__()
        self.layers = nn.ModuleList([
            nn.ModuleList([_PreNorm(dim, _SelfAttention(dim, heads, dropout)),
                           _PreNorm(dim, _FeedForward(dim, mlp_dim, dropout))])
            for _ in range(depth)])

    fused_train = True      # training forward (GPU): _DropResLN residuals and _GeluDropout (with a seed)

    def _train_fused_ok(self, x):
        return (self.fused_train and x.is_cuda and torch.is_grad_enabled() and torch.is_autocast_enabled("cuda") and
                x.dtype == torch.float32 and x.shape[-1] == 512 and _PreNorm.hip_layernorm and
                all(pn.fn.norm.elementwise_affine for blk in self.layers for pn in blk))

    def _forward_train_fused(self, x, first_only, seed, start=None):
        """forward() of the training pass with every residual that feeds a LayerNorm as one _DropResLN
        (the residual add, its dropout and the next PreNorm's LayerNorm) and the MLP's GELU + dropout as
        _GeluDropout; the same operations and rounding points, the dropout masks from the kernels'
        hash (sites salted 2 li, 2 li + 1, 16 + li).  start: (z, x) -- the first PreNorm's output and its
        residual made already (_TokensLN); x is then unused."""
        L = len(self.layers)
        z, res = self.layers[0][0]._norm(x) if start is None else start
        for li, (att, ff) in enumerate(self.layers):
            a, f = att.fn.fn, ff.fn.fn
            if first_only and li == L - 1:
                y = a.forward_first_core(z)
                res = res[:, :1]
            else:
                y = a.forward_core(z)
            nrm = ff.fn.norm
            z, res = _DropResLN.apply(res, y, nrm.weight, nrm.bias, nrm.eps, _drop_p(a.do1), seed, 2 * li)
            y = f.forward_core(z, seed, 16 + li)
            if li + 1 < L:
                nrm = self.layers[li + 1][0].fn.norm
                z, res = _DropResLN.apply(res, y, nrm.weight, nrm.bias, nrm.eps, _drop_p(f.do2), seed, 2 * li + 1)
            else:
                return res + f.do2(y)

    def forward(self, x, first_only=False, seed=None):
        """first_only: return token 0 of the last block's output only ([b, 1, d]).  SCRIMPNet reads
        nothing else (net.py:140-141 takes x[:, 0]), so the last block's queries, output
        projection and MLP of tokens 1..16 are skipped; keys/values still see every token.
        seed: the training forward's device dropout seed (SCRIMPNet._train_seed): the fused training path."""
        if seed is not None and self._train_fused_ok(x):
            return self._forward_train_fused(x, first_only, seed)
        for li, (att, ff) in enumerate(self.layers):
            if first_only and li == len(self.layers) - 1:
                return ff(att.forward_first(x))
            x = ff(att(x))
        return x


class SCRIMPNet(nn.Module):
    def __init__(self, numChannel=None, num_agents=None, fov=None):
        super().__init__()
        W = NetParameters.NET_SIZE
        self.L = 16
        self.cT = W
        self.num_channel = NetParameters.NUM_CHANNEL if numChannel is None else numChannel
        self.num_agents = num_agents
        self.fov = fov
        self.conv1 = nn.Conv2d(self.num_channel, W // 4, 3, 1, 1)
        self.conv1a = nn.Conv2d(W // 4, W // 4, 3, 1, 1)
        self.conv1b = nn.Conv2d(W // 4, W // 4, 3, 1, 1)
        self.pool1 = nn.MaxPool2d(2)
        self.conv2 = nn.Conv2d(W // 4, W // 2, 2, 1, 1)
        self.conv2a = nn.Conv2d(W // 2, W // 2, 2, 1, 1)
        self.conv2b = nn.Conv2d(W // 2, W // 2, 2, 1, 1)
        self.pool2 = nn.MaxPool2d(2)
        self.conv3 = nn.Conv2d(W // 2, W - NetParameters.GOAL_REPR_SIZE, 3, 1, 0)
        self.fully_connected_1 = nn.Linear(NetParameters.VECTOR_LEN, NetParameters.GOAL_REPR_SIZE)
        self.fully_connected_2 = nn.Linear(W, W)
        self.fully_connected_3 = nn.Linear(W, W)
        self.token_wA = nn.Parameter(torch.empty(8, self.L, 512))
        nn.init.xavier_uniform_(self.token_wA)
        self.token_wV = nn.Parameter(torch.empty(8, 512, self.cT))
        nn.init.xavier_uniform_(self.token_wV)
        self.pos_embedding = nn.Parameter(torch.empty(1, self.L + 1, self.cT))
        nn.init.normal_(self.pos_embedding, std=0.02)
        self.cls_token = nn.Parameter(torch.zeros(1, 1, self.cT))
        self.dropout = nn.Dropout(0.2)
        self.transformer = _Encoder(self.cT, 2, 16, 512, 0.2)
        self.nn_same = nn.Linear(self.cT, self.cT)
        nn.init.xavier_uniform_(self.nn_same.weight)
        nn.init.normal_(self.nn_same.bias, std=1e-6)
        self.policy_layer = nn.Linear(W, EnvParameters.N_ACTIONS)
        self.value_layer = nn.Linear(W, 1)
        self.cost_value_layer = nn.Linear(W, 1)
        self.blocking_layer = nn.Linear(W, 1)
        self.apply(_xavier_like)
        self.fused_acting = True      # no-grad GPU forward through _forward_fused (csrc/mapf_policy.hip)
        self.fused_attention = True   # short-sequence attention kernel (mapf_attention_f16) instead of SDPA
        self.fused_residual_ln = True  # residual + next LayerNorm in one pass (mapf_dropout_residual_layernorm)
        self.own_conv = True           # 128/256-channel convolutions as the MFMA implicit GEMM (mapf_conv_nhwc_f16)
        self.fused_linear = True       # 512x512 linears + their dropout/residual/LayerNorm or GELU epilogue, one launch
        self._h16 = {}                 # fp16 weights of the acting forward (_half)

    # (Cin, Cout, kernel) of mapf_conv_nhwc_f16; (256, 128, 2) is conv2's data gradient (_HipConv)
    _OWN_CONV = {(128, 128, 3), (128, 256, 2), (256, 256, 2), (256, 128, 2)}
    cast_params = True             # training forward: conv / linear weights to fp16 in one launch (_CastParams)
    _in_cast = False

    hip_bias_relu = True           # training forward: conv bias + ReLU on _BiasReLU (GPU, autocast)
    hip_conv = True                # training forward: the _OWN_CONV layers' convolutions on _HipConv (MFMA)
    conv3_gemm = True              # training forward: a conv whose kernel covers its unpadded input as one GEMM
    conv_bias_relu = True          # training forward: _HipConv's epilogue adds the bias and applies the ReLU
    cast_flips = True              # training forward: _HipConv's flipped weights made in _CastParams' launch
    fused_tokens = True            # training forward: tokens + dropout + first LayerNorm as _TokensLN

    def _conv_nobias(self, x, m):
        """conv2d(x, m.weight) without the bias, fp16 NHWC: a plain GEMM where the kernel covers its whole
        unpadded input (conv3: 3x3 on 3x3 -> 1x1, as the acting path runs it; MIOpen's backward-data kernel
        took ~160 us for it in a 256 x 8-row update, profiles/r06h_update_profile_c3.txt), _HipConv for the
        MFMA kernel's shapes, else MIOpen"""
        w = m.weight
        co, ci, ks, _ = w.shape
        if (self.conv3_gemm and m.padding == (0, 0) and m.stride == (1, 1) and m.dilation == (1, 1) and m.groups == 1
                and x.shape[2] == ks and x.shape[3] == ks and x.dtype == torch.float16 and w.dtype == torch.float16
                and x.is_contiguous(memory_format=torch.channels_last)
                and w.is_contiguous(memory_format=torch.channels_last)):
            # [B, ks*ks*ci] x [co, ks*ks*ci]^T with K ordered (ky, kx, c): both operands are views of the
            # channels_last storage; autograd's GEMMs give the data and weight gradients
            B = x.shape[0]
            y = F.linear(x.permute(0, 2, 3, 1).reshape(B, -1), w.permute(0, 2, 3, 1).reshape(co, -1))
            return y.view(B, co, 1, 1)
        if self._own_conv_ok(x, m):
            return _HipConv.apply(x, w, m.padding[0], None, self._wt(m))
        return F.conv2d(x, w, None, m.stride, m.padding)

    def _wt(self, m):
        """m's flipped, transposed fp16 weight from this forward's _CastParams launch, or None"""
        return self.__dict__.get("_wt16", {}).get(m)

    def _own_conv_ok(self, x, m):
        """m's convolution of x runs on _HipConv (mapf_conv_nhwc_f16)"""
        w = m.weight
        co, ci, ks, _ = w.shape
        return (self.hip_conv and (ci, co, ks) in self._OWN_CONV and w.dtype == torch.float16
                and x.dtype == torch.float16 and m.stride == (1, 1) and m.dilation == (1, 1) and m.groups == 1
                and m.padding[0] == m.padding[1] and m.padding[0] < ks
                and x.is_contiguous(memory_format=torch.channels_last)
                and w.is_contiguous(memory_format=torch.channels_last) and x.shape[0] > 0)

    def _conv_relu(self, x, m):
        """F.relu(m(x)) under autocast; on the GPU with grad, the convolution without its bias and
        _BiasReLU after it (NHWC fp16)"""
        if (self.hip_bias_relu and x.is_cuda and torch.is_grad_enabled() and torch.is_autocast_enabled("cuda") and
                m.bias is not None and m.out_channels % 4 == 0 and m.out_channels <= 1024 and
                m.weight.is_contiguous(memory_format=torch.channels_last)):
            if self.conv_bias_relu and self._own_conv_ok(x, m):
                b = m.bias if m.bias.dtype == torch.float16 else m.bias.to(torch.float16)
                return _HipConv.apply(x, m.weight, m.padding[0], b, self._wt(m))
            y = self._conv_nobias(x, m)
            if y.dtype == torch.float16 and y.is_contiguous(memory_format=torch.channels_last) and y.numel() > 0:
                b = m.bias if m.bias.dtype == torch.float16 else m.bias.to(torch.float16)
                return _BiasReLU.apply(y, b)
            return F.relu(y + m.bias.view(-1, 1, 1))
        return F.relu(m(x))

    def _conv_relu_pool(self, x, m, pool):
        """pool(F.relu(m(x))) under autocast; on the GPU with grad and a 2x2 / stride-2 max-pool, the
        convolution without its bias and _BiasReLUPool after it (NHWC fp16)"""
        ks = pool.kernel_size if isinstance(pool.kernel_size, int) else None
        st = pool.stride if isinstance(pool.stride, int) else None
        if (self.hip_bias_relu and ks == 2 and st == 2 and pool.padding == 0 and pool.dilation == 1 and
                not pool.ceil_mode and x.is_cuda and torch.is_grad_enabled() and torch.is_autocast_enabled("cuda") and
                m.bias is not None and m.out_channels % 4 == 0 and m.out_channels <= 1024 and
                m.weight.is_contiguous(memory_format=torch.channels_last)):
            r = self._conv_nobias(x, m)
            if (r.dtype == torch.float16 and r.is_contiguous(memory_format=torch.channels_last) and r.numel() > 0 and
                    r.shape[2] >= 2 and r.shape[3] >= 2):
                b = m.bias if m.bias.dtype == torch.float16 else m.bias.to(torch.float16)
                return _BiasReLUPool.apply(r, b)
            return pool(F.relu(r + m.bias.view(-1, 1, 1)))
        return pool(self._conv_relu(x, m))

    def _cast_names(self):
        """the parameters autocast would cast to fp16 in the training forward: every Conv2d / Linear
        weight and bias (LayerNorm's stay fp32; token_wA / token_wV are summed in fp32 first)"""
        names = getattr(self, "_cast_names_cache", None)
        if names is None:
            names = [f"{mn}.{pn}" for mn, m in self.named_modules() if isinstance(m, (nn.Conv2d, nn.Linear))
                     for pn, p in m.named_parameters(recurse=False)]
            self._cast_names_cache = names
        return names

    def _flip_names(self, names, own):
        """{conv module name: index in names of its weight} for the layers whose data gradient _HipConv runs
        on its own kernel (SCRIMPNet._OWN_CONV, channels_last weights): their flipped, transposed fp16 copies
        come from _CastParams' launch instead of a flip + copy per backward"""
        if not self.hip_conv:
            return {}
        key = tuple(names)
        cache = self.__dict__.get("_flip_cache")
        if cache is None or cache[0] != key:
            out = {}
            for mn, m in self.named_modules():
                if isinstance(m, nn.Conv2d) and f"{mn}.weight" in names:
                    co, ci, ks, ks2 = m.weight.shape
                    if (ks == ks2 and (ci, co, ks) in self._OWN_CONV and m.stride == (1, 1) and m.groups == 1
                            and m.dilation == (1, 1)):
                        out[mn] = names.index(f"{mn}.weight")
            cache = (key, out)
            self.__dict__["_flip_cache"] = cache
        out = cache[1]
        if not all(own[names[i]].is_contiguous(memory_format=torch.channels_last) for i in out.values()):
            return {}
        return out

    def _next_train_seed(self, x):
        """The training forward's dropout seed for the fused kernels (_DropResLN, _GeluDropout): an int64
        counter in device memory, incremented on the device by every training forward (so a captured
        update draws new masks on every replay; two models built from the same torch seed, or copies,
        draw the same).  None off the GPU training path."""
        if not (x.is_cuda and torch.is_grad_enabled() and torch.is_autocast_enabled("cuda")):
            return None
        t = self.__dict__.get("_train_seed")
        if t is None or t.device != x.device:
            t = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).to(x.device)
            self.__dict__["_train_seed"] = t
        t.add_(1)
        return t

    def weights_updated(self):
        """Forget the acting path's fp16 weight copies: an update replayed from a captured graph
        changes the parameters without bumping their version counters (_half's key)."""
        self._h16.clear()

    def forward(self, obs, vector, input_state=None):
        """Returns (policy, value, blocking, policy_sig, x, policy_logits, cost_value) like net.py:101-155.
        obs: [..., N, C, F, F] (any leading shape); the agent axis is num_agents (EnvParameters.N_AGENTS
        when not given at construction).  Acting on the GPU (no grad): _forward_fused."""
        if self.fused_acting and obs.is_cuda and not torch.is_grad_enabled() and self.cT == 512:
            return self._forward_fused(obs, vector)
        if self.cast_params and obs.is_cuda and torch.is_grad_enabled() and not self._in_cast:
            # the same forward on fp16 copies of the conv / linear weights, made in one launch
            # (autocast would cast each weight on use and its ToCopyBackward each gradient)
            names = self._cast_names()
            own = dict(self.named_parameters())
            flips = self._flip_names(names, own) if self.cast_flips else ()
            p16 = _CastParams.apply(tuple(flips.values()) if flips else (), *[own[n] for n in names])
            self._in_cast = True
            # the flipped weights of _HipConv's data gradients, by module (read in _conv_relu / _conv_nobias)
            self.__dict__["_wt16"] = {self.get_submodule(mn): wt for mn, wt in zip(flips, p16[len(names):])}
            try:
                return torch.func.functional_call(self, dict(zip(names, p16[:len(names)])), (obs, vector, input_state))
            finally:
                self._in_cast = False
                self.__dict__["_wt16"] = {}
        with torch.autocast(device_type=obs.device.type, enabled=obs.device.type == "cuda"):
            n_agents = self.num_agents or EnvParameters.N_AGENTS
            F_ = self.fov or obs.shape[-1]
            x = obs.reshape(-1, self.num_channel, F_, F_)
            if self.conv1.weight.is_contiguous(memory_format=torch.channels_last) and x.is_cuda:
                x = x.contiguous(memory_format=torch.channels_last)
            v = vector.reshape(-1, NetParameters.VECTOR_LEN)
            cr = self._conv_relu
            x = cr(x, self.conv1)
            x = cr(x, self.conv1a)
            x = self._conv_relu_pool(x, self.conv1b, self.pool1)
            x = cr(x, self.conv2)
            x = cr(x, self.conv2a)
            x = self._conv_relu_pool(x, self.conv2b, self.pool2)
            x = cr(x, self.conv3).flatten(1)
            g = F.relu(self.fully_connected_1(v))
            x3 = torch.cat((x, g), -1)
            fc2, fc3 = self.fully_connected_2, self.fully_connected_3
            h = _train_linear(F.relu(_train_linear(x3, fc2.weight, fc2.bias)), fc3.weight, fc3.bias)
            h = F.relu(h + x3).unsqueeze(1)                                   # [b, 1, 512]
            # tokeniser (net.py:124-130): sums over the 8 token matrices, softmax over a length-1 axis
            A = torch.matmul(h, self.token_wA.sum(0).transpose(0, 1))         # [b, 1, 16]
            A = A.transpose(1, 2).softmax(dim=-1)                             # [b, 16, 1]
            VV = torch.matmul(h, self.token_wV.sum(0))                        # [b, 1, 512]
            seed = self._next_train_seed(h)
            enc = self.transformer
            if (seed is not None and self.fused_tokens and enc._train_fused_ok(self.pos_embedding) and
                    A.dtype == torch.float32 and VV.dtype == torch.float16 and A.shape[1:] == (16, 1) and
                    VV.shape[1:] == (1, 512) and tuple(self.pos_embedding.shape) == (1, 17, 512) and
                    self.cls_token.numel() == 512 and self.cls_token.is_contiguous() and
                    self.pos_embedding.is_contiguous()):
                # tokens + dropout + the first PreNorm in one launch (_TokensLN)
                ln = enc.layers[0][0].fn.norm
                start = _TokensLN.apply(A.reshape(-1, 16).contiguous(), VV.reshape(-1, 512).contiguous(),
                                        self.cls_token, self.pos_embedding, ln.weight, ln.bias, ln.eps,
                                        _drop_p(self.dropout), seed, 32)
                x = enc._forward_train_fused(None, True, seed, start=start)
            else:
                T = A * VV                       # [b, 16, 512]: matmul(A, VV) over a length-1 axis
                x = torch.cat((self.cls_token.expand(T.shape[0], -1, -1), T), dim=1) + self.pos_embedding
                x = enc(self.dropout(x), first_only=True, seed=seed)
            ns = self.nn_same
            x = _train_linear(_train_linear(x[:, 0], ns.weight, ns.bias), ns.weight, ns.bias)
            x = x.reshape(-1, n_agents, NetParameters.NET_SIZE)
            logits = self.policy_layer(x)
            policy = logits.softmax(dim=-1)
            policy_sig = torch.sigmoid(logits)
            value = self.value_layer(x)
            cost_value = self.cost_value_layer(x)
            blocking = torch.sigmoid(self.blocking_layer(x))
        return policy, value, blocking, policy_sig, x, logits, cost_value

    # ------------------------------------------------------------ acting fast path
    def _forward_fused(self, obs, vector):
        """forward() for acting (no grad, GPU): the same operations at the same precision
        as forward() under autocast, with the elementwise epilogues in the HIP kernels of
        csrc/mapf_policy.hip -- conv bias + ReLU (+ max-pool) in one pass over each NHWC
        activation, LayerNorm written straight as the fp16 the next linear reads, dropout
        + residual add, GELU + dropout, tokeniser + positional embedding + dropout in one
        pass.  Dropout masks come from the kernels' counter-hash stream (seeded from torch's
        CPU generator), not from torch's."""
        from . import _lib
        lib, chk = _lib.lib(), _lib.check
        dev = obs.device
        st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        ptr = lambda t: ctypes.c_void_p(t.data_ptr())
        seeds = iter(torch.randint(0, 2 ** 62, (16,), dtype=torch.int64).tolist())
        drop = lambda m: float(m.p) if m.training else 0.0
        h16, lin = self._half, self._lin16
        with torch.autocast(device_type="cuda"):
            n_agents = self.num_agents or EnvParameters.N_AGENTS
            F_ = self.fov or obs.shape[-1]
            x = obs.reshape(-1, self.num_channel, F_, F_)
            v = vector.reshape(-1, NetParameters.VECTOR_LEN)

            def conv(x, m, pool=False):        # F.relu(conv(x)) (+ pool): bias and ReLU in the epilogue kernel
                b = h16(m.bias)
                co, ci, ks, _ = m.weight.shape
                if (pool and self.own_conv and (ci, co, ks) in ((128, 128, 3), (256, 256, 2)) and
                        x.is_contiguous(memory_format=torch.channels_last)):
                    # conv + bias + ReLU + 2x2 max-pool in one launch (mapf_conv_nhwc_pool_f16): the
                    # conv's output never reaches HBM
                    p = m.padding[0]
                    B_, _, H_, W_ = x.shape
                    Ho_, Wo_ = H_ + 2 * p - ks + 1, W_ + 2 * p - ks + 1
                    yp = torch.empty((B_, co, Ho_ // 2, Wo_ // 2), dtype=torch.float16, device=dev,
                                     memory_format=torch.channels_last)
                    rc = lib.mapf_conv_nhwc_pool_f16(ptr(x), ptr(h16(m.weight, "ohwi")), ptr(b), ptr(yp), B_, H_, W_,
                                                     ci, co, ks, p, st)
                    if rc == 0:
                        return yp
                if self.own_conv and (ci, co, ks) in self._OWN_CONV and x.is_contiguous(memory_format=torch.channels_last):
                    # the MFMA implicit GEMM (csrc/mapf_conv.hip); bias + ReLU in its epilogue unless pooled
                    p = m.padding[0]
                    B_, _, H_, W_ = x.shape
                    y = torch.empty((B_, co, H_ + 2 * p - ks + 1, W_ + 2 * p - ks + 1), dtype=torch.float16,
                                    device=dev, memory_format=torch.channels_last)
                    chk(lib.mapf_conv_nhwc_f16(ptr(x), ptr(h16(m.weight, "ohwi")), ptr(b), ptr(y), B_, H_, W_, ci, co,
                                               ks, p, 0 if pool else 1, st))
                    if not pool:
                        return y
                elif (self.own_conv and m.padding[0] == 0 and x.shape[2] == ks and x.shape[3] == ks
                      and x.is_contiguous(memory_format=torch.channels_last)):
                    # a kernel covering its whole input (conv3: 3x3 on 3x3 -> 1x1) is a plain GEMM over
                    # the NHWC pixel, K ordered (ky, kx, c): [B, KS*KS*Cin] x [Cout, KS*KS*Cin]^T
                    B_ = x.shape[0]
                    y = F.linear(x.permute(0, 2, 3, 1).reshape(B_, -1), h16(m.weight, "ohwi2d"))
                    chk(lib.mapf_nhwc_bias_relu(ptr(y), ptr(b), B_, co, st))
                    return y.view(B_, co, 1, 1)
                else:
                    y = F.conv2d(x, h16(m.weight), None, m.stride, m.padding).contiguous(memory_format=torch.channels_last)
                B_, C_, H_, W_ = y.shape
                if pool:
                    out = torch.empty((B_, C_, H_ // 2, W_ // 2), dtype=y.dtype, device=dev,
                                      memory_format=torch.channels_last)
                    chk(lib.mapf_nhwc_bias_relu_pool2(ptr(y), ptr(b), ptr(out), B_, H_, W_, C_, st))
                    return out
                chk(lib.mapf_nhwc_bias_relu(ptr(y), ptr(b), B_ * H_ * W_, C_, st))
                return y
            # (a pooled layer's raw output takes bias + ReLU + pool in one pass: mapf_nhwc_bias_relu_pool2)

            xin = obs.reshape(-1, self.num_channel, F_, F_)
            if (self.own_conv and self.num_channel <= 7 and self.conv1.weight.shape[0] == 128 and
                    xin.dtype == torch.float32 and xin.is_contiguous()):
                # conv1 from the fp32 NCHW observation: cast, im2col, MFMA, bias + ReLU in one launch
                x1 = torch.empty((xin.shape[0], 128, F_, F_), dtype=torch.float16, device=dev,
                                 memory_format=torch.channels_last)
                chk(lib.mapf_conv_first_f32(ptr(xin), ptr(h16(self.conv1.weight, "k64")), ptr(h16(self.conv1.bias)),
                                            ptr(x1), xin.shape[0], self.num_channel, F_, F_, 128, st))
            else:
                x1 = conv(x.contiguous(memory_format=torch.channels_last), self.conv1)
            x = conv(conv(x1, self.conv1a), self.conv1b, pool=True)
            x = conv(conv(conv(x, self.conv2), self.conv2a), self.conv2b, pool=True)
            x = conv(x, self.conv3).flatten(1)
            g = F.relu(lin(self.fully_connected_1, v))
            x3 = torch.cat((x, g), -1)
            h = lin(self.fully_connected_3, F.relu(lin(self.fully_connected_2, x3)))
            h = F.relu(h + x3).unsqueeze(1)                                   # [b, 1, 512]
            b = h.shape[0]
            hf = h.reshape(b, self.cT)                                        # 2-D GEMMs, not [b,1,512] bmm
            A = torch.matmul(hf, h16(self.token_wA, "sumT")).unsqueeze(-1).softmax(dim=-1)
            A = A.reshape(b, self.L).float().contiguous()                     # [b, 16] (all ones: length-1 softmax)
            VV = torch.matmul(hf, h16(self.token_wV, "sum")).contiguous()      # [b, 512] fp16
            xt = torch.empty(b, self.L + 1, self.cT, dtype=torch.float32, device=dev)
            cls, pos = self.cls_token.detach().contiguous(), self.pos_embedding.detach().contiguous()
            y0 = tok = None
            if self.fused_residual_ln:                     # tokens + the first LayerNorm in one pass
                norm = self.transformer.layers[0][0].fn.norm
                y0 = torch.empty(xt.shape, dtype=torch.float16, device=dev)
                # the first block's fused out-projection recomputes the tokens (same mask bits): their
                # fp32 copy is then never written nor read back (mapf_linear512_tokens_residual_layernorm)
                layers = self.transformer.layers
                recompute = (self.fused_linear and self.cT == 512 and len(layers) >= 2 and
                             layers[0][0].fn.fn.nn1.weight.shape == (512, 512))
                p_tok, seed_tok = drop(self.dropout), next(seeds)
                chk(lib.mapf_tokens_layernorm(None if recompute else ptr(xt), ptr(A), ptr(VV), ptr(cls), ptr(pos), b,
                                              self.L, self.cT, p_tok, seed_tok, ptr(norm.weight), ptr(norm.bias),
                                              float(norm.eps), ptr(y0), st))
                if recompute:
                    tok = (A, VV, cls, pos, p_tok, seed_tok)
            else:
                chk(lib.mapf_tokens(ptr(xt), ptr(A), ptr(VV), ptr(cls), ptr(pos), b, self.L, self.cT,
                                    drop(self.dropout), next(seeds), st))
            x = self._encoder_fused(xt, lib, chk, st, ptr, seeds, drop, y0, tok)[:, 0]
            x = lin(self.nn_same, lin(self.nn_same, x))
            x = x.reshape(-1, n_agents, NetParameters.NET_SIZE)
            logits = self.policy_layer(x)
            policy = logits.softmax(dim=-1)
            policy_sig = torch.sigmoid(logits)
            value = self.value_layer(x)
            cost_value = self.cost_value_layer(x)
            blocking = torch.sigmoid(self.blocking_layer(x))
        return policy, value, blocking, policy_sig, x, logits, cost_value

    _HALF_VIEWS = {"sumT": lambda t: t.sum(0).transpose(0, 1), "sum": lambda t: t.sum(0),
                   "ohwi": lambda t: t.permute(0, 2, 3, 1),        # conv weight for mapf_conv_nhwc_f16
                   "ohwi2d": lambda t: t.permute(0, 2, 3, 1).reshape(t.shape[0], -1),   # ... as a GEMM operand
                   "k64": lambda t: F.pad(t.reshape(t.shape[0], -1), (0, 64 - t[0].numel())),   # mapf_conv_first_f32
                   "q": lambda t: t[:t.shape[0] // 3], "kv": lambda t: t[t.shape[0] // 3:]}

    def _half(self, t, view=None):
        """fp16 copy of parameter t (or of a fixed view of it) for the acting forward, kept
        until t changes in place (optimizer step, load_state_dict bump its version) --
        autocast would re-cast every weight on every forward."""
        key = (id(t), view)
        ver = (t._version, t.data_ptr())
        hit = self._h16.get(key)
        if hit is None or hit[0] != ver:
            src = self._HALF_VIEWS[view](t) if view else t
            hit = (ver, src.detach().to(torch.float16).contiguous())
            self._h16[key] = hit
        return hit[1]

    def _lin16(self, m, x):
        return F.linear(x, self._half(m.weight), None if m.bias is None else self._half(m.bias))

    def _encoder_fused(self, x, lib, chk, st, ptr, seeds, drop, y0=None, tok=None):
        """self.transformer(x, first_only=True) on the fused epilogues; x fp32 [b, n, d] is
        updated in place (the residual stream) and token 0 after the last block returned; y0 is
        the first block's LayerNorm of x when the caller already computed it; tok = (A, VV, cls,
        pos, p, seed) when x was NOT written and the first fused out-projection recomputes it."""
        layers = self.transformer.layers
        b, n, d = x.shape
        h16, lin = self._half, self._lin16

        def ln(x, norm):                        # LayerNorm -> the fp16 the next linear reads
            y = torch.empty(x.shape, dtype=torch.float16, device=x.device)
            chk(lib.mapf_layernorm_f16(ptr(x), d, ptr(norm.weight), ptr(norm.bias), ptr(y), x.numel() // d, d,
                                       float(norm.eps), st))
            return y

        def residual(x, y, m, norm=None):       # x += dropout(y); then LayerNorm(x) -> fp16 if norm
            y = y.contiguous()
            if norm is None or not self.fused_residual_ln:
                chk(lib.mapf_dropout_residual(ptr(x), ptr(y), x.numel(), drop(m), next(seeds), st))
                return None if norm is None else ln(x, norm)
            z = torch.empty(x.shape, dtype=torch.float16, device=x.device)
            chk(lib.mapf_dropout_residual_layernorm(ptr(x), ptr(y), ptr(norm.weight), ptr(norm.bias), ptr(z),
                                                    x.numel() // d, d, float(norm.eps), drop(m), next(seeds), st))
            return z

        fused_lin = self.fused_linear and d == 512 and self.fused_residual_ln

        def lin_residual(m, inp, x, drop_m, norm, tok=None, x_every=1):   # x += dropout(m(inp)); LayerNorm(x)
            if not fused_lin or norm is None or m.weight.shape != (512, 512):
                assert tok is None
                return residual(x, lin(m, inp), drop_m, norm)
            inp = inp.contiguous()
            z = torch.empty(x.shape, dtype=torch.float16, device=x.device)
            if tok is not None:                         # x = tokens (recomputed) + dropout(m(inp))
                A, VV, cls, pos, p_tok, seed_tok = tok
                chk(lib.mapf_linear512_tokens_residual_layernorm(
                    ptr(inp), ptr(h16(m.weight)), ptr(h16(m.bias)), ptr(x), ptr(norm.weight), ptr(norm.bias), ptr(z),
                    x.shape[0], x.shape[1] - 1, float(norm.eps), drop(drop_m), next(seeds), ptr(A), ptr(VV), ptr(cls),
                    ptr(pos), p_tok, seed_tok, st))
                return z
            if x_every > 1:                             # only token 0's residual rows are read again
                chk(lib.mapf_linear512_residual_layernorm_rows(
                    ptr(inp), ptr(h16(m.weight)), ptr(h16(m.bias)), ptr(x), ptr(norm.weight), ptr(norm.bias), ptr(z),
                    x.numel() // d, float(norm.eps), drop(drop_m), next(seeds), x_every, st))
                return z
            chk(lib.mapf_linear512_residual_layernorm(ptr(inp), ptr(h16(m.weight)), ptr(h16(m.bias)), ptr(x),
                                                      ptr(norm.weight), ptr(norm.bias), ptr(z), x.numel() // d,
                                                      float(norm.eps), drop(drop_m), next(seeds), st))
            return z

        def lin_gelu(m, inp, drop_m):                   # dropout(gelu(m(inp))), one launch
            if not fused_lin or m.weight.shape != (512, 512):
                hid = lin(m, inp).contiguous()
                chk(lib.mapf_gelu_dropout_f16(ptr(hid), hid.numel(), drop(drop_m), next(seeds), st))
                return hid
            inp = inp.contiguous()
            hid = torch.empty(inp.shape[:-1] + (512,), dtype=torch.float16, device=inp.device)
            chk(lib.mapf_linear512_gelu_dropout(ptr(inp), ptr(h16(m.weight)), ptr(h16(m.bias)), ptr(hid),
                                                inp.numel() // 512, drop(drop_m), next(seeds), st))
            return hid

        def attend(q, k, v, rows, q_ts, kv_ts, a):     # fp16 [b, rows, d], heads concatenated
            o = torch.empty(b, rows, d, dtype=torch.float16, device=x.device)
            chk(lib.mapf_attention_f16(ptr(q), ptr(k), ptr(v), ptr(o), b, n, rows, q_ts, q_ts * (n if rows > 1 else 1),
                                       kv_ts, kv_ts * n, a.heads, d // a.heads, float(a.scale), st))
            return o

        y = ln(x, layers[0][0].fn.norm) if y0 is None else y0
        for li, (att, ff) in enumerate(layers):
            a = att.fn.fn
            hh = a.heads
            f = ff.fn.fn
            own_attn = self.fused_attention and hh * 32 == d == 512 and n <= 17
            if li < len(layers) - 1:
                qkv = lin(a.to_qkv, y)
                if own_attn:
                    assert qkv.dtype == torch.float16 and qkv.is_contiguous()
                    out = attend(qkv, qkv[..., d:], qkv[..., 2 * d:], n, 3 * d, 3 * d, a)
                else:
                    qkv = qkv.view(b, n, 3, hh, d // hh).permute(2, 0, 3, 1, 4)
                    out = F.scaled_dot_product_attention(qkv[0], qkv[1], qkv[2], scale=a.scale)
                    out = out.transpose(1, 2).reshape(b, n, d)
                yf = lin_residual(a.nn1, out, x, a.do1, ff.fn.norm, tok if li == 0 else None)
            else:                               # the last block: token 0's query only (see _Encoder)
                w, bias = a.to_qkv.weight, a.to_qkv.bias
                q = F.linear(y[:, 0], h16(w, "q"), h16(bias, "q"))
                kv = F.linear(y, h16(w, "kv"), h16(bias, "kv"))
                if own_attn:
                    assert q.dtype == kv.dtype == torch.float16 and q.is_contiguous() and kv.is_contiguous()
                    out = attend(q, kv, kv[..., d:], 1, d, 2 * d, a)
                else:
                    q = q.view(b, 1, hh, d // hh).transpose(1, 2)
                    kv = kv.view(b, n, 2, hh, d // hh).permute(2, 0, 3, 1, 4)
                    out = F.scaled_dot_product_attention(q, kv[0], kv[1], scale=a.scale)
                    out = out.transpose(1, 2).reshape(b, 1, d)
                x = x[:, :1].contiguous()
                yf = lin_residual(a.nn1, out, x, a.do1, ff.fn.norm)
            hid = lin_gelu(f.nn1, yf, f.do1)
            # before the last block only token 0 of the stream is carried on (x[:, :1] below)
            y = lin_residual(f.nn2, hid, x, f.do2, layers[li + 1][0].fn.norm if li + 1 < len(layers) else None,
                             x_every=n if li + 2 == len(layers) and x.shape[1] == n else 1)
        return x
