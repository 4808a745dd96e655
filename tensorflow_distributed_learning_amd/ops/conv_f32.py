"""Generic f32 convolution and Dense on the hand-written f32-MFMA kernels (csrc/kernels/gemm_f32.hip).

The bf16 kernels of ops/conv.py and ops/dense.py cover the shapes of the mixed-precision models
(channels in multiples of 64, symmetric padding, the 1x1 stride-2 and stride-1 input gradients).
Everything else -- the f32 layers of the reference CNN in the generic engine (``Conv2D(32, 3)`` over a
1-channel image, ``padding='same'`` variants, Dense in f32), asymmetric 'same' padding, dilation,
strided 3x3 input gradients, weight gradients with >= 2^24 reduction rows -- runs here instead of
on MIOpen / hipBLASLt: one implicit-GEMM kernel family on ``v_mfma_f32_16x16x4_f32`` (exact f32
products) with per-mode operand gathers, deterministic split-K for the long reductions.

Reference: ``tf.keras.layers.Conv2D`` / ``Dense`` of tf_dist_example.py:41-47 (Keras semantics:
NHWC activations, HWIO kernels, [in, out] Dense kernels).
"""
from __future__ import annotations

import torch

from . import hip


def _c32(t: torch.Tensor) -> torch.Tensor:
    t = t.float().contiguous()
    return t if t.data_ptr() % 16 == 0 else t.clone()


def supported(x: torch.Tensor, groups: int = 1) -> bool:
    """Any 4-D NHWC GPU activation of a floating dtype, ungrouped."""
    return (x.is_cuda and x.dim() == 4 and x.dtype in (torch.float32, torch.bfloat16, torch.float16)
            and int(groups) == 1)


def out_size(i, k, s, d, p0, p1):
    return (i + p0 + p1 - (k - 1) * d - 1) // s + 1


def fwd(x, w_hwio, bias, stride, pads, dil=(1, 1), act=0) -> torch.Tensor:
    """f32 ``y = conv(x, w) + bias`` (``act=1``: ReLU in the epilogue); ``pads = (top, bottom, left, right)``."""
    R, S = w_hwio.shape[0], w_hwio.shape[1]
    oh = out_size(x.shape[1], R, stride[0], dil[0], pads[0], pads[1])
    ow = out_size(x.shape[2], S, stride[1], dil[1], pads[2], pads[3])
    b = _c32(bias) if bias is not None else None
    return hip().conv_f32_fwd(_c32(x), _c32(w_hwio), b, oh, ow, stride[0], stride[1], pads[0], pads[2], dil[0], dil[1],
                              act=int(act))


def dgrad(dy, w_hwio, hw, stride, pads, dil=(1, 1), dy_mask=None, pin=None) -> torch.Tensor:
    """f32 input gradient of :func:`fwd` for an input of spatial size ``hw`` (``dy_mask``: the ReLU
    output whose mask applies to ``dy``).  ``pin = (argmax, out_h, out_w)``: ``dy`` is the gradient of a
    2x2 max pool over the conv's ReLU output and ``dy_mask`` the pooled maximum (conv2d_pool's backward:
    the loader routes and masks it, no max-pool backward pass)."""
    kw = dict(pin_arg=pin[0], out_h=pin[1], out_w=pin[2]) if pin is not None else {}
    import os

    if w_hwio.numel() <= int(os.environ.get("TDL_F32_DGRAD_HWIO_MAX", 1 << 16)):
        # small kernels (the generic engine's layers): read w HWIO transposed in the kernel (w_hwio), no
        # [R][S][K][C] copy kernel per step; large ones keep the copy for 16-B operand loads
        return hip().conv_f32_dgrad(_c32(dy), _c32(w_hwio), hw[0], hw[1], stride[0], stride[1], pads[0], pads[2],
                                    dil[0], dil[1], dy_mask=dy_mask, w_hwio=True, **kw)
    wt = _c32(w_hwio).permute(0, 1, 3, 2).contiguous()  # [R][S][K][C]
    return hip().conv_f32_dgrad(_c32(dy), wt, hw[0], hw[1], stride[0], stride[1], pads[0], pads[2], dil[0], dil[1],
                                dy_mask=dy_mask, **kw)


def wgrad(x, dy, rs, stride, pads, dil=(1, 1), out=None, accumulate=False, dy_mask=None, dbias=None,
          pin=None) -> torch.Tensor:
    """f32 HWIO weight gradient of :func:`fwd` (added into the f32 ``out`` when ``accumulate``); with
    ``dbias`` the bias gradient comes from the same kernel (a column of ones appended to the gathered
    input: no separate reduction).  ``pin``: as for :func:`dgrad`."""
    kw = dict(pin_arg=pin[0], out_h=pin[1], out_w=pin[2]) if pin is not None else {}
    return hip().conv_f32_wgrad(_c32(x), _c32(dy), rs[0], rs[1], stride[0], stride[1], pads[0], pads[2], dil[0],
                                dil[1], out=out, accumulate=accumulate, dy_mask=dy_mask, dbias=dbias, **kw)


class _ConvF32(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, pads, dil, grad_out, anchor=None, act=0, gb_out=None):
        y = fwd(x, w, b, stride, pads, dil, act)
        ctx.save_for_backward(x, w, y if act else None)
        ctx.geo = (stride, pads, dil)
        ctx.has_b = b is not None
        ctx.grad_out, ctx.gb_out = grad_out, gb_out
        ctx.dtypes = (x.dtype, w.dtype)
        return y.to(x.dtype)

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        return _conv_backward(ctx, x, w, y, _c32(dy))


def _conv_backward(ctx, x, w, y, dy, pin=None, unpool=None):
    """Input / weight / bias gradients of :func:`fwd` from the f32 output gradient ``dy`` (``y``: the saved
    ReLU output whose mask applies, or None).  ``pin``: ``dy`` / ``y`` are the pooled gradient / maximum
    of conv2d_pool (see :func:`dgrad`); ``unpool()`` then gives the plain conv-output gradient and ReLU
    output for the one path the kernels do not cover (a bias gradient without a weight gradient)."""
    stride, pads, dil = ctx.geo
    dx = dw = db = None
    if ctx.needs_input_grad[0]:
        dx = dgrad(dy, w, (x.shape[1], x.shape[2]), stride, pads, dil, dy_mask=y, pin=pin).to(ctx.dtypes[0])
    rs = (w.shape[0], w.shape[1])
    want_db = ctx.has_b and (ctx.gb_out is not None or ctx.needs_input_grad[2])
    if ctx.grad_out is not None:
        # slab targets: dW (and db, from the same kernel) added in place
        dbt = ctx.gb_out if ctx.gb_out is not None else (
            torch.zeros(w.shape[-1], dtype=torch.float32, device=dy.device) if want_db else None)
        wgrad(x, dy, rs, stride, pads, dil, out=ctx.grad_out, accumulate=True, dy_mask=y, dbias=dbt, pin=pin)
        if ctx.gb_out is None and want_db:
            db = dbt
    elif ctx.needs_input_grad[1]:
        dbt = torch.empty(w.shape[-1], dtype=torch.float32, device=dy.device) if want_db else None
        dw = wgrad(x, dy, rs, stride, pads, dil, dy_mask=y, dbias=dbt, pin=pin).to(ctx.dtypes[1])
        db = dbt
    elif want_db:
        if pin is not None:
            dy, y = unpool()
        g = dy.float() if y is None else dy.float() * (y > 0)
        if ctx.gb_out is not None:
            ctx.gb_out.add_(g.sum((0, 1, 2)))
        else:
            db = g.sum((0, 1, 2))
    return dx, dw, db, None, None, None, None, None, None, None


class _ConvPoolF32(torch.autograd.Function):
    """conv (+ bias, + ReLU) followed by a 2x2 / stride-2 'valid' max pool: ONE forward launch (the pool in
    the GEMM epilogue, conv_f32_fwd_pool); the backward is the pool's (maxpool_bwd over the epilogue's
    argmax) and then the conv's, exactly as the unfused pair."""

    @staticmethod
    def forward(ctx, x, w, b, stride, pads, dil, grad_out, anchor=None, act=0, gb_out=None):
        R, S = w.shape[0], w.shape[1]
        oh = out_size(x.shape[1], R, stride[0], dil[0], pads[0], pads[1])
        ow = out_size(x.shape[2], S, stride[1], dil[1], pads[2], pads[3])
        bb = _c32(b) if b is not None else None
        y, p, arg = hip().conv_f32_fwd_pool(_c32(x), _c32(w), bb, oh, ow, stride[0], stride[1], pads[0], pads[2],
                                            dil[0], dil[1], act=int(act))
        ctx.save_for_backward(x, w, y if act else None, arg, p if act else None)
        ctx.geo = (stride, pads, dil)
        ctx.yshape = list(y.shape)
        ctx.has_b = b is not None
        ctx.grad_out, ctx.gb_out = grad_out, gb_out
        ctx.dtypes = (x.dtype, w.dtype)
        return p.to(x.dtype)

    @staticmethod
    def backward(ctx, dp):
        import os

        x, w, y, arg, p = ctx.saved_tensors
        dp = _c32(dp)

        def unpool():
            return _c32(hip().maxpool_bwd(dp, arg, ctx.yshape, 2, 2, 2, 2, 0, 0)), y

        if y is not None and os.environ.get("TDL_FUSE_CONV_POOL_BWD", "0") == "1":
            # the input / weight gradient kernels read the POOLED gradient and route it through the argmax
            # (and the ReLU mask: maximum > 0) in their operand loaders: no max-pool backward pass.  Off by
            # default: the per-element window decode and argmax loads cost the weight-gradient kernels
            # ~4-5 us each, more than the two pool-backward launches they replace (+1.7 % per step,
            # profiles/generic_engine_r6.txt)
            return _conv_backward(ctx, x, w, p, dp, pin=(arg, ctx.yshape[1], ctx.yshape[2]), unpool=unpool)
        dy, _ = unpool()
        return _conv_backward(ctx, x, w, y, dy)


def conv_pool_supported(x: torch.Tensor, oh: int, ow: int, k: int) -> bool:
    """The fused conv + 2x2 max pool forward (generic engine): f32 GPU activations, an output of at
    least one window, a channel count the pool backward kernel takes (multiple of 8, <= 2048)."""
    return (x.is_cuda and x.dim() == 4 and x.dtype == torch.float32 and oh >= 2 and ow >= 2 and k % 8 == 0
            and k <= 2048)


def conv2d_pool(x, w_hwio, bias=None, stride=(1, 1), pads=(0, 0, 0, 0), dil=(1, 1), grad_out=None, anchor=None,
                act=0, gb_out=None):
    """``max_pool_2x2(act(conv(x, w) + bias))`` with the pool fused into the convolution's launch (see
    :func:`conv2d` for the arguments)."""
    return _ConvPoolF32.apply(x, w_hwio, bias, tuple(int(s) for s in stride), tuple(int(p) for p in pads),
                              tuple(int(d) for d in dil), grad_out, anchor, int(act), gb_out)


def conv2d(x, w_hwio, bias=None, stride=(1, 1), pads=(0, 0, 0, 0), dil=(1, 1), grad_out=None, anchor=None, act=0,
           gb_out=None):
    """``conv(x NHWC, w HWIO) + bias`` with zero padding ``pads = (top, bottom, left, right)``, computed
    in f32 (bf16 / f16 operands are widened), returned in x's dtype.  ``act=1``: ReLU fused into the
    epilogue and, in the backward, into the operand loads of the input- and weight-gradient kernels
    (the mask comes from the saved output).  ``grad_out`` / ``gb_out``: f32 slab views the weight /
    bias gradients are ADDED into (``w`` / ``bias`` then need no autograd; ``anchor`` -- the variable's
    leaf -- keeps the backward alive when nothing else needs a gradient, as in ops/conv.py)."""
    return _ConvF32.apply(x, w_hwio, bias, tuple(int(s) for s in stride), tuple(int(p) for p in pads),
                          tuple(int(d) for d in dil), grad_out, anchor, int(act), gb_out)


# ------------------------------------------------------------------------------------------ Dense
def dense_supported(x: torch.Tensor) -> bool:
    return x.is_cuda and x.dtype == torch.float32 and x.dim() >= 2


class _DenseF32(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, targets, anchor=None, act=0):
        C = hip()
        x2 = _c32(x.reshape(-1, x.shape[-1]))
        wc = _c32(w)
        y = C.gemm_f32(x2, 0, wc, 1, bias=_c32(b) if b is not None else None, act=int(act))
        ctx.save_for_backward(x2, wc, y if act else None)
        ctx.has_b = b is not None
        ctx.targets = targets
        ctx.xshape = x.shape
        return y.reshape(*x.shape[:-1], w.shape[1])

    @staticmethod
    def backward(ctx, dy):
        C = hip()
        x, w, y = ctx.saved_tensors
        dy = _c32(dy.reshape(-1, dy.shape[-1]))
        dx = C.gemm_f32(dy, 0, w, 0, amask=y).reshape(ctx.xshape) if ctx.needs_input_grad[0] else None
        gw_t, gb_t = ctx.targets if ctx.targets is not None else (None, None)
        dw = db = None
        want_db = ctx.has_b and (gb_t is not None or ctx.needs_input_grad[2])
        if gw_t is not None:
            # dW (+ db as an appended row of ones) added straight into the slab views
            dbt = gb_t if gb_t is not None else (
                torch.zeros(w.shape[1], dtype=torch.float32, device=dy.device) if want_db else None)
            C.gemm_f32(x, 1, dy, 1, out=gw_t, accumulate=True, bmask=y, dbias=dbt)
            if gb_t is None and want_db:
                db = dbt
        elif ctx.needs_input_grad[1]:
            dbt = torch.empty(w.shape[1], dtype=torch.float32, device=dy.device) if want_db else None
            dw = C.gemm_f32(x, 1, dy, 1, bmask=y, dbias=dbt)
            db = dbt
        elif want_db:
            s = (dy if y is None else dy * (y > 0)).sum(0)
            if gb_t is not None:
                gb_t.add_(s)
            else:
                db = s
        return dx, dw, db, None, None, None


def dense(x, w, b=None, targets=None, anchor=None, act=0):
    """f32 ``x [..., in] @ w [in, out] (+ b)`` on the f32-MFMA GEMM; ``targets = (dW, db)`` f32 slab views
    the gradients are added into (as ops/dense.py ``dense_bf16``); ``act=1``: ReLU fused (epilogue
    forward; operand masks of the input- and weight-gradient GEMMs backward, the bias gradient as a
    row of ones in the weight-gradient GEMM)."""
    return _DenseF32.apply(x, w, b, targets, anchor, int(act))
