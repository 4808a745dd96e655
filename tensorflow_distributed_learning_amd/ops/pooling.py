"""NHWC max pooling on the hand-written kernels (csrc/kernels/pool.hip).

``max_pool_nhwc(x, pool, strides, pads, pad_zero)``: ``pads = ((top, bottom), (left, right))`` of
implicit padding; ``pad_zero`` makes padding elements zeros (a fused ``ZeroPadding2D`` in front,
keras/fusion.py) instead of -inf (TF 'same' max pooling).  GPU tensors with C % 8 == 0 run the HIP
kernels; everything else runs PyTorch with the same semantics.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import hip


def supported(x: torch.Tensor) -> bool:
    return x.is_cuda and x.dim() == 4 and x.shape[-1] % 8 == 0 and x.shape[-1] <= 2048 and \
        x.dtype in (torch.float32, torch.bfloat16)


def _out(i, k, s, p0, p1):
    return (i + p0 + p1 - k) // s + 1


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kh, kw, sh, sw, pads, pad_zero):
        C = hip()
        xc = x.contiguous()
        if xc.data_ptr() % 16:
            xc = xc.clone()
        (pt, pb), (pl, pr) = pads
        OH, OW = _out(xc.shape[1], kh, sh, pt, pb), _out(xc.shape[2], kw, sw, pl, pr)
        y, arg = C.maxpool_fwd(xc, kh, kw, sh, sw, pt, pl, OH, OW, bool(pad_zero))
        ctx.save_for_backward(arg)
        ctx.geo = (list(xc.shape), kh, kw, sh, sw, pt, pl)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = hip()
        (arg,) = ctx.saved_tensors
        shape, kh, kw, sh, sw, pt, pl = ctx.geo
        dy = dy.contiguous()
        if dy.data_ptr() % 16:
            dy = dy.clone()
        return C.maxpool_bwd(dy, arg, shape, kh, kw, sh, sw, pt, pl), None, None, None, None, None, None


def max_pool_nhwc(x, pool, strides, pads=((0, 0), (0, 0)), pad_zero=False):
    kh, kw = pool
    sh, sw = strides
    if supported(x):
        return _MaxPool.apply(x, kh, kw, sh, sw, pads, pad_zero)
    (pt, pb), (pl, pr) = pads
    h = x.permute(0, 3, 1, 2)
    if pt or pb or pl or pr:
        h = F.pad(h, (pl, pr, pt, pb), value=0.0 if pad_zero else float("-inf"))
    return F.max_pool2d(h, (kh, kw), (sh, sw)).permute(0, 2, 3, 1)


def bn_pool_supported(x: torch.Tensor) -> bool:
    """The BN -> ReLU -> max-pool fusion: HIP dtype / layout, and C / 8 a power of two <= 256."""
    g = x.shape[-1] // 8 if x.dim() == 4 else 0
    return supported(x) and g > 0 and (g & (g - 1)) == 0 and g <= 256


class _BnReluMaxPool(torch.autograd.Function):
    """relu(batch_norm(x)) -> max pool in one forward pass over x (the normalised tensor is never
    written) and one backward pass that also reduces the BN backward sums (keras/fusion.py: the
    ResNet stem's BN -> ReLU -> ZeroPadding2D -> MaxPooling2D)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, conv_bias, moving_mean, moving_var, momentum, eps, kh, kw, sh, sw, pads,
                pad_zero, grad_out, part):
        C = hip()
        xc = x.contiguous()
        if xc.data_ptr() % 16:
            xc = xc.clone()
        st = C.bn_stats_train(xc, gamma, beta, moving_mean, moving_var, float(momentum), float(eps),
                              conv_bias.detach() if conv_bias is not None else None, part)
        (pt, pb), (pl, pr) = pads
        OH, OW = _out(xc.shape[1], kh, sh, pt, pb), _out(xc.shape[2], kw, sw, pl, pr)
        y, arg = C.maxpool_fwd(xc, kh, kw, sh, sw, pt, pl, OH, OW, bool(pad_zero), st)
        ctx.save_for_backward(xc, gamma if gamma is not None else st, st, arg,
                              conv_bias if conv_bias is not None else st)
        ctx.geo = (list(xc.shape), kh, kw, sh, sw, pt, pl)
        ctx.flags = (gamma is not None, conv_bias is not None)
        ctx.grad_out = grad_out
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import batchnorm as _bn

        C = hip()
        xc, gamma, st, arg, conv_bias = ctx.saved_tensors
        has_g, has_cb = ctx.flags
        shape, kh, kw, sh, sw, pt, pl = ctx.geo
        dy = dy.to(xc.dtype).contiguous()
        if dy.data_ptr() % 16:
            dy = dy.clone()
        dz, part = C.maxpool_bwd_bn(dy, arg, shape, kh, kw, sh, sw, pt, pl, xc, st)
        go = ctx.grad_out or (None, None)
        _bn.FUSED_BWD[0] += 1
        _bn.FUSED_BWD_MODES[1] += 1
        dx, dgamma, dbeta = C.bn_backward(dz, xc, None, gamma if has_g else None, st, 1, go[0], go[1], part)[:3]
        dcb = torch.zeros_like(conv_bias) if (has_cb and ctx.needs_input_grad[3]) else None
        return (dx, dgamma if ctx.needs_input_grad[1] else None, dbeta if ctx.needs_input_grad[2] else None, dcb,
                None, None, None, None, None, None, None, None, None, None, None, None)


def bn_relu_max_pool(x, gamma, beta, moving_mean, moving_var, momentum, eps, pool, strides, pads, pad_zero,
                     conv_bias=None, grad_out=None, part=None):
    """``max_pool_nhwc(relu(batch_norm_train(x, ...)), ...)`` with the normalisation applied inside the
    pooling kernel (see :class:`_BnReluMaxPool`); the caller checked :func:`bn_pool_supported`.
    ``grad_out`` / ``part`` / ``conv_bias``: as for ops/batchnorm.py ``batch_norm_train``."""
    if grad_out is not None:
        gamma = gamma.detach() if gamma is not None else None
        beta = beta.detach() if beta is not None else None
    return _BnReluMaxPool.apply(x, gamma, beta, conv_bias, moving_mean, moving_var, momentum, eps, pool[0], pool[1],
                                strides[0], strides[1], pads, pad_zero, grad_out, part)
