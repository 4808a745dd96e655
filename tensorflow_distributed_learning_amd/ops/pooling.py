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
