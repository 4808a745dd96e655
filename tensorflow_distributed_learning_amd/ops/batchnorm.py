"""Training-mode batch normalisation on the hand-written NHWC kernels (csrc/kernels/bn.hip).

``batch_norm_train(x, gamma, beta, moving_mean, moving_var, momentum, eps, relu, residual,
conv_bias)`` normalises the last axis of a ``[..., C]`` tensor with its batch statistics, updates
the moving statistics in place (Keras momentum convention; unbiased moving variance) and fuses the
neighbours the functional-model executor hands it (keras/models.py ``_fusion_plan``):

* ``relu=True``                   : BN -> ReLU
* ``residual=r, relu=True``       : BN -> Add(r) -> ReLU (ResNet block tail)
* ``conv_bias=b``                 : the preceding Conv2D's bias, folded in.  In training mode a
  per-channel bias before BN only shifts the batch mean, so the output is unchanged, the moving mean
  gets ``+ b`` and the bias gradient is exactly zero (returned as zeros).

On a GPU tensor the HIP kernels are the only path (:func:`..ops.hip` raises if the extension is not
built); CPU tensors use PyTorch ops with the same semantics.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn.functional as F

from . import hip


FUSED_BWD = [0]  # backward calls that took their reduction from a conv epilogue (tests)
FUSED_BWD_MODES = {0: 0, 1: 0, 2: 0}  # the same, by mode (0 plain, 1 relu, 2 add+relu)


def supported(x: torch.Tensor) -> bool:
    C = x.shape[-1]
    return x.is_cuda and x.dim() >= 2 and C % 8 == 0 and C <= 2048 and x.dtype in (torch.float32, torch.bfloat16)


def _aligned(t: torch.Tensor) -> torch.Tensor:
    t = t.contiguous()
    return t if t.data_ptr() % 16 == 0 else t.clone()


_DEBUG_SEEN = set()


def _debug(*key):
    """TDL_BN_DEBUG=1: name each (direction, shape, mode, fused) combination once on stderr (which
    BN layers still take a separate statistics / gradient-sum pass)."""
    if os.environ.get("TDL_BN_DEBUG") == "1" and key not in _DEBUG_SEEN:
        import sys

        _DEBUG_SEEN.add(key)
        print(f"[tdl bn] {key}", file=sys.stderr, flush=True)


class _BatchNormTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, residual, conv_bias, moving_mean, moving_var, momentum, eps, relu, grad_out,
                part=None, stats_out=None, defer=False):
        C = hip()
        xc = _aligned(x)
        rc = _aligned(residual.to(xc.dtype)) if residual is not None else None
        if defer:
            # BN -> ReLU applied by its only reader, a 1x1 conv's operand loader (ops/conv.py bn_in): the
            # statistics (and moving averages) only; the output is a stand-in view of the BN input
            st = C.bn_stats_train(xc, gamma, beta, moving_mean, moving_var, float(momentum), float(eps),
                                  conv_bias.detach() if conv_bias is not None else None, part)
            y = xc.view_as(xc)
        else:
            y, st = C.bn_forward_train(xc, gamma, beta, moving_mean, moving_var, float(momentum), float(eps),
                                       bool(relu), rc, conv_bias.detach() if conv_bias is not None else None, part)
        ctx.mode = 2 if residual is not None else (1 if relu else 0)
        if stats_out is not None:  # [4][C]: mean, invstd, scale, shift of this batch
            stats_out.append(st)
        _debug("fwd", tuple(x.shape), ctx.mode, "stats-fused" if part is not None else "stats-pass",
               "apply-deferred" if defer else "apply")
        ctx.flags = (gamma is not None, beta is not None, residual is not None, conv_bias is not None)
        ctx.res_dtype = residual.dtype if residual is not None else None
        ctx.grad_out = grad_out
        ctx.save_for_backward(xc, gamma if gamma is not None else st, st, y if ctx.mode == 2 else st,
                              conv_bias if conv_bias is not None else st)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = hip()
        xc, gamma, st, y, conv_bias = ctx.saved_tensors
        has_g, has_b, has_r, has_cb = ctx.flags
        # precomputed reductions (ops/conv.py): a group's from the consuming conv's input-gradient
        # epilogue; a plain BN's (mode 0) when its output gradient is such a group's dz
        part = getattr(dy, "_tdl_bn_bwd_part", None)
        part2 = getattr(dy, "_tdl_bn_bwd_part2", None) if ctx.mode == 2 else None
        dy = _aligned(dy.to(xc.dtype))
        go = ctx.grad_out or (None, None)
        fused = part is not None and dy.dtype == xc.dtype and dy.is_contiguous() and dy.data_ptr() % 16 == 0
        _debug("bwd", tuple(xc.shape), ctx.mode, "sums-fused" if fused else "sums-pass")
        if fused:
            # dy is already this group's masked dz, reduced by the consuming conv's dgrad epilogue
            FUSED_BWD[0] += 1
            FUSED_BWD_MODES[ctx.mode] += 1
            out = C.bn_backward(dy, xc, None, gamma if has_g else None, st, ctx.mode, go[0], go[1], part)
        else:
            out = C.bn_backward(dy, xc, y if ctx.mode == 2 else None, gamma if has_g else None, st, ctx.mode,
                                go[0], go[1])
        dx, dgamma, dbeta = out[0], out[1], out[2]
        dres = out[3].to(ctx.res_dtype) if has_r else None
        if fused and dres is not None:
            # dres IS dy here, which carries this group's own part: hand the residual's producer a
            # fresh view, with the sums the conv epilogue reduced for it (a plain projection-shortcut
            # BN: part2) or none
            dres = dres.view_as(dres)
            if part2 is not None:
                dres._tdl_bn_bwd_part = part2
        dcb = torch.zeros_like(conv_bias) if (has_cb and ctx.needs_input_grad[4]) else None
        return (dx, dgamma if ctx.needs_input_grad[1] else None, dbeta if ctx.needs_input_grad[2] else None, dres,
                dcb, None, None, None, None, None, None, None, None, None)


def batch_norm_train(x: torch.Tensor, gamma: Optional[torch.Tensor], beta: Optional[torch.Tensor],
                     moving_mean: Optional[torch.Tensor], moving_var: Optional[torch.Tensor], momentum: float,
                     eps: float, relu: bool = False, residual: Optional[torch.Tensor] = None,
                     conv_bias: Optional[torch.Tensor] = None, grad_out=None, part=None,
                     stats_out: Optional[list] = None, defer_apply: bool = False) -> torch.Tensor:
    """Keras-convention ``momentum`` (moving = moving*momentum + batch*(1-momentum)).

    ``grad_out = (dgamma_target, dbeta_target)``: f32 slab views the GPU backward ADDS the gamma /
    beta gradients into (Variable.grad_target); gamma / beta are then passed without autograd.
    ``part``: the batch statistics' partial sums already computed by the conv that produced x
    (ops/conv.py ``bn_stats``); the statistics pass over x is skipped.  ``stats_out``: a list the HIP
    path appends the batch's [4][C] statistics (mean, invstd, scale, shift) to.  ``defer_apply`` (HIP,
    ``relu=True``, no residual, with ``stats_out``): statistics only -- the returned tensor is a view of
    x standing for relu(bn(x)), valid only as the ``bn_in`` input of the one conv that applies it."""
    if defer_apply and not (relu and residual is None and stats_out is not None and supported(x)):
        raise ValueError("defer_apply: a GPU BN -> ReLU with stats_out")
    if residual is not None and not relu:
        raise ValueError("the fused residual form is BN -> Add -> ReLU")
    if supported(x) and (residual is None or tuple(residual.shape) == tuple(x.shape)):
        if grad_out is not None:
            gamma = gamma.detach() if gamma is not None else None
            beta = beta.detach() if beta is not None else None
        return _BatchNormTrain.apply(x, gamma, beta, residual, conv_bias, moving_mean, moving_var, momentum, eps, relu,
                                     grad_out, part, stats_out, defer_apply)
    h = x if conv_bias is None else x + conv_bias.to(x.dtype)
    perm = [0, h.dim() - 1] + list(range(1, h.dim() - 1))
    hp = h.permute(*perm)
    y = F.batch_norm(hp, moving_mean, moving_var, gamma.to(hp.dtype) if gamma is not None else None,
                     beta.to(hp.dtype) if beta is not None else None, training=True, momentum=1.0 - momentum, eps=eps)
    inv = [0] * len(perm)
    for i, p in enumerate(perm):
        inv[p] = i
    y = y.permute(*inv)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y
