"""Classifier head of the generic engine on hand-written gfx950 kernels (csrc/kernels/gemm.hip):
GlobalAveragePooling2D, Dense and sparse softmax cross-entropy for bf16 activations on the GPU
(the ResNet-50 of BASELINE configs 4/5: ``avg_pool -> predictions(1000) -> SCCE(from_logits)``).

* ``gap_nhwc``: NHWC mean over the pixels (f32 sums), backward broadcasts dy / HW.
* ``dense_bf16``: ``y = x W + b`` on a bf16 MFMA GEMM whose operands are read in their stored
  layouts (forward x.W, input gradient dy.W^T, weight gradient x^T.dy: no transposed copies).
  With gradient-slab targets (``Variable.grad_target``) dW and db are ADDED into the f32 slab.
* ``softmax_xent``: per-example ``logsumexp(z) - z[label]`` on f32 logits, backward
  ``(softmax - onehot) * g`` in one pass.

Reference: the Keras layers / loss of ``tf_dist_example.py:41-50`` (and keras.applications.ResNet50).
"""
from __future__ import annotations

from typing import Optional

import torch

from . import hip


def _aligned(t: torch.Tensor) -> torch.Tensor:
    t = t.contiguous()
    return t if t.data_ptr() % 16 == 0 else t.clone()


def gap_supported(x: torch.Tensor) -> bool:
    return x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[-1] % 8 == 0


class _GAP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[1], x.shape[2])
        return hip().gap_fwd(_aligned(x))

    @staticmethod
    def backward(ctx, dy):
        return hip().gap_bwd(_aligned(dy.to(torch.bfloat16)), *ctx.hw)


def gap_nhwc(x: torch.Tensor) -> torch.Tensor:
    return _GAP.apply(x)


def dense_supported(x: torch.Tensor, units: int) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 2 and x.shape[0] % 8 == 0
            and x.shape[1] % 8 == 0 and units % 8 == 0)


class _Dense(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, targets, anchor=None):
        C = hip()
        x = _aligned(x)
        wc = _aligned(w)
        bias = b.detach().float().contiguous() if b is not None else None
        y = C.gemm_bf16(x, 0, wc, 1, bias=bias)
        ctx.save_for_backward(x, wc)
        ctx.has_b = b is not None
        ctx.targets = targets
        return y

    @staticmethod
    def backward(ctx, dy):
        C = hip()
        x, w = ctx.saved_tensors
        dy = _aligned(dy.to(torch.bfloat16))
        dx = C.gemm_bf16(dy, 0, w, 0) if ctx.needs_input_grad[0] else None
        gw_t, gb_t = ctx.targets if ctx.targets is not None else (None, None)
        dw = db = None
        if gw_t is not None:
            C.gemm_bf16(x, 1, dy, 1, out=gw_t, accumulate=True)
        elif ctx.needs_input_grad[1]:
            dw = C.gemm_bf16(x, 1, dy, 1, out=torch.empty(w.shape, dtype=torch.float32, device=w.device)).to(w.dtype)
        if ctx.has_b:
            s = dy.float().sum(0)
            if gb_t is not None:
                gb_t.add_(s)
            elif ctx.needs_input_grad[2]:
                db = s
        return dx, dw, db, None, None


def dense_bf16(x, w, b=None, targets=None, anchor=None):
    """``x [N, in] bf16 @ w [in, out] bf16 (+ b f32)`` -> bf16 [N, out].  ``targets = (dW, db)``:
    f32 slab views the gradients are added into (``w`` / ``b`` then need no autograd).  ``anchor``:
    with targets, the kernel variable's leaf, so that the backward runs when nothing else needs a
    gradient (a first layer reading the input batch)."""
    return _Dense.apply(x, w, b, targets, anchor)


class _SoftmaxXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, labels):
        z = z.contiguous()
        labels = labels.contiguous()
        loss, _ = hip().xent_fwd(z, labels)
        ctx.save_for_backward(z, labels)
        return loss

    @staticmethod
    def backward(ctx, g):
        z, labels = ctx.saved_tensors
        return hip().xent_bwd(z, labels, g.float().contiguous()), None


def xent_supported(z: torch.Tensor, labels: torch.Tensor) -> bool:
    return z.is_cuda and z.dtype == torch.float32 and z.dim() == 2 and labels.dim() == 1


def softmax_xent(z: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """Per-example sparse softmax cross-entropy of f32 logits ``z [N, K]`` and int64 ``labels [N]``."""
    return _SoftmaxXent.apply(z, labels)


class _XentHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, labels, gn, accs, seed):
        loss, dz = hip().xent_head(z.contiguous(), labels.contiguous(), float(gn), *accs)
        ctx.save_for_backward(dz)
        ctx.seed_ptr = seed.data_ptr() if seed is not None else None
        return loss

    @staticmethod
    def backward(ctx, g):
        (dz,) = ctx.saved_tensors
        if ctx.seed_ptr is not None and g.data_ptr() == ctx.seed_ptr:
            return dz, None, None, None, None  # the trainer's own backward seed (1.0): no scaling kernel
        return dz * g, None, None, None, None


def xent_head_supported(z: torch.Tensor, labels: torch.Tensor) -> bool:
    """f32 [N, K] logits with int64 [N] labels (one workgroup up to 64K logits, two kernels beyond)."""
    return xent_supported(z, labels) and z.shape[0] >= 1 and z.shape[1] >= 1


def xent_head(z: torch.Tensor, labels: torch.Tensor, global_n: int, loss_acc=(None, None), acc_acc=(None, None),
              seed: Optional[torch.Tensor] = None):
    """The generic engine's loss head in ONE kernel (csrc/kernels/gemm.hip k_xent_head): the mean-reduced
    sparse softmax cross-entropy ``sum(per-example loss) / global_n`` (tf.nn.compute_average_loss), its
    logit gradient (saved for the backward), and the loss-tracker / SparseCategoricalAccuracy f64
    accumulators ``(total, count)`` advanced in place -- instead of ~15 PyTorch reduction / elementwise
    kernels per step (tf_dist_example.py:49-52)."""
    return _XentHead.apply(z, labels, float(global_n), tuple(loss_acc) + tuple(acc_acc), seed)
