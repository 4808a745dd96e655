"""Keras losses.  Under a distribution strategy the training loss is summed per replica and
divided by the GLOBAL batch size (tf.nn.compute_average_loss semantics), so SUM all-reduced
gradients equal the gradient of the global-batch mean loss."""
from __future__ import annotations

import enum

import torch
import torch.nn.functional as F


class Reduction(enum.Enum):
    AUTO = "auto"
    NONE = "none"
    SUM = "sum"
    SUM_OVER_BATCH_SIZE = "sum_over_batch_size"


class Loss:
    def __init__(self, reduction=Reduction.AUTO, name=None):
        self.reduction = Reduction(reduction) if isinstance(reduction, str) else reduction
        self.name = name or _snake(type(self).__name__)

    def per_example(self, y_true, y_pred) -> torch.Tensor:
        raise NotImplementedError

    def __call__(self, y_true, y_pred, sample_weight=None):
        l = self.per_example(y_true, y_pred)
        if sample_weight is not None:
            sw = torch.as_tensor(sample_weight, dtype=l.dtype, device=l.device)
            l = l * sw.reshape(sw.shape + (1,) * (l.dim() - sw.dim()))
        if self.reduction == Reduction.NONE:
            return l
        if self.reduction == Reduction.SUM:
            return l.sum()
        return l.sum() / max(1, l.numel())

    def get_config(self):
        return {"reduction": self.reduction.value, "name": self.name}


def _snake(n):
    import re

    return re.sub(r"(?<!^)(?=[A-Z])", "_", n).lower()


class SparseCategoricalCrossentropy(Loss):
    """Integer labels; ``from_logits=True`` fuses log-softmax + NLL (tf_dist_example.py:50)."""

    def __init__(self, from_logits=False, ignore_class=None, reduction=Reduction.AUTO,
                 name="sparse_categorical_crossentropy"):
        super().__init__(reduction, name)
        self.from_logits = from_logits
        self.ignore_class = ignore_class

    def per_example(self, y_true, y_pred):
        y = y_true.reshape(-1).long() if y_true.dim() > 1 and y_true.shape[-1] == 1 else y_true.long()
        logits = y_pred if self.from_logits else torch.log(y_pred.clamp_min(1e-7))
        logits = logits.float() if logits.dtype in (torch.float16, torch.bfloat16) else logits
        if logits.dim() > 2:
            logits = logits.reshape(-1, logits.shape[-1])
            y = y.reshape(-1)
        if self.from_logits and self.ignore_class is None:
            from ..ops import dense as _dense

            if _dense.xent_supported(logits, y):
                return _dense.softmax_xent(logits, y)  # hand-written kernel (csrc/kernels/gemm.hip)
        l = F.cross_entropy(logits, y, reduction="none")
        if self.ignore_class is not None:
            l = l * (y != self.ignore_class)
        return l

    def get_config(self):
        return dict(super().get_config(), from_logits=self.from_logits)


class CategoricalCrossentropy(Loss):
    def __init__(self, from_logits=False, label_smoothing=0.0, reduction=Reduction.AUTO,
                 name="categorical_crossentropy"):
        super().__init__(reduction, name)
        self.from_logits, self.label_smoothing = from_logits, float(label_smoothing)

    def per_example(self, y_true, y_pred):
        y = y_true.to(y_pred.dtype)
        if self.label_smoothing:
            y = y * (1 - self.label_smoothing) + self.label_smoothing / y.shape[-1]
        logp = torch.log_softmax(y_pred, -1) if self.from_logits else torch.log(
            (y_pred / y_pred.sum(-1, keepdim=True)).clamp_min(1e-7))
        return -(y * logp).sum(-1)


class BinaryCrossentropy(Loss):
    def __init__(self, from_logits=False, label_smoothing=0.0, reduction=Reduction.AUTO, name="binary_crossentropy"):
        super().__init__(reduction, name)
        self.from_logits, self.label_smoothing = from_logits, float(label_smoothing)

    def per_example(self, y_true, y_pred):
        y = y_true.to(y_pred.dtype)
        if self.label_smoothing:
            y = y * (1 - self.label_smoothing) + 0.5 * self.label_smoothing
        if self.from_logits:
            l = F.binary_cross_entropy_with_logits(y_pred, y, reduction="none")
        else:
            l = F.binary_cross_entropy(y_pred.clamp(1e-7, 1 - 1e-7), y, reduction="none")
        return l.mean(-1) if l.dim() > 1 else l


class MeanSquaredError(Loss):
    def __init__(self, reduction=Reduction.AUTO, name="mean_squared_error"):
        super().__init__(reduction, name)

    def per_example(self, y_true, y_pred):
        d = (y_pred - y_true.to(y_pred.dtype)) ** 2
        return d.mean(-1) if d.dim() > 1 else d


class MeanAbsoluteError(Loss):
    def __init__(self, reduction=Reduction.AUTO, name="mean_absolute_error"):
        super().__init__(reduction, name)

    def per_example(self, y_true, y_pred):
        d = (y_pred - y_true.to(y_pred.dtype)).abs()
        return d.mean(-1) if d.dim() > 1 else d


class Huber(Loss):
    def __init__(self, delta=1.0, reduction=Reduction.AUTO, name="huber_loss"):
        super().__init__(reduction, name)
        self.delta = delta

    def per_example(self, y_true, y_pred):
        l = F.huber_loss(y_pred, y_true.to(y_pred.dtype), reduction="none", delta=self.delta)
        return l.mean(-1) if l.dim() > 1 else l


def sparse_categorical_crossentropy(y_true, y_pred, from_logits=False):
    return SparseCategoricalCrossentropy(from_logits=from_logits).per_example(y_true, y_pred)


def categorical_crossentropy(y_true, y_pred, from_logits=False):
    return CategoricalCrossentropy(from_logits=from_logits).per_example(y_true, y_pred)


def mean_squared_error(y_true, y_pred):
    return MeanSquaredError().per_example(y_true, y_pred)


mse = MSE = mean_squared_error

_ALIASES = {
    "sparse_categorical_crossentropy": SparseCategoricalCrossentropy,
    "categorical_crossentropy": CategoricalCrossentropy,
    "binary_crossentropy": BinaryCrossentropy,
    "mean_squared_error": MeanSquaredError, "mse": MeanSquaredError,
    "mean_absolute_error": MeanAbsoluteError, "mae": MeanAbsoluteError,
    "huber": Huber, "huber_loss": Huber,
}


class _FnLoss(Loss):
    def __init__(self, fn):
        super().__init__(Reduction.AUTO, getattr(fn, "__name__", "loss"))
        self.fn = fn

    def per_example(self, y_true, y_pred):
        return self.fn(y_true, y_pred)


def get(identifier) -> Loss:
    if isinstance(identifier, Loss):
        return identifier
    if isinstance(identifier, str):
        if identifier not in _ALIASES:
            raise ValueError(f"unknown loss {identifier!r}")
        return _ALIASES[identifier]()
    if callable(identifier):
        return _FnLoss(identifier)
    raise ValueError(f"could not interpret loss {identifier!r}")
