"""Keras metrics with cross-replica state (tf_dist_example.py:52).

Metric state lives in ON_READ (SyncOnRead) variables on the replica's device: updating is a
device-side accumulation (no host sync); ``result()`` in cross-replica context all-reduces the
state across replicas (SUM aggregation) and only then divides.  The fused MNIST step updates the
same accumulators from inside its loss kernel.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..parallel.values import VariableAggregation, VariableSynchronization, create_variable


class Metric:
    def __init__(self, name: Optional[str] = None, dtype=None):
        import re

        self.name = name or re.sub(r"(?<!^)(?=[A-Z])", "_", type(self).__name__).lower()
        self.dtype = dtype or torch.float32
        self._vars = []
        self._device = None

    def add_weight(self, name, shape=(), initializer="zeros", dtype=None):
        v = create_variable(torch.zeros(shape, dtype=dtype or torch.float64), name=f"{self.name}/{name}",
                            trainable=False, synchronization=VariableSynchronization.ON_READ,
                            aggregation=VariableAggregation.SUM)
        self._vars.append(v)
        return v

    @property
    def variables(self):
        return list(self._vars)

    def _to(self, device):
        if self._device != device:
            for v in self._vars:
                v._value = v._value.to(device)
            self._device = device

    def update_state(self, *args, **kwargs):
        raise NotImplementedError

    def result(self):
        raise NotImplementedError

    def reset_state(self):
        for v in self._vars:
            with torch.no_grad():
                v._value.zero_()

    reset_states = reset_state

    def __call__(self, *args, **kwargs):
        self.update_state(*args, **kwargs)
        return self.result()

    def get_config(self):
        return {"name": self.name}


class Reduce(Metric):
    def __init__(self, name=None, dtype=None):
        super().__init__(name, dtype)
        self.total = self.add_weight("total")
        self.count = self.add_weight("count")

    def update_state(self, values, sample_weight=None):
        v = torch.as_tensor(values).detach()
        self._to(v.device)
        v = v.to(torch.float64)
        if sample_weight is not None:
            w = torch.as_tensor(sample_weight, device=v.device, dtype=torch.float64)
            self.total._value.add_((v * w).sum())
            self.count._value.add_(w.sum() if w.dim() else w * max(1, v.numel()))
        else:
            self.total._value.add_(v.sum())
            self.count._value.add_(float(v.numel()))


class Mean(Reduce):
    def result(self):
        t, c = self.total.read_value(), self.count.read_value()
        return (t / c.clamp_min(1e-12)).to(torch.float32) if float(c) > 0 else torch.tensor(0.0)


class Sum(Reduce):
    def result(self):
        return self.total.read_value().to(torch.float32)


class MeanMetricWrapper(Mean):
    def __init__(self, fn, name=None, dtype=None, **fn_kwargs):
        super().__init__(name or getattr(fn, "__name__", "metric"), dtype)
        self.fn = fn
        self.fn_kwargs = fn_kwargs

    def update_state(self, y_true, y_pred, sample_weight=None):
        super().update_state(self.fn(y_true, y_pred, **self.fn_kwargs), sample_weight)


def sparse_categorical_accuracy(y_true, y_pred):
    y = y_true.reshape(-1).long() if (y_true.dim() > 1 and y_true.shape[-1] == 1) else y_true.long()
    return (y_pred.argmax(-1) == y).to(torch.float32)


def categorical_accuracy(y_true, y_pred):
    return (y_pred.argmax(-1) == y_true.argmax(-1)).to(torch.float32)


def binary_accuracy(y_true, y_pred, threshold=0.5):
    return ((y_pred > threshold).to(y_true.dtype) == y_true).to(torch.float32).reshape(y_true.shape[0], -1).mean(-1)


def accuracy(y_true, y_pred):
    return (y_true == y_pred).to(torch.float32)


def sparse_top_k_categorical_accuracy(y_true, y_pred, k=5):
    y = y_true.reshape(-1).long()
    top = y_pred.topk(min(k, y_pred.shape[-1]), -1).indices
    return (top == y[:, None]).any(-1).to(torch.float32)


def top_k_categorical_accuracy(y_true, y_pred, k=5):
    return sparse_top_k_categorical_accuracy(y_true.argmax(-1), y_pred, k)


class SparseCategoricalAccuracy(MeanMetricWrapper):
    def __init__(self, name="sparse_categorical_accuracy", dtype=None):
        super().__init__(sparse_categorical_accuracy, name, dtype)


class CategoricalAccuracy(MeanMetricWrapper):
    def __init__(self, name="categorical_accuracy", dtype=None):
        super().__init__(categorical_accuracy, name, dtype)


class BinaryAccuracy(MeanMetricWrapper):
    def __init__(self, name="binary_accuracy", dtype=None, threshold=0.5):
        super().__init__(binary_accuracy, name, dtype, threshold=threshold)


class Accuracy(MeanMetricWrapper):
    def __init__(self, name="accuracy", dtype=None):
        super().__init__(accuracy, name, dtype)


class SparseTopKCategoricalAccuracy(MeanMetricWrapper):
    def __init__(self, k=5, name="sparse_top_k_categorical_accuracy", dtype=None):
        super().__init__(sparse_top_k_categorical_accuracy, name, dtype, k=k)


class TopKCategoricalAccuracy(MeanMetricWrapper):
    def __init__(self, k=5, name="top_k_categorical_accuracy", dtype=None):
        super().__init__(top_k_categorical_accuracy, name, dtype, k=k)


class MeanSquaredError(MeanMetricWrapper):
    def __init__(self, name="mean_squared_error", dtype=None):
        super().__init__(lambda t, p: ((p - t.to(p.dtype)) ** 2).reshape(p.shape[0], -1).mean(-1), name, dtype)


class MeanAbsoluteError(MeanMetricWrapper):
    def __init__(self, name="mean_absolute_error", dtype=None):
        super().__init__(lambda t, p: (p - t.to(p.dtype)).abs().reshape(p.shape[0], -1).mean(-1), name, dtype)


class Precision(Metric):
    def __init__(self, thresholds=0.5, name="precision", dtype=None):
        super().__init__(name, dtype)
        self.threshold = thresholds
        self.tp = self.add_weight("true_positives")
        self.fp = self.add_weight("false_positives")

    def update_state(self, y_true, y_pred, sample_weight=None):
        self._to(y_pred.device)
        p = (y_pred > self.threshold)
        t = y_true.bool()
        self.tp._value.add_((p & t).sum().double())
        self.fp._value.add_((p & ~t).sum().double())

    def result(self):
        tp, fp = self.tp.read_value(), self.fp.read_value()
        return (tp / (tp + fp).clamp_min(1e-12)).float()


class Recall(Metric):
    def __init__(self, thresholds=0.5, name="recall", dtype=None):
        super().__init__(name, dtype)
        self.threshold = thresholds
        self.tp = self.add_weight("true_positives")
        self.fn = self.add_weight("false_negatives")

    def update_state(self, y_true, y_pred, sample_weight=None):
        self._to(y_pred.device)
        p = (y_pred > self.threshold)
        t = y_true.bool()
        self.tp._value.add_((p & t).sum().double())
        self.fn._value.add_((~p & t).sum().double())

    def result(self):
        tp, fn = self.tp.read_value(), self.fn.read_value()
        return (tp / (tp + fn).clamp_min(1e-12)).float()


_ALIASES = {
    "sparse_categorical_accuracy": SparseCategoricalAccuracy, "categorical_accuracy": CategoricalAccuracy,
    "binary_accuracy": BinaryAccuracy, "sparse_top_k_categorical_accuracy": SparseTopKCategoricalAccuracy,
    "top_k_categorical_accuracy": TopKCategoricalAccuracy, "mse": MeanSquaredError,
    "mean_squared_error": MeanSquaredError, "mae": MeanAbsoluteError, "mean_absolute_error": MeanAbsoluteError,
    "precision": Precision, "recall": Recall,
}


def get(identifier, loss=None) -> Metric:
    if isinstance(identifier, Metric):
        return identifier
    if isinstance(identifier, str):
        if identifier in ("accuracy", "acc"):
            from . import losses

            if isinstance(loss, losses.SparseCategoricalCrossentropy):
                return SparseCategoricalAccuracy(name=identifier)
            if isinstance(loss, losses.CategoricalCrossentropy):
                return CategoricalAccuracy(name=identifier)
            if isinstance(loss, losses.BinaryCrossentropy):
                return BinaryAccuracy(name=identifier)
            return SparseCategoricalAccuracy(name=identifier)
        if identifier not in _ALIASES:
            raise ValueError(f"unknown metric {identifier!r}")
        return _ALIASES[identifier]()
    if callable(identifier):
        return MeanMetricWrapper(identifier)
    raise ValueError(f"could not interpret metric {identifier!r}")
