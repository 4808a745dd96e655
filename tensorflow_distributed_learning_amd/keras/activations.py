"""Keras activations (functional, on torch tensors)."""
from __future__ import annotations

import torch
import torch.nn.functional as F


def linear(x):
    return x


def relu(x, alpha=0.0, max_value=None, threshold=0.0):
    if alpha == 0.0 and max_value is None and threshold == 0.0:
        return F.relu(x)
    y = torch.where(x >= threshold, x, alpha * (x - threshold))
    if max_value is not None:
        y = torch.clamp(y, max=max_value)
    return y


def relu6(x):
    return F.relu6(x)


def sigmoid(x):
    return torch.sigmoid(x)


def tanh(x):
    return torch.tanh(x)


def softmax(x, axis=-1):
    return torch.softmax(x, dim=axis)


def log_softmax(x, axis=-1):
    return torch.log_softmax(x, dim=axis)


def elu(x, alpha=1.0):
    return F.elu(x, alpha)


def selu(x):
    return F.selu(x)


def softplus(x):
    return F.softplus(x)


def softsign(x):
    return F.softsign(x)


def swish(x):
    return F.silu(x)


silu = swish


def gelu(x, approximate=False):
    return F.gelu(x, approximate="tanh" if approximate else "none")


def exponential(x):
    return torch.exp(x)


def hard_sigmoid(x):
    return torch.clamp(0.2 * x + 0.5, 0.0, 1.0)


_MAP = {f.__name__: f for f in (linear, relu, relu6, sigmoid, tanh, softmax, log_softmax, elu, selu, softplus,
                                  softsign, swish, gelu, exponential, hard_sigmoid)}
_MAP["silu"] = swish


def get(identifier):
    if identifier is None:
        return linear
    if isinstance(identifier, str):
        if identifier not in _MAP:
            raise ValueError(f"unknown activation {identifier!r}")
        return _MAP[identifier]
    if callable(identifier):
        return identifier
    raise ValueError(f"could not interpret activation {identifier!r}")


def serialize(fn) -> str:
    for k, v in _MAP.items():
        if v is fn:
            return k
    return getattr(fn, "__name__", "custom")
