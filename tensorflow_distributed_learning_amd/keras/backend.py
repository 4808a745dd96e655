"""tf.keras.backend subset."""
from __future__ import annotations

import torch

_FLOATX = ["float32"]


def clear_session():
    """Reset layer-name counters (so names restart at conv2d, dense, ...)."""
    from .layers import reset_uids

    reset_uids()


def floatx():
    return _FLOATX[0]


def set_floatx(v):
    _FLOATX[0] = v


def image_data_format():
    return "channels_last"


def epsilon():
    return 1e-7


def get_value(x):
    return x.numpy() if hasattr(x, "numpy") else x


def set_value(x, v):
    x.assign(v)
