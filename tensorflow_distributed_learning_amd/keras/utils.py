"""tf.keras.utils subset."""
from __future__ import annotations

import random

import numpy as np
import torch


def to_categorical(y, num_classes=None, dtype="float32"):
    y = np.asarray(y, dtype=np.int64).reshape(-1)
    n = num_classes or int(y.max()) + 1
    out = np.zeros((len(y), n), dtype=dtype)
    out[np.arange(len(y)), y] = 1
    return out


def set_random_seed(seed: int):
    from ..data import dataset as D
    from . import initializers

    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    initializers.set_seed(seed)
    D.set_global_seed(seed)
