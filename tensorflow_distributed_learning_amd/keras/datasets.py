"""``tf.keras.datasets`` (offline): ``mnist.load_data()``.

Keras loads ``~/.keras/datasets/<path>`` (an ``.npz`` with ``x_train``, ``y_train``, ``x_test``,
``y_test``), downloading it first.  Here nothing is downloaded: an existing ``.npz`` (the given path, or
``$KERAS_HOME/datasets/<path>``) is read with ``numpy.load(allow_pickle=False)``; otherwise the MNIST
IDX files are used when present, else the deterministic synthetic MNIST of ``data/tfds.py``.  Shapes and
dtypes follow Keras: uint8 images [n][28][28], uint8 labels [n].
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np


def _npz_path(path: str) -> Optional[str]:
    if os.path.isfile(path):
        return path
    home = os.environ.get("KERAS_HOME", os.path.join(os.path.expanduser("~"), ".keras"))
    p = os.path.join(home, "datasets", path)
    return p if os.path.isfile(p) else None


class mnist:  # noqa: N801
    @staticmethod
    def load_data(path: str = "mnist.npz"):
        f = _npz_path(path)
        if f is not None:
            with np.load(f, allow_pickle=False) as d:
                return (d["x_train"], d["y_train"]), (d["x_test"], d["y_test"])
        from ..data.tfds import mnist_arrays

        xtr, ytr, _ = mnist_arrays("train")
        xte, yte, _ = mnist_arrays("test")

        def u8(a):
            a = np.asarray(a)
            if a.ndim == 4 and a.shape[-1] == 1:
                a = a[..., 0]
            return a.astype(np.uint8)

        return (u8(xtr), np.asarray(ytr).astype(np.uint8)), (u8(xte), np.asarray(yte).astype(np.uint8))
