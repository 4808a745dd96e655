"""tf.keras.datasets (offline): mnist.load_data() -> real IDX files if present, else synthetic."""
from __future__ import annotations


class mnist:  # noqa: N801
    @staticmethod
    def load_data(path="mnist.npz"):
        from ..data.tfds import mnist_arrays

        xtr, ytr, _ = mnist_arrays("train")
        xte, yte, _ = mnist_arrays("test")
        return (xtr, ytr.astype("uint8")), (xte, yte.astype("uint8"))
