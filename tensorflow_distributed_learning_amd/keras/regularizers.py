"""tf.keras.regularizers (added to the loss, scaled 1/num_replicas under distribution)."""
from __future__ import annotations


class Regularizer:
    def __call__(self, w):
        raise NotImplementedError


class L1L2(Regularizer):
    def __init__(self, l1=0.0, l2=0.0):
        self.l1, self.l2 = float(l1), float(l2)

    def __call__(self, w):
        out = 0.0
        if self.l1:
            out = out + self.l1 * w.abs().sum()
        if self.l2:
            out = out + self.l2 * (w * w).sum()
        return out


def L1(l1=0.01):  # noqa: N802
    return L1L2(l1=l1)


def L2(l2=0.01):  # noqa: N802
    return L1L2(l2=l2)


l1, l2, l1_l2 = L1, L2, L1L2
