"""Device-resident input pipelines (SURVEY.md §3.2 target, §7.1 principle 4).

``fit`` lowers an in-memory pipeline of the form

    <columnar source> [.cache()] [.shuffle(buf, seed)] [.repeat(n)] .batch(B) [.repeat(n)]
    [.prefetch()] [.with_options()]

(the reference's ``map(scale).cache().shuffle(10000).batch(128)``, tf_dist_example.py:31-37) to
a :class:`DevicePipeline`: the columns are uploaded to HBM once, and each step only needs the
``B`` sample indices of its global batch, produced on the host by the SAME buffered-shuffle
algorithm and seeds as the host pipeline (so both paths see identical batches).  The fused HIP
step gathers its rows straight from HBM, so the training loop does no host data work and no
H2D copies beyond the per-execution index vector.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Optional

import numpy as np
import torch

from . import dataset as D


@dataclass
class LoweredPipeline:
    columns: Any                 # structure of host tensors with leading dim n
    n: int
    batch_size: int              # GLOBAL batch size
    drop_remainder: bool
    shuffle: Optional[D.ShuffleDataset]
    repeat: Optional[int]        # None = infinite, k = k passes
    batch_crosses_epochs: bool   # repeat below batch: a batch may straddle an epoch boundary


_PASS = (D.OptionsDataset, D.PrefetchDataset)


def lower(ds: D.Dataset) -> Optional[LoweredPipeline]:
    if not ds.options().experimental_optimization.device_resident:
        return None
    node = ds
    repeat_above, repeat_below = 1, 1

    def strip(n):
        while isinstance(n, _PASS):
            n = n._inputs[0]
        return n

    node = strip(node)
    if isinstance(node, D.RepeatDataset):
        repeat_above = node.count
        node = strip(node._inputs[0])
    if not isinstance(node, D.BatchDataset):
        return None
    batch = node
    node = strip(node._inputs[0])
    if isinstance(node, D.RepeatDataset):
        if repeat_above != 1:
            return None
        repeat_below = node.count
        node = strip(node._inputs[0])
    shuffle = None
    if isinstance(node, D.ShuffleDataset):
        shuffle = node
        node = strip(node._inputs[0])
    if not node._identity_order():
        return None
    cols = node._columns()
    if cols is None:
        return None
    leaves = D.flatten(cols)
    if not all(isinstance(t, torch.Tensor) for t in leaves):
        return None
    n = len(leaves[0])
    rep = repeat_below if repeat_below != 1 else repeat_above
    return LoweredPipeline(cols, n, batch.batch_size, batch.drop_remainder, shuffle, rep,
                           batch_crosses_epochs=repeat_below != 1)


class IndexStream:
    """Global-batch sample indices of a lowered pipeline, epoch after epoch.

    Epoch ``e`` of the stream shuffles with the dataset's RNG of iteration ``ep0 + e``, ``ep0``
    being the dataset's iteration counter when the stream was created (so a stream reproduces the
    host pipeline's order); the stream never mutates the dataset, which makes it safe to run ahead
    in a producer thread.  :meth:`commit` advances the dataset's counter by the epochs a consumer
    actually used.
    """

    def __init__(self, lp: LoweredPipeline, seed: Optional[int] = None):
        self.lp = lp
        self._epoch = 0
        self._buf = np.empty(0, dtype=np.int64)
        self._done = False
        self._seed = seed
        self._shuffle_seed_base = None
        self._ep0 = lp.shuffle._epoch if lp.shuffle is not None else 0

    def commit(self, epochs_used: int) -> None:
        sh = self.lp.shuffle
        if sh is not None:
            sh._epoch = max(sh._epoch, self._ep0 + int(epochs_used))

    def _epoch_order(self) -> Optional[np.ndarray]:
        lp = self.lp
        if lp.repeat is not None and self._epoch >= lp.repeat:
            return None
        e = self._epoch
        self._epoch += 1
        if lp.shuffle is None:
            return np.arange(lp.n, dtype=np.int64)
        sh = lp.shuffle
        override = None
        if self._seed is not None and sh.seed is None:
            # synchronised (DATA) sharding: same derivation as input_lib.reseed
            override = (int(self._seed) * 1_000_003 + 1) & ((1 << 62) - 1)
        return D._shuffle_indices(lp.n, sh.buffer_size, sh._rng_at(self._ep0 + e, override))

    def next_batch(self) -> Optional[np.ndarray]:
        """Indices of the next global batch (may be short at the very end), or None."""
        lp = self.lp
        B = lp.batch_size
        if lp.batch_crosses_epochs:
            while len(self._buf) < B and not self._done:
                o = self._epoch_order()
                if o is None:
                    self._done = True
                else:
                    self._buf = np.concatenate([self._buf, o])
        else:
            if len(self._buf) == 0 and not self._done:
                o = self._epoch_order()
                if o is None:
                    self._done = True
                else:
                    self._buf = o
        if len(self._buf) == 0:
            return None
        take = min(B, len(self._buf))
        if take < B and lp.drop_remainder:
            self._buf = self._buf[:0]
            if lp.batch_crosses_epochs or self._done:
                return None
            return self.next_batch()
        out, self._buf = self._buf[:take], self._buf[take:]
        return out


def upload(columns, device: torch.device):
    return D.map_structure(lambda t: t.to(device, non_blocking=False).contiguous(), columns)
