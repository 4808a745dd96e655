"""Dataset distribution: auto-sharding + rebatching (tf_dist_example.py:33-37).

The dataset yields GLOBAL batches (``batch(GLOBAL_BATCH_SIZE)``, ex:33).  Each replica process
receives its slice of every global batch (per-replica batch = global / num_replicas_in_sync;
partial final batches are split as evenly as possible).  Auto-shard policies:

* ``OFF``  – every worker runs the full pipeline with its own (unseeded) shuffle order and takes
  its replica slice of each of its own global batches (the reference's setting, ex:35).
* ``DATA`` – the shuffle seeds of every worker are synchronised (broadcast from the chief), so
  all workers produce the same global batches and the replica slices are disjoint.
* ``FILE`` – file-based pipelines read a disjoint subset of files per worker and are rebatched
  to the per-replica batch size.
* ``AUTO`` – FILE when the pipeline reads files, else DATA.
"""
from __future__ import annotations

import copy
from typing import List, Optional

import numpy as np
import torch

from ..data import dataset as D
from ..data.options import AutoShardPolicy


def find_batch(ds: D.Dataset) -> Optional[D.BatchDataset]:
    node = ds
    while node is not None:
        if isinstance(node, D.BatchDataset):
            return node
        if len(node._inputs) != 1:
            return None
        node = node._inputs[0]
    return None


def reseed(ds: D.Dataset, seed: int, _pos=None) -> D.Dataset:
    """Copy of the pipeline where every UNSEEDED shuffle gets a deterministic seed from `seed`."""
    pos = _pos if _pos is not None else [0]
    new = copy.copy(ds)
    new._inputs = tuple(reseed(i, seed, pos) for i in ds._inputs)
    if isinstance(new, D.ShuffleDataset):
        pos[0] += 1
        if new.seed is None:
            new.seed = (int(seed) * 1_000_003 + pos[0]) & ((1 << 62) - 1)
            new._epoch = 0
            new._base = None
    if isinstance(new, D.MapDataset):
        new._vec = ds._vec
    if isinstance(new, D.CacheDataset):
        # share the materialised cache with the original node
        ds.materialize()
        new._cache, new._cols = ds._cache, ds._cols
    return new


def shared_seed(strategy) -> int:
    """A seed drawn by the chief and broadcast to every replica."""
    t = torch.tensor([int(np.random.SeedSequence().entropy % (1 << 62))], dtype=torch.int64)
    comm = strategy.extended.communicator
    if comm.world_size > 1:
        dev = strategy.extended.device
        t = t.to(dev) if comm.name == "rccl" else t
        comm.broadcast(t, 0)
    return int(t.cpu()[0])


def split_sizes(n: int, parts: int) -> List[int]:
    base, extra = divmod(n, parts)
    return [base + (1 if i < extra else 0) for i in range(parts)]


def effective_policy(ds: D.Dataset) -> AutoShardPolicy:
    pol = ds.options().experimental_distribute.auto_shard_policy
    if pol == AutoShardPolicy.HINT:
        pol = AutoShardPolicy.DATA
    if pol == AutoShardPolicy.AUTO:
        pol = AutoShardPolicy.FILE if ds.source_files() is not None else AutoShardPolicy.DATA
    return pol


class InputContext:
    """tf.distribute.InputContext."""

    def __init__(self, num_input_pipelines=1, input_pipeline_id=0, num_replicas_in_sync=1):
        self.num_input_pipelines = num_input_pipelines
        self.input_pipeline_id = input_pipeline_id
        self.num_replicas_in_sync = num_replicas_in_sync

    def get_per_replica_batch_size(self, global_batch_size: int) -> int:
        if global_batch_size % self.num_replicas_in_sync:
            raise ValueError(f"global batch {global_batch_size} is not divisible by {self.num_replicas_in_sync} replicas")
        return global_batch_size // self.num_replicas_in_sync


class DistributedDataset:
    """Per-replica view of a dataset of global batches."""

    def __init__(self, dataset: D.Dataset, strategy, options=None):
        self.dataset = dataset
        self.strategy = strategy
        self.options = options
        R = strategy.num_replicas_in_sync
        self.rank = strategy.extended.rank
        self.num_replicas = R
        self.policy = effective_policy(dataset) if R > 1 else AutoShardPolicy.OFF
        b = find_batch(dataset)
        self.global_batch_size = b.batch_size if b is not None else None
        self._pipeline = dataset
        if R > 1:
            if self.policy == AutoShardPolicy.FILE:
                sharded = D.auto_shard(dataset, R, self.rank, AutoShardPolicy.FILE)
                gb = self.global_batch_size
                if gb is None:
                    raise ValueError("FILE auto-sharding needs a batched dataset")
                self._pipeline = sharded.unbatch().batch(max(1, gb // R), b.drop_remainder)
                self._slice = False
            else:
                if self.policy == AutoShardPolicy.DATA:
                    self._pipeline = reseed(dataset, shared_seed(strategy))
                self._slice = True
        else:
            self._slice = False

    @property
    def per_replica_batch_size(self) -> Optional[int]:
        if self.global_batch_size is None:
            return None
        return self.global_batch_size // self.num_replicas

    def __iter__(self):
        return DistributedIterator(self)

    def cardinality(self):
        return self._pipeline.cardinality()


class DistributedIterator:
    def __init__(self, dd: DistributedDataset):
        self.dd = dd
        self._it = iter(dd._pipeline)

    def __iter__(self):
        return self

    def __next__(self):
        batch = next(self._it)
        dd = self.dd
        if not dd._slice:
            return batch
        n = len(D.flatten(batch)[0])
        sizes = split_sizes(n, dd.num_replicas)
        lo = sum(sizes[: dd.rank])
        hi = lo + sizes[dd.rank]
        return D.map_structure(lambda t: t[lo:hi], batch)

    def get_next(self):
        return next(self)

    def get_next_as_optional(self):
        try:
            return next(self)
        except StopIteration:
            return None


class LocalDistributedDataset:
    """``experimental_distribute_dataset`` of a single-process multi-device MirroredStrategy: ONE
    pipeline of global batches, each split into per-replica slices (split_sizes) and yielded as a
    :class:`~.values.PerReplica` (TF: the worker's batch is divided among its local replicas), which
    ``strategy.run`` hands to the replicas one slice each."""

    def __init__(self, dataset: D.Dataset, strategy, options=None):
        self.dataset, self.strategy, self.options = dataset, strategy, options
        self.num_replicas = strategy.num_replicas_in_sync
        b = find_batch(dataset)
        self.global_batch_size = b.batch_size if b is not None else None

    @property
    def per_replica_batch_size(self) -> Optional[int]:
        if self.global_batch_size is None:
            return None
        return self.global_batch_size // self.num_replicas

    def cardinality(self):
        return self.dataset.cardinality()

    def __iter__(self):
        from .values import PerReplica

        G = self.num_replicas
        for batch in self.dataset:
            n = len(D.flatten(batch)[0])
            sizes = split_sizes(n, G)
            lo, parts = 0, []
            for r in range(G):
                parts.append(D.map_structure(lambda t, lo=lo, hi=lo + sizes[r]: t[lo:hi], batch))
                lo += sizes[r]
            yield _per_replica_structure(parts, PerReplica)


class LocalDistributedDatasetFromFunction:
    """``distribute_datasets_from_function`` of a single-process multi-device MirroredStrategy: the
    function runs once (one input pipeline, ``input_pipeline_id`` 0) and returns a dataset batched
    by the per-replica batch size; consecutive batches go to consecutive replicas, G of them form
    one :class:`~.values.PerReplica` step input."""

    def __init__(self, dataset: D.Dataset, strategy, ctx: InputContext):
        self.dataset, self.strategy, self.ctx = dataset, strategy, ctx
        self.num_replicas = strategy.num_replicas_in_sync
        b = find_batch(dataset)
        self.global_batch_size = b.batch_size * self.num_replicas if b is not None else None

    def __iter__(self):
        from .values import PerReplica

        it = iter(self.dataset)
        while True:
            parts = []
            for _ in range(self.num_replicas):
                try:
                    parts.append(next(it))
                except StopIteration:
                    break
            if len(parts) < self.num_replicas:
                return  # (TF drops an incomplete final round of per-replica batches the same way)
            yield _per_replica_structure(parts, PerReplica)


def _per_replica_structure(parts, PerReplica):
    """[structure per replica] -> structure of PerReplica leaves (tuples / lists / dicts kept)."""
    first = parts[0]
    if isinstance(first, dict):
        return {k: _per_replica_structure([p[k] for p in parts], PerReplica) for k in first}
    if isinstance(first, (tuple, list)):
        return type(first)(_per_replica_structure([p[i] for p in parts], PerReplica) for i in range(len(first)))
    return PerReplica(parts)


class DistributedDatasetFromFunction:
    """Each replica builds its own input pipeline from an InputContext (no slicing)."""

    def __init__(self, dataset: D.Dataset, strategy, ctx: InputContext):
        self.dataset, self.strategy, self.ctx = dataset, strategy, ctx
        b = find_batch(dataset)
        self.global_batch_size = b.batch_size * strategy.num_replicas_in_sync if b is not None else None

    @property
    def per_replica_batch_size(self):
        b = find_batch(self.dataset)
        return b.batch_size if b is not None else None

    def __iter__(self):
        return iter(self.dataset)
