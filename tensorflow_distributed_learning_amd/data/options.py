"""tf.data.Options / AutoShardPolicy (tf_dist_example.py:34-37)."""
from __future__ import annotations

import enum
from dataclasses import dataclass, field
from typing import Optional


class AutoShardPolicy(enum.IntEnum):
    """How a dataset is split across workers when it is distributed.

    OFF  – no sharding: every worker iterates the full dataset (the reference, ex:35).
    AUTO – FILE if the pipeline reads files, else DATA.
    FILE – shard the input files across workers (error if the source is not file based).
    DATA – every replica takes a disjoint slice of every global batch (shuffle seeds are
           synchronised across workers so the slices never overlap).
    HINT – treated as DATA.
    """

    OFF = -1
    AUTO = 0
    FILE = 1
    DATA = 2
    HINT = 3


@dataclass
class DistributeOptions:
    auto_shard_policy: AutoShardPolicy = AutoShardPolicy.AUTO
    num_devices: Optional[int] = None


@dataclass
class OptimizationOptions:
    map_vectorization: bool = True      # run element-wise map fns once over whole columns when verified
    device_resident: bool = True        # allow fit() to lower in-memory pipelines to the device
    apply_default_optimizations: bool = True
    map_parallelization: bool = True


@dataclass
class ThreadingOptions:
    private_threadpool_size: int = 0
    max_intra_op_parallelism: int = 1


@dataclass
class Options:
    experimental_distribute: DistributeOptions = field(default_factory=DistributeOptions)
    experimental_optimization: OptimizationOptions = field(default_factory=OptimizationOptions)
    threading: ThreadingOptions = field(default_factory=ThreadingOptions)
    experimental_deterministic: Optional[bool] = None
    deterministic: Optional[bool] = None
    experimental_slack: bool = False

    def merge(self, other: "Options") -> "Options":
        """Later options win (Dataset.with_options semantics)."""
        import copy

        out = copy.deepcopy(self)
        if other is None:
            return out
        d = other.experimental_distribute
        if d.auto_shard_policy != AutoShardPolicy.AUTO:
            out.experimental_distribute.auto_shard_policy = d.auto_shard_policy
        if d.num_devices is not None:
            out.experimental_distribute.num_devices = d.num_devices
        out.experimental_optimization = copy.deepcopy(other.experimental_optimization)
        for k in ("experimental_deterministic", "deterministic"):
            if getattr(other, k) is not None:
                setattr(out, k, getattr(other, k))
        return out
