"""tf.data equivalent."""
from .dataset import (  # noqa: F401
    AUTOTUNE,
    INFINITE_CARDINALITY,
    UNKNOWN_CARDINALITY,
    Dataset,
    TextLineDataset,
    TensorSpec,
    set_global_seed,
)
from .options import AutoShardPolicy, DistributeOptions, OptimizationOptions, Options  # noqa: F401


class experimental:  # noqa: N801 - tf.data.experimental namespace
    AutoShardPolicy = AutoShardPolicy
    AUTOTUNE = AUTOTUNE
    INFINITE_CARDINALITY = INFINITE_CARDINALITY
    UNKNOWN_CARDINALITY = UNKNOWN_CARDINALITY
    DistributeOptions = DistributeOptions
    OptimizationOptions = OptimizationOptions

    @staticmethod
    def cardinality(ds):
        import torch

        return torch.tensor(ds.cardinality())
