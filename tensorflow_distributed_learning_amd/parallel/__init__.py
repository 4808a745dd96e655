"""tf.distribute equivalent: strategies, communicators, distributed values and datasets."""
from .communication import (  # noqa: F401
    CollectiveCommunication,
    CommunicationImplementation,
    CommunicationOptions,
)
from .strategy import (  # noqa: F401
    HierarchicalCopyAllReduce,
    MirroredStrategy,
    MultiWorkerMirroredStrategy,
    NcclAllReduce,
    OneDeviceStrategy,
    ReduceOp,
    ReductionToOneDevice,
    ReplicaContext,
    Strategy,
    experimental,
    get_replica_context,
    get_strategy,
    has_strategy,
    in_cross_replica_context,
)
from .input_lib import DistributedDataset, InputContext  # noqa: F401
from .values import (  # noqa: F401
    MirroredVariable,
    PerReplica,
    SyncOnReadVariable,
    Variable,
    VariableAggregation,
    VariableSynchronization,
)


class cluster_resolver:  # noqa: N801
    from ..cluster.tf_config import TFConfigClusterResolver
