"""Cluster definition (TF_CONFIG) and native rendezvous."""
from .tf_config import (  # noqa: F401
    ALL_ROLES,
    TRAINING_ROLES,
    ClusterConfigError,
    ClusterSpec,
    TaskSpec,
    TFConfig,
    TFConfigClusterResolver,
    make_tf_config,
    parse_tf_config,
)
