"""TF-compatible namespaces so the reference script runs with two changed import lines:

    from tensorflow_distributed_learning_amd.compat import tf, tfds
"""
from . import tf, tfds  # noqa: F401
