"""tensorflow_distributed_learning_amd — MI355X-native synchronous mirrored data-parallel training.

Capabilities of Jackxiini/Tensorflow-distributed-learning (tf.distribute MirroredStrategy /
MultiWorkerMirroredStrategy, TF_CONFIG clusters, tf.data pipelines with auto-sharding, Keras
compile/fit with chief-only checkpoints) re-designed for AMD Instinct MI355X (gfx950):
one process per GPU, RCCL over xGMI, hand-written HIP kernels with f32 MFMA, hipGraph-captured
train steps, a native C++ rendezvous store and TCP ring.

    import tensorflow_distributed_learning_amd as tdl
    strategy = tdl.distribute.MultiWorkerMirroredStrategy()
    with strategy.scope():
        model = tdl.keras.Sequential([...]); model.compile(...)
    model.fit(dataset, epochs=10, steps_per_epoch=20)

A `tf`-compatible namespace for unmodified TF scripts: ``from tensorflow_distributed_learning_amd.compat import tf, tfds``.
"""
__version__ = "0.1.0"

from . import cluster, data, keras, ops  # noqa: F401
from . import parallel as distribute  # noqa: F401
from . import parallel  # noqa: F401
from .ckpt import checkpoint as _ckpt


class train:  # noqa: N801 - tf.train namespace
    Checkpoint = _ckpt.Checkpoint
    CheckpointManager = _ckpt.CheckpointManager
    latest_checkpoint = staticmethod(_ckpt.latest_checkpoint)
    list_variables = staticmethod(_ckpt.list_variables)
