"""Hand-written kernels only on the hot path: a ResNet-50 bf16 training step and an
Adam-compiled reference-CNN step run no library convolution (ops/conv.py LIB_CALLS counts every conv
that falls back to MIOpen; the default TDL_CONV mode is the hand-written kernels)."""
import pytest
import torch

import tensorflow_distributed_learning_amd as tdl
from tensorflow_distributed_learning_amd.ops import conv as CV

pytestmark = pytest.mark.gpu


def test_resnet50_step_runs_no_library_conv():
    from tensorflow_distributed_learning_amd.models.resnet50 import ResNet50

    tdl.keras.backend.clear_session()
    tdl.keras.mixed_precision.set_global_policy("mixed_bfloat16")
    try:
        tdl.keras.utils.set_random_seed(1)
        with tdl.distribute.MirroredStrategy(devices=["/gpu:0"]).scope():
            m = ResNet50(weights=None, input_shape=(112, 112, 3), classes=10)
            m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                      optimizer=tdl.keras.optimizers.SGD(learning_rate=0.01, momentum=0.9))
        g = torch.Generator().manual_seed(0)
        ds = tdl.data.Dataset.from_tensor_slices((torch.randn(16, 112, 112, 3, generator=g),
                                                  torch.randint(0, 10, (16,), generator=g))).batch(8).repeat()
        CV.reset_library_calls()
        h = m.fit(ds, epochs=1, steps_per_epoch=3, verbose=0)
        torch.cuda.synchronize()
        assert CV.library_calls() == {}, CV.library_calls()
        assert torch.isfinite(torch.tensor(h.history["loss"])).all()
    finally:
        tdl.keras.mixed_precision.set_global_policy("float32")


def test_adam_reference_cnn_runs_on_fused_kernels_only():
    from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn

    tdl.keras.backend.clear_session()
    with tdl.distribute.MirroredStrategy(devices=["/gpu:0"]).scope():
        m = build_mnist_cnn()
        m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tdl.keras.optimizers.Adam(1e-3), metrics=["sparse_categorical_accuracy"],
                  steps_per_execution=2)
    g = torch.Generator().manual_seed(0)
    ds = tdl.data.Dataset.from_tensor_slices((torch.rand(256, 28, 28, 1, generator=g),
                                              torch.randint(0, 10, (256,), generator=g))).batch(64).repeat()
    CV.reset_library_calls()
    m.fit(ds, epochs=1, steps_per_epoch=4, verbose=0)
    assert m._trainer.kind == "fused", m._fused_reason
    assert CV.library_calls() == {}, CV.library_calls()
