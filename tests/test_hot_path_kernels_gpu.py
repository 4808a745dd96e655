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


# ---------------------------------------------------------------------------------------------
# Every kernel, not only convolutions: the profiler's device-kernel names (utils/kernel_audit.py)
# must contain no vendor-library kernel (hipBLASLt / rocBLAS / Tensile / MIOpen / CK).  Graph capture
# is off in these runs so that every launch is visible to the tracer.

def _mnist_ds(n=512, b=64):
    g = torch.Generator().manual_seed(0)
    return tdl.data.Dataset.from_tensor_slices((torch.rand(n, 28, 28, 1, generator=g),
                                                torch.randint(0, 10, (n,), generator=g))).batch(b).repeat()


def _audit_fit(m, ds, steps):
    from tensorflow_distributed_learning_amd.utils.kernel_audit import audit

    m.fit(ds, epochs=1, steps_per_epoch=2, verbose=0)  # warm-up (allocations, first-use set-up)
    rep = audit(lambda: m.fit(ds, epochs=1, steps_per_epoch=steps, verbose=0))
    print({k: dict(v) for k, v in rep.items() if v})
    return rep


def test_fused_reference_cnn_step_kernels_are_hand_written(monkeypatch):
    from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn

    monkeypatch.setenv("TDL_GRAPH", "0")
    tdl.keras.backend.clear_session()
    with tdl.distribute.MirroredStrategy(devices=["/gpu:0"]).scope():
        m = build_mnist_cnn()
        m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tdl.keras.optimizers.SGD(1e-3), metrics=["sparse_categorical_accuracy"])
    rep = _audit_fit(m, _mnist_ds(), 3)
    assert m._trainer.kind == "fused"
    assert not rep["library"], rep["library"]
    assert any("k_fwd_conv" in n for n in rep["tdl"]) and any("k_finalize" in n for n in rep["tdl"]), rep


def test_generic_reference_cnn_step_kernels_and_graph(monkeypatch):
    """The generic engine (any model; here the reference CNN with the fused path disabled): its
    conv / dense GEMMs are the hand-written f32-MFMA kernels, the rest PyTorch's own elementwise /
    pooling / loss kernels -- no library GEMM or convolution; and with capture on (the default) the
    step becomes ONE whole-step hipGraph."""
    from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn

    monkeypatch.setenv("TDL_DISABLE_FUSED", "1")
    monkeypatch.setenv("TDL_GRAPH_STEP", "0")
    tdl.keras.backend.clear_session()
    with tdl.distribute.MirroredStrategy(devices=["/gpu:0"]).scope():
        m = build_mnist_cnn()
        m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tdl.keras.optimizers.SGD(1e-3), metrics=["sparse_categorical_accuracy"])
    rep = _audit_fit(m, _mnist_ds(), 3)
    assert m._trainer.kind == "generic"
    assert not rep["library"], rep["library"]
    assert any("gemm_f32" in n for n in rep["tdl"]), rep["tdl"]
    monkeypatch.setenv("TDL_GRAPH_STEP", "1")
    with tdl.distribute.MirroredStrategy(devices=["/gpu:0"]).scope():
        m2 = build_mnist_cnn()
        m2.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                   optimizer=tdl.keras.optimizers.SGD(1e-3), metrics=["sparse_categorical_accuracy"])
    m2.fit(_mnist_ds(), epochs=1, steps_per_epoch=6, verbose=0)
    assert m2._trainer.kind == "generic" and m2._trainer._graph_ok and m2._trainer._graphs


def test_resnet50_step_kernels_have_no_library_kernel(monkeypatch):
    from tensorflow_distributed_learning_amd.models.resnet50 import ResNet50

    monkeypatch.setenv("TDL_GRAPH_STEP", "0")
    tdl.keras.backend.clear_session()
    tdl.keras.mixed_precision.set_global_policy("mixed_bfloat16")
    try:
        tdl.keras.utils.set_random_seed(1)
        with tdl.distribute.MirroredStrategy(devices=["/gpu:0"]).scope():
            m = ResNet50(weights=None, input_shape=(64, 64, 3), classes=10)
            m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                      optimizer=tdl.keras.optimizers.SGD(learning_rate=0.01, momentum=0.9))
        g = torch.Generator().manual_seed(0)
        ds = tdl.data.Dataset.from_tensor_slices((torch.randn(16, 64, 64, 3, generator=g),
                                                  torch.randint(0, 10, (16,), generator=g))).batch(8).repeat()
        rep = _audit_fit(m, ds, 2)
        assert not rep["library"], rep["library"]
        assert sum(rep["tdl"].values()) > 100, rep["tdl"]
    finally:
        tdl.keras.mixed_precision.set_global_policy("float32")
