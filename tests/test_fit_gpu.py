"""End-to-end: Keras fit on one MI355X through the fused HIP engine vs the generic engine."""
import os

import numpy as np
import pytest
import torch

import tensorflow_distributed_learning_amd as tdl
from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn

pytestmark = pytest.mark.gpu


def _data(n=2048, seed=0):
    from tensorflow_distributed_learning_amd.data.tfds import synthetic_mnist

    x, y = synthetic_mnist(n, seed)
    return x.reshape(-1, 28, 28, 1), y


def _pipeline(x, y, B, seed=7):
    def scale(image, label):
        return image.to(torch.float32) / 255, label

    return tdl.data.Dataset.from_tensor_slices((x, y)).map(scale).cache().shuffle(1000, seed=seed).batch(B).repeat()


def _train(fused: bool, steps=12, spe=4, n=2048):
    tdl.keras.backend.clear_session()
    tdl.keras.utils.set_random_seed(3)
    os.environ["TDL_DISABLE_FUSED"] = "0" if fused else "1"
    try:
        x, y = _data(n)
        strategy = tdl.distribute.MirroredStrategy(devices=["/gpu:0"])
        with strategy.scope():
            m = build_mnist_cnn()
            m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                      optimizer=tdl.keras.optimizers.SGD(learning_rate=0.05),
                      metrics=[tdl.keras.metrics.SparseCategoricalAccuracy()], steps_per_execution=spe)
        h = m.fit(_pipeline(x, y, 64), epochs=2, steps_per_epoch=steps // 2, verbose=0)
        return m, h
    finally:
        os.environ.pop("TDL_DISABLE_FUSED", None)


def test_fused_engine_selected_and_matches_generic():
    mf, hf = _train(True)
    assert mf._trainer.kind == "fused", mf._fused_reason
    mg, hg = _train(False)
    assert mg._trainer.kind == "generic"
    for a, b in zip(mf.get_weights(), mg.get_weights()):
        np.testing.assert_allclose(a, b, rtol=2e-3, atol=2e-4)
    for k in ("loss", "sparse_categorical_accuracy"):
        np.testing.assert_allclose(hf.history[k], hg.history[k], rtol=1e-3, atol=6e-3)  # 1-2 argmax near-ties


def test_fused_fit_learns():
    m, h = _train(True, steps=60, spe=10)
    assert h.history["loss"][-1] < h.history["loss"][0]
    assert h.history["sparse_categorical_accuracy"][-1] > 0.3


def test_fused_epoch_boundary_partial_batches_match_generic():
    """n=300, B=64: every epoch ends in a 44-sample batch, so 3-step executions get cut short in
    front of it (eager remainder) and the partial batch runs as its own step."""
    mf, hf = _train(True, steps=14, spe=3, n=300)
    assert mf._trainer.kind == "fused", mf._fused_reason
    mg, hg = _train(False, steps=14, spe=3, n=300)
    for a, b in zip(mf.get_weights(), mg.get_weights()):
        np.testing.assert_allclose(a, b, rtol=2e-3, atol=2e-4)
    np.testing.assert_allclose(hf.history["loss"], hg.history["loss"], rtol=1e-3, atol=1e-4)
