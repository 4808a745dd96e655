"""Forward-only evaluate / predict / fit(validation_data=...) on the hand-written gfx950 forward
kernel (head mode 2) vs the generic (torch-op) engine, on the reference CNN (README.md:121-129
builds val_data from numpy arrays with Dataset.from_tensor_slices)."""
import os

import numpy as np
import pytest
import torch

import tensorflow_distributed_learning_amd as tdl
from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn

pytestmark = pytest.mark.gpu


def _data(n, seed):
    from tensorflow_distributed_learning_amd.data.tfds import synthetic_mnist

    x, y = synthetic_mnist(n, seed)
    x = torch.from_numpy(np.ascontiguousarray(x)).reshape(-1, 28, 28, 1).float() / 255
    return x.contiguous(), torch.from_numpy(np.ascontiguousarray(y)).long()


def _model():
    tdl.keras.backend.clear_session()
    tdl.keras.utils.set_random_seed(5)
    strategy = tdl.distribute.MirroredStrategy(devices=["/gpu:0"])
    with strategy.scope():
        m = build_mnist_cnn()
        m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tdl.keras.optimizers.SGD(learning_rate=0.05),
                  metrics=[tdl.keras.metrics.SparseCategoricalAccuracy()], steps_per_execution=4)
    x, y = _data(1024, 0)
    m.fit(tdl.data.Dataset.from_tensor_slices((x, y)).batch(64).repeat(), epochs=1, steps_per_epoch=8, verbose=0)
    assert m._trainer.kind == "fused", m._fused_reason
    return m


def _generic(fn):
    os.environ["TDL_FUSED_EVAL"] = "0"
    try:
        return fn()
    finally:
        os.environ.pop("TDL_FUSED_EVAL", None)


def test_fused_evaluate_matches_generic_with_partial_batch():
    m = _model()
    xv, yv = _data(1000, 1)  # 7 full batches of 128 + a partial batch of 104
    val = tdl.data.Dataset.from_tensor_slices((xv, yv)).batch(128)
    fused = m.evaluate(val, return_dict=True, verbose=0)
    gen = _generic(lambda: m.evaluate(val, return_dict=True, verbose=0))
    np.testing.assert_allclose(fused["loss"], gen["loss"], rtol=2e-5)
    assert abs(fused["sparse_categorical_accuracy"] - gen["sparse_categorical_accuracy"]) <= 1.0 / 1000
    # numpy inputs (the README's val_x / val_y) take the same path
    fused_np = m.evaluate(xv.numpy(), yv.numpy(), batch_size=100, return_dict=True, verbose=0)
    np.testing.assert_allclose(fused_np["loss"], gen["loss"], rtol=2e-5)


def test_fused_predict_matches_generic_and_reference():
    m = _model()
    xv, _ = _data(300, 2)
    ds = tdl.data.Dataset.from_tensor_slices(xv).batch(64)
    fused = m.predict(ds, verbose=0)
    gen = _generic(lambda: m.predict(ds, verbose=0))
    assert fused.shape == (300, 10)
    np.testing.assert_allclose(fused, gen, rtol=1e-4, atol=1e-5)
    from tensorflow_distributed_learning_amd.models.mnist_cnn import reference_logits

    params = [torch.from_numpy(w).double() for w in m.get_weights()]
    ref = reference_logits(params, xv.double()).numpy()
    np.testing.assert_allclose(fused, ref, rtol=1e-4, atol=1e-5)


def test_fit_with_validation_data_and_training_metrics_untouched():
    m = _model()
    x, y = _data(1024, 3)
    xv, yv = _data(500, 4)
    h = m.fit(tdl.data.Dataset.from_tensor_slices((x, y)).batch(64).repeat(), epochs=2, steps_per_epoch=4,
              validation_data=(xv, yv), validation_batch_size=50, verbose=0)
    assert len(h.history["val_loss"]) == 2 and np.isfinite(h.history["val_loss"]).all()
    ev = m.evaluate(xv, yv, batch_size=50, return_dict=True, verbose=0)
    np.testing.assert_allclose(h.history["val_loss"][-1], ev["loss"], rtol=1e-6)
    # the training metrics of the last epoch are not mixed with the validation pass
    assert h.history["loss"][-1] != h.history["val_loss"][-1]
