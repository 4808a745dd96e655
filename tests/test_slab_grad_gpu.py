"""Direct gradient-slab writes of the generic engine under mixed_bfloat16 (engine/trainer.py):
one bf16 cast of the whole weight slab per step, the conv weight-gradient kernel adding dW straight
into the f32 slab view, the BN backward adding dgamma/dbeta into it, folded conv biases left at zero.
Training must match the plain autograd accumulation path (TDL_CAST_ACCUMULATE=0)."""
import os

import numpy as np
import pytest
import torch

import tensorflow_distributed_learning_amd as tdl

pytestmark = pytest.mark.gpu


def _model():
    tdl.keras.utils.set_random_seed(5)
    L = tdl.keras.layers
    inp = L.Input(shape=(16, 16, 64))
    x = L.Conv2D(64, 3, padding="same")(inp)
    x = L.BatchNormalization()(x)
    x = L.Activation("relu")(x)
    y = L.Conv2D(64, 1)(x)
    y = L.BatchNormalization()(y)
    x = L.Activation("relu")(L.Add()([x, y]))
    x = L.Conv2D(128, 1, strides=2)(x)  # strided 1x1: hand-written stride-2 input gradient
    x = L.BatchNormalization()(x)
    x = L.Activation("relu")(x)
    x = L.GlobalAveragePooling2D()(x)
    out = L.Dense(10)(x)
    return tdl.keras.Model(inp, out)


def _train(direct: bool, steps=2):
    env = {"TDL_CAST_ACCUMULATE": "1" if direct else "0", "TDL_GRAPH_STEP": "0", "TDL_CONV": "hip"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        tdl.keras.backend.clear_session()
        tdl.keras.mixed_precision.set_global_policy("mixed_bfloat16")
        g = torch.Generator().manual_seed(0)
        x = torch.rand(256, 16, 16, 64, generator=g)
        y = torch.randint(0, 10, (256,), generator=g)
        ds = tdl.data.Dataset.from_tensor_slices((x, y)).batch(64).repeat()
        strategy = tdl.distribute.MirroredStrategy(devices=["/gpu:0"])
        with strategy.scope():
            m = _model()
            m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                      optimizer=tdl.keras.optimizers.SGD(learning_rate=0.05, momentum=0.9))
        h = m.fit(ds, epochs=1, steps_per_epoch=steps, verbose=0)
        return m, h
    finally:
        tdl.keras.mixed_precision.set_global_policy("float32")
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_direct_slab_gradients_match_autograd_accumulation():
    md, hd = _train(True)
    assert md._trainer.kind == "generic" and md._trainer._Wc is not None
    ma, ha = _train(False)
    assert ma._trainer._Wc is None
    for v, a, b in zip(md.weights, md.get_weights(), ma.get_weights()):
        scale = max(float(np.abs(b).max()), 1e-3)
        np.testing.assert_allclose(a, b, atol=5e-2 * scale, rtol=2e-2, err_msg=v.name)  # (the direct path keeps dW in f32, autograd rounds it to bf16)
    np.testing.assert_allclose(hd.history["loss"], ha.history["loss"], rtol=2e-2)
    # folded conv biases before a BN keep exactly their initial value (zero gradient)
    for v in md.weights:
        if "conv" in v.name and v.name.endswith("bias:0"):
            assert float(np.abs(v.numpy()).max()) == 0.0, v.name
