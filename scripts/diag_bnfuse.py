"""Which BN-backward fusion variant moves training away from the unfused path (diagnostic)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import tensorflow_distributed_learning_amd as tdl  # noqa: E402
from tensorflow_distributed_learning_amd.ops import conv as CV  # noqa: E402


L = tdl.keras.layers


def bn_relu(t):
    return L.Activation("relu")(L.BatchNormalization()(t))


def block(x, s=1, project=False):
    y = bn_relu(L.Conv2D(64, 1, strides=s)(x))
    y = bn_relu(L.Conv2D(64, 3, padding="same")(y))
    y = L.BatchNormalization()(L.Conv2D(128, 1)(y))
    sc = L.BatchNormalization()(L.Conv2D(128, 1, strides=s)(x)) if project else x
    return L.Activation("relu")(L.Add()([y, sc]))


def model():
    tdl.keras.utils.set_random_seed(11)
    inp = L.Input(shape=(8, 8, 64))
    x = bn_relu(L.Conv2D(64, 3, padding="same")(inp))
    x = block(x, 1, True)
    x = block(x)
    x = block(x, 2, True)
    x = block(x)
    x = L.GlobalAveragePooling2D()(x)
    return tdl.keras.Model(inp, L.Dense(16)(x))


def run(fuse, s2, sc, steps):
    CV._FUSE_BN_BWD[0], CV._FUSE_BN_BWD_S2[0], CV._FUSE_BN_BWD_SHORTCUT[0] = fuse, s2, sc
    os.environ.update({"TDL_GRAPH_STEP": "0", "TDL_CONV": "hip"})
    tdl.keras.backend.clear_session()
    tdl.keras.mixed_precision.set_global_policy("mixed_bfloat16")
    g = torch.Generator().manual_seed(0)
    ds = tdl.data.Dataset.from_tensor_slices((torch.rand(128, 8, 8, 64, generator=g),
                                              torch.randint(0, 16, (128,), generator=g))).batch(32).repeat()
    with tdl.distribute.MirroredStrategy(devices=["/gpu:0"]).scope():
        m = model()
        m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tdl.keras.optimizers.SGD(learning_rate=0.05, momentum=0.9))
    m.fit(ds, epochs=1, steps_per_epoch=steps, verbose=0)
    return m


def worst(m, ref):
    w = []
    for v, a, b in zip(m.weights, m.get_weights(), ref.get_weights()):
        scale = max(float(np.abs(b).max()), 1e-3)
        w.append((round(float(np.abs(a - b).max()) / scale, 4), v.name))
    return sorted(w, reverse=True)[:3]


if __name__ == "__main__":
    runs = [run(False, False, False, 2) for _ in range(2)]
    print("unfused run1 vs run2", worst(runs[0], runs[1]), flush=True)
    f = [run(True, True, True, 2) for _ in range(2)]
    print("fused run1 vs run2", worst(f[0], f[1]), flush=True)
    print("fused run1 vs unfused run2", worst(f[0], runs[1]), flush=True)
