"""Probe: generic-engine whole-step graph vs eager, step by step (weights after every step)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import tensorflow_distributed_learning_amd as tdl  # noqa: E402
from tensorflow_distributed_learning_amd.engine.trainer import HostDataHandler  # noqa: E402


def model_small(policy):
    tdl.keras.mixed_precision.set_global_policy(policy)
    tdl.keras.utils.set_random_seed(1)
    L = tdl.keras.layers
    inp = L.Input(shape=(16, 16, 8))
    x = L.Conv2D(16, 3, padding="same")(inp)
    x = L.BatchNormalization()(x)
    x = L.Activation("relu")(x)
    y = L.Conv2D(16, 3, padding="same")(x)
    y = L.BatchNormalization()(y)
    x = L.Activation("relu")(L.Add()([x, y]))
    x = L.GlobalAveragePooling2D()(x)
    return tdl.keras.Model(inp, L.Dense(10)(x))


def run(graph, policy, steps, n, device_data):
    os.environ["TDL_GRAPH_STEP"] = "1" if graph else "0"
    tdl.keras.backend.clear_session()
    g = torch.Generator().manual_seed(0)
    x = torch.rand(n, 16, 16, 8, generator=g)
    y = torch.randint(0, 10, (n,), generator=g)
    if device_data:
        x, y = x.cuda(), y.cuda()
    ds = tdl.data.Dataset.from_tensor_slices((x, y)).batch(64).repeat()
    strategy = tdl.distribute.MirroredStrategy(devices=["/gpu:0"])
    with strategy.scope():
        m = model_small(policy)
        m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tdl.keras.optimizers.SGD(0.1, momentum=0.9))
    tr = m._get_trainer()
    h = HostDataHandler(ds, strategy)
    out = []
    for s in range(steps):
        tr.run_train(h, 1)
        torch.cuda.synchronize()
        out.append(np.concatenate([w.ravel() for w in m.get_weights()]))
    tdl.keras.mixed_precision.set_global_policy("float32")
    return out


for policy in ():
    for dd in (False, True):
        a = run(True, policy, 8, 300, dd)
        b = run(False, policy, 8, 300, dd)
        print(policy, "device_data" if dd else "host_data",
              [float(np.abs(u - v).max()) for u, v in zip(a, b)], flush=True)


def run_mnist(graph, steps=14):
    from tensorflow_distributed_learning_amd.data.tfds import synthetic_mnist
    from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn

    os.environ["TDL_GRAPH_STEP"] = "1" if graph else "0"
    os.environ["TDL_DISABLE_FUSED"] = "1"
    tdl.keras.backend.clear_session()
    tdl.keras.utils.set_random_seed(3)
    x, y = synthetic_mnist(300, 0)
    ds = tdl.data.Dataset.from_tensor_slices((x.reshape(-1, 28, 28, 1), y)).map(
        lambda i, l: (i.to(torch.float32) / 255, l)).cache().shuffle(1000, seed=7).batch(64).repeat()
    strategy = tdl.distribute.MirroredStrategy(devices=["/gpu:0"])
    with strategy.scope():
        m = build_mnist_cnn()
        m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tdl.keras.optimizers.SGD(learning_rate=0.05))
    tr = m._get_trainer()
    h = HostDataHandler(ds, strategy)
    out = []
    for s in range(steps):
        tr.run_train(h, 1)
        torch.cuda.synchronize()
        out.append(np.concatenate([w.ravel() for w in m.get_weights()]))
    return out


a = run_mnist(True)
a2 = run_mnist(True)
b = run_mnist(False)
print("mnist graph-eager", [float(np.abs(u - v).max()) for u, v in zip(a, b)])
print("mnist graph-graph", [float(np.abs(u - v).max()) for u, v in zip(a, a2)])
sizes = [288, 32, 18432, 64, 204800, 128, 1280, 10]
offs = np.cumsum([0] + sizes)
for st in (6, 7, 8):
    d = np.abs(a[st] - b[st])
    print("step", st + 1, [float(d[offs[i]:offs[i + 1]].max()) for i in range(len(sizes))])
