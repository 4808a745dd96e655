"""Model.evaluate / predict of the reference CNN on one MI355X (forward-only path on the gfx950
kernels, engine/fused.py): run under `rocprofv3 --kernel-trace --stats` to list what executes.

    python scripts/eval_profile.py [--n 10000] [--batch 128]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorflow_distributed_learning_amd as tdl  # noqa: E402
from tensorflow_distributed_learning_amd.data.tfds import synthetic_mnist  # noqa: E402
from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10000)
    ap.add_argument("--batch", type=int, default=128)
    a = ap.parse_args()
    strategy = tdl.distribute.MirroredStrategy(devices=["/gpu:0"])
    with strategy.scope():
        m = build_mnist_cnn()
        m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tdl.keras.optimizers.SGD(learning_rate=0.05),
                  metrics=[tdl.keras.metrics.SparseCategoricalAccuracy()], steps_per_execution=10)
    x, y = synthetic_mnist(4096, 0)
    x = torch.from_numpy(np.ascontiguousarray(x)).reshape(-1, 28, 28, 1).float() / 255
    m.fit(tdl.data.Dataset.from_tensor_slices((x, torch.from_numpy(y))).batch(64).repeat(), epochs=1,
          steps_per_epoch=20, verbose=0)
    xv, yv = synthetic_mnist(a.n, 1)
    xv = torch.from_numpy(np.ascontiguousarray(xv)).reshape(-1, 28, 28, 1).float() / 255
    val = tdl.data.Dataset.from_tensor_slices((xv, torch.from_numpy(yv))).batch(a.batch)
    m.evaluate(val, verbose=0)  # warm
    torch.cuda.synchronize()
    t = time.perf_counter()
    out = m.evaluate(val, return_dict=True, verbose=0)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    p = m.predict(tdl.data.Dataset.from_tensor_slices(xv).batch(a.batch), verbose=0)
    print(f"evaluate {a.n} images: {dt * 1e3:.2f} ms ({a.n / dt:,.0f} img/s) -> {out}; predict {p.shape}")


if __name__ == "__main__":
    main()
