"""The generic engine's device-resident executions (engine/trainer.py GenericTrainer.prepare /
_run_device): an in-memory pipeline is uploaded once and each execution of steps_per_execution
steps is ONE captured hipGraph gathering its batches from HBM.  It must train exactly like the host
pipeline path (same batches in the same order, same kernels): weights, optimizer state and metrics
compared after several executions, including a partial final batch and Adam's per-step bias
correction inside a multi-step graph."""
import numpy as np
import pytest
import torch

import tensorflow_distributed_learning_amd as tdl

pytestmark = pytest.mark.gpu


def _model(opt):
    L = tdl.keras.layers
    tdl.keras.utils.set_random_seed(3)
    with tdl.distribute.MirroredStrategy(devices=["/gpu:0"]).scope():
        m = tdl.keras.Sequential([L.Conv2D(16, 3, activation="relu", padding="same", input_shape=(28, 28, 1)),
                                  L.MaxPooling2D(), L.Conv2D(32, 3, activation="relu"), L.MaxPooling2D(),
                                  L.Flatten(), L.Dense(64, activation="relu"), L.Dense(10)])
        m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=opt(),
                  metrics=["sparse_categorical_accuracy"], steps_per_execution=3)
    return m


def _ds(n):
    g = torch.Generator().manual_seed(0)
    x, y = torch.rand(n, 28, 28, 1, generator=g), torch.randint(0, 10, (n,), generator=g)
    return tdl.data.Dataset.from_tensor_slices((x, y)).shuffle(n, seed=5).batch(32)


@pytest.mark.parametrize("opt", [lambda: tdl.keras.optimizers.SGD(0.05),
                                 lambda: tdl.keras.optimizers.Adam(1e-3)], ids=["sgd", "adam"])
def test_device_executions_match_host_pipeline(monkeypatch, opt):
    monkeypatch.setenv("TDL_DISABLE_FUSED", "1")
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("TDL_GENERIC_DEVICE_DATA", mode)
        tdl.keras.backend.clear_session()
        m = _model(opt)
        # 7 full batches + a partial one per epoch: executions of 3, 3, 1 and the ragged step
        h = m.fit(_ds(7 * 32 + 12), epochs=3, verbose=0)
        tr = m._trainer
        assert tr.kind == "generic"
        if mode == "1":
            assert any(k[0] == "dev" for k in tr._graphs), "no device execution graph was captured"
        out[mode] = (torch.cat([w.reshape(-1) for w in map(torch.as_tensor, m.get_weights())]).cpu(),
                     h.history, tr.optimizer.iterations)
    wd, hd, itd = out["1"]
    wh, hh, ith = out["0"]
    assert itd == ith == 3 * 8
    torch.testing.assert_close(wd, wh, rtol=2e-5, atol=2e-6)
    for k in ("loss", "sparse_categorical_accuracy"):
        np.testing.assert_allclose(hd[k], hh[k], rtol=1e-4)


def test_bench_generic_engine_device_graphs():
    """bench.py --engine generic: every timed step is a replay of a captured multi-step execution."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--engine", "generic", "--steps", "50",
                        "--warmup", "25"], capture_output=True, text=True, timeout=300, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["config"]["engine"] == "generic" and d["config"]["graph_captured"], d
    assert d["value"] > 0
