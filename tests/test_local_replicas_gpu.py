"""Single-process multi-device MirroredStrategy on the GPU (tf_dist_example.py:13, README.md:15-19):
ONE process, ONE host thread drives every replica's device (engine/mirrored.py).  The reference CNN
trains on the fused MI355X kernels with each replica's execution captured into a hipGraph on its
device and the gradient all-reduce inside those graphs (xGMI over in-process channels); replicas stay
bit-identical and match one replica on the same global batches.  The devices are mapped onto the
box's one GPU (TDL_SHARE_GPU=1)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import tensorflow_distributed_learning_amd as tdl
from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _fit(strategy, steps=8, opt=None):
    tdl.keras.utils.set_random_seed(11)
    g = torch.Generator().manual_seed(3)
    x = torch.rand(1024, 28, 28, 1, generator=g)
    y = torch.randint(0, 10, (1024,), generator=g, dtype=torch.int64)
    ds = tdl.data.Dataset.from_tensor_slices((x, y)).batch(64).repeat()
    with strategy.scope():
        m = build_mnist_cnn()
        m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=opt or tdl.keras.optimizers.SGD(learning_rate=0.05),
                  metrics=[tdl.keras.metrics.SparseCategoricalAccuracy()], steps_per_execution=4)
    h = m.fit(ds, epochs=2, steps_per_epoch=steps // 2, verbose=0)
    return m, h


@pytest.mark.parametrize("dp2", ["0", "1"], ids=["standalone-xgmi", "xgmi-in-finalize"])
def test_two_devices_one_process_one_thread_device_path(monkeypatch, dp2):
    monkeypatch.setenv("TDL_SHARE_GPU", "1")
    monkeypatch.setenv("TDL_MNIST_DP2_FWD", dp2)  # dp2 = 1: the fused backward -> exchange in finalize
    monkeypatch.setenv("TDL_XGMI_TIMEOUT", "30")
    s = tdl.distribute.MirroredStrategy(devices=["/gpu:0", "/gpu:1"])
    assert s.num_replicas_in_sync == 2 and s._local_group is not None
    m, h = _fit(s)
    tr = m._trainer
    assert type(tr).__name__ == "MirroredFusedTrainer", getattr(m, "_fused_reason", None)
    want = "xgmi-in-finalize" if dp2 == "1" else "xgmi-oneshot-in-graph"
    assert tr.allreduce_mode == want and tr.capture_comm and tr.fallbacks == [], (tr.allreduce_mode, tr.fallbacks)
    assert all(isinstance(g[0], torch.cuda.CUDAGraph) for sub in tr.subs for g in sub._graphs.values())
    assert tr.replicas_identical()
    (c,) = m._local_clones
    for a, b in zip(m.get_weights(), c.get_weights()):
        assert np.array_equal(a, b), "replicas differ"
    m1, h1 = _fit(tdl.distribute.MirroredStrategy(devices=["/gpu:0"]))
    for a, b in zip(m.get_weights(), m1.get_weights()):
        np.testing.assert_allclose(a, b, rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(h.history["loss"], h1.history["loss"], rtol=1e-4)
    ev = m.evaluate(tdl.data.Dataset.from_tensor_slices((torch.rand(256, 28, 28, 1), torch.randint(0, 10, (256,))))
                    .batch(64), verbose=0, return_dict=True)
    assert np.isfinite(ev["loss"])
    s.shutdown()


def test_two_devices_adam_on_device_path(monkeypatch):
    """A non-SGD optimizer: the in-graph all-reduce of the gradient, then each device's Adam kernel."""
    monkeypatch.setenv("TDL_SHARE_GPU", "1")
    monkeypatch.setenv("TDL_XGMI_TIMEOUT", "30")
    s = tdl.distribute.MirroredStrategy(devices=["/gpu:0", "/gpu:1"])
    m, h = _fit(s, opt=tdl.keras.optimizers.Adam(1e-3))
    assert type(m._trainer).__name__ == "MirroredFusedTrainer" and m._trainer.capture_comm
    assert m._trainer.replicas_identical()
    m1, h1 = _fit(tdl.distribute.MirroredStrategy(devices=["/gpu:0"]), opt=tdl.keras.optimizers.Adam(1e-3))
    for a, b in zip(m.get_weights(), m1.get_weights()):
        np.testing.assert_allclose(a, b, rtol=1e-3, atol=2e-5)
    s.shutdown()


def _bench(args, **env_extra):
    env = dict(os.environ, PYTHONPATH=ROOT, **env_extra)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "TF_CONFIG", "TDL_LAUNCHED"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=400, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_single_process_eight_replicas():
    """R = 8 in ONE process (BASELINE config 3's replica count) on the shared GPU: 8 streams, each on
    its own hardware queue (GPU_MAX_HW_QUEUES), every replica's graph holds the two-shot xGMI
    all-reduce with SGD fused; replicas bit-identical, no fallback."""
    d = _bench(["--gpus", "8", "--mode", "single", "--per-replica-batch", "8", "--steps", "20", "--warmup", "5"],
               TDL_SHARE_GPU="1", GPU_MAX_HW_QUEUES="16", TDL_XGMI_TIMEOUT="30")
    cfg = d["config"]
    assert d["n_gpus"] == 8 and cfg["global_batch"] == 64 and cfg["process_model"] == "single-process"
    assert cfg["allreduce"] == "xgmi-twoshot-in-graph", cfg
    assert cfg["allreduce_in_graph"] and cfg["graph_captured"] and cfg["replicas_identical"], cfg
    assert cfg["fallbacks"] == [], cfg


def test_bench_single_process_two_replicas_in_finalize():
    d = _bench(["--gpus", "2", "--mode", "single", "--per-replica-batch", "16", "--steps", "40", "--warmup", "8"],
               TDL_SHARE_GPU="1", TDL_MNIST_DP2_FWD="1", TDL_XGMI_TIMEOUT="30")
    cfg = d["config"]
    assert cfg["allreduce"] == "xgmi-in-finalize" and cfg["kernels_per_step"] == 2, cfg
    assert cfg["replicas_identical"] and cfg["fallbacks"] == [], cfg
