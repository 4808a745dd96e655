"""Fused MI355X engine with 2 replica processes sharing the box's GPU over the native RING
communicator: replicas stay bit-identical and train like one replica on the global batch."""
import json
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

BODY = """
import json, os, sys, numpy as np, torch
import tensorflow_distributed_learning_amd as tdl
from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn
from tensorflow_distributed_learning_amd.data.tfds import synthetic_mnist
out = sys.argv[1]
strategy = tdl.distribute.MirroredStrategy(communication=os.environ.get("JOB_COMM") or None)
R = strategy.num_replicas_in_sync
tdl.keras.utils.set_random_seed(5)
x, y = synthetic_mnist(2048, 2)
ds = tdl.data.Dataset.from_tensor_slices((x.reshape(-1, 28, 28, 1), y))
ds = ds.map(lambda i, l: (i.to(torch.float32) / 255, l)).cache().shuffle(2048, seed=9).batch(128).repeat()
with strategy.scope():
    m = build_mnist_cnn()
    m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
              optimizer=tdl.keras.optimizers.SGD(0.01), metrics=["sparse_categorical_accuracy"],
              steps_per_execution=4)
h = m.fit(ds, epochs=2, steps_per_epoch=8, verbose=0)
w = np.concatenate([v.ravel() for v in m.get_weights()])
np.save(os.path.join(out, f"w{strategy.extended.rank}_{R}.npy"), w)
comm = strategy.extended.communicator
json.dump({"loss": h.history["loss"], "engine": m._trainer.kind, "comm": comm.name,
           "algorithm": getattr(comm, "algorithm", comm.name), "graph": bool(m._trainer.capture_comm)},
          open(os.path.join(out, f"r{strategy.extended.rank}_{R}.json"), "w"))
"""


def _run(tmp_path, n, comm="RING"):
    s = tmp_path / "job.py"
    s.write_text(textwrap.dedent(BODY))
    env = dict(os.environ, PYTHONPATH=ROOT, TDL_SHARE_GPU="1", JOB_COMM=comm)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "TF_CONFIG"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "tensorflow_distributed_learning_amd.launch", "--nproc-per-node", str(n),
                        str(s), str(tmp_path)], env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]


def test_fused_two_replicas_match_single(tmp_path):
    _run(tmp_path, 1)
    _run(tmp_path, 2)
    r1 = json.load(open(tmp_path / "r0_1.json"))
    a, b = (json.load(open(tmp_path / f"r{i}_2.json")) for i in range(2))
    assert r1["engine"] == a["engine"] == "fused" and a["comm"] == "ring"
    w0, w1, ws = (np.load(tmp_path / f) for f in ("w0_2.npy", "w1_2.npy", "w0_1.npy"))
    assert np.array_equal(w0, w1)
    # lr 0.01: R=2 vs R=1 differ only by fp32 summation order (at lr 0.1 ReLU flips amplify it)
    np.testing.assert_allclose(w0, ws, rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(a["loss"], r1["loss"], rtol=1e-4)


def test_fused_two_replicas_xgmi_auto(tmp_path):
    """AUTO on replicas sharing one GPU: gloo control plane + the xGMI one-shot kernels (IPC),
    all-reduce + SGD fused and captured in the execution graph."""
    _run(tmp_path, 1, comm="")
    _run(tmp_path, 2, comm="")
    a, b = (json.load(open(tmp_path / f"r{i}_2.json")) for i in range(2))
    assert a["engine"] == "fused" and a["comm"] == "gloo"
    assert a["algorithm"] == "xgmi-oneshot+gloo" and a["graph"], a
    w0, w1, ws = (np.load(tmp_path / f) for f in ("w0_2.npy", "w1_2.npy", "w0_1.npy"))
    assert np.array_equal(w0, w1)
    np.testing.assert_allclose(w0, ws, rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(a["loss"], json.load(open(tmp_path / "r0_1.json"))["loss"], rtol=2e-3)


MWMS_BODY = """
import json, os, sys, numpy as np, torch
import tensorflow_distributed_learning_amd as tdl
from tensorflow_distributed_learning_amd.compat import tf
from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn
from tensorflow_distributed_learning_amd.data.tfds import synthetic_mnist
out = sys.argv[1]
strategy = tf.distribute.experimental.MultiWorkerMirroredStrategy(tf.distribute.experimental.CollectiveCommunication.AUTO)
R = strategy.num_replicas_in_sync
ext = strategy.extended
tdl.keras.utils.set_random_seed(5)
x, y = synthetic_mnist(2048, 2)
ds = tdl.data.Dataset.from_tensor_slices((x.reshape(-1, 28, 28, 1), y))
ds = ds.map(lambda i, l: (i.to(torch.float32) / 255, l)).cache().shuffle(2048, seed=9).batch(64 * R).repeat()
opts = tdl.data.Options()
opts.experimental_distribute.auto_shard_policy = tdl.data.AutoShardPolicy.DATA
ds = ds.with_options(opts)
with strategy.scope():
    m = build_mnist_cnn()
    m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
              optimizer=tdl.keras.optimizers.SGD(0.01), metrics=["sparse_categorical_accuracy"],
              steps_per_execution=4)
h = m.fit(ds, epochs=2, steps_per_epoch=8, verbose=0)
w = np.concatenate([v.ravel() for v in m.get_weights()])
np.save(os.path.join(out, f"mw{ext.rank}.npy"), w)
comm = ext.communicator
json.dump({"R": R, "rank": ext.rank, "task": [ext.task_type, ext.task_id], "engine": m._trainer.kind,
           "algorithm": getattr(comm, "algorithm", comm.name), "loss": h.history["loss"],
           "device": str(ext.device)}, open(os.path.join(out, f"mw{ext.rank}.json"), "w"))
"""


def test_config5_shape_two_workers_two_gpus_each(tmp_path):
    """BASELINE config 5's layout (TF_CONFIG workers x GPUs per worker, auto-shard DATA) at 2 x 2,
    the 4 replica processes sharing this box's GPU: every replica ends bit-identical, the task
    layout follows TF_CONFIG, and training progresses."""
    s = tmp_path / "job.py"
    s.write_text(textwrap.dedent(MWMS_BODY))
    env = dict(os.environ, PYTHONPATH=ROOT, TDL_SHARE_GPU="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "TF_CONFIG"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "tensorflow_distributed_learning_amd.launch", "--local-workers", "2",
                        "--gpus-per-worker", "2", str(s), str(tmp_path)], env=env, capture_output=True, text=True,
                       timeout=400, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    res = [json.load(open(tmp_path / f"mw{i}.json")) for i in range(4)]
    assert [d["R"] for d in res] == [4] * 4 and all(d["engine"] == "fused" for d in res)
    assert [tuple(d["task"]) for d in res] == [("worker", 0), ("worker", 0), ("worker", 1), ("worker", 1)]
    ws = [np.load(tmp_path / f"mw{i}.npy") for i in range(4)]
    assert all(np.array_equal(ws[0], w) for w in ws[1:])
    assert res[0]["loss"] == res[3]["loss"] and res[0]["loss"][-1] < res[0]["loss"][0]
