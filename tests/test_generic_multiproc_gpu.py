"""The generic (autograd) engine with REAL peer replicas on the box's one GPU: a small NHWC bf16
CNN of ResNet-style blocks trains with 2 and 4 replica processes sharing the GPU (gloo control
plane, the xGMI all-reduce kernel as the device data plane), gradient buckets launched from the
backward hooks on a side stream and recorded in the whole-step hipGraph.  Replicas must stay
bit-identical and the loss must match one replica on the same global batch within bf16 tolerance.
Also the BASELINE config-5 layout (2 TF_CONFIG workers x 2 replica processes) on that model."""
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
out = sys.argv[1]
if os.environ.get("TF_CONFIG"):
    strategy = tdl.distribute.MultiWorkerMirroredStrategy()
else:
    strategy = tdl.distribute.MirroredStrategy()
R = strategy.num_replicas_in_sync
tdl.keras.mixed_precision.set_global_policy("mixed_bfloat16")
tdl.keras.utils.set_random_seed(3)
g = torch.Generator().manual_seed(0)
x = torch.rand(512, 16, 16, 64, generator=g)
y = torch.randint(0, 10, (512,), generator=g)
ds = tdl.data.Dataset.from_tensor_slices((x, y)).batch(64).repeat()
L = tdl.keras.layers
with strategy.scope():
    inp = L.Input(shape=(16, 16, 64))
    h = L.Activation("relu")(L.BatchNormalization()(L.Conv2D(64, 3, padding="same")(inp)))
    r = L.BatchNormalization()(L.Conv2D(64, 1)(h))
    h = L.Activation("relu")(L.Add()([h, r]))
    h = L.Activation("relu")(L.BatchNormalization()(L.Conv2D(128, 3, strides=2, padding="same")(h)))
    r = L.BatchNormalization()(L.Conv2D(128, 3, padding="same")(h))
    h = L.Activation("relu")(L.Add()([h, r]))
    h = L.GlobalAveragePooling2D()(h)
    m = tdl.keras.Model(inp, L.Dense(10)(h))
    m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
              optimizer=tdl.keras.optimizers.SGD(learning_rate=0.05, momentum=0.9), bucket_bytes=200_000,
              steps_per_execution=int(os.environ.get("TDL_TEST_SPE", "1")))
hist = m.fit(ds, epochs=2, steps_per_epoch=5, verbose=0)
tr = m._trainer
w = np.concatenate([v.ravel() for v in m.get_weights()]).astype(np.float64)
rank = strategy.extended.rank
np.save(os.path.join(out, f"w{rank}_{R}.npy"), w)
comm = strategy.extended.communicator
from tensorflow_distributed_learning_amd.ops import conv as CV
json.dump({"choices": sorted([str(k), v] for k, v in CV.choices().items()), "loss": hist.history["loss"], "engine": tr.kind, "comm": comm.name,
           "algorithm": getattr(comm, "algorithm", comm.name), "buckets": tr.plan.n_buckets,
           "bucketed": tr._buckets is not None, "graphs": len(tr._graphs), "fired": len(getattr(tr, "_works", [])),
           "task": [strategy.extended.task_type, strategy.extended.task_id]},
          open(os.path.join(out, f"r{rank}_{R}.json"), "w"))
"""


def _run(tmp_path, args, conv="hip", spe=1):
    s = tmp_path / "job.py"
    s.write_text(textwrap.dedent(BODY))
    env = dict(os.environ, PYTHONPATH=ROOT, TDL_SHARE_GPU="1", TDL_CONV=conv, TDL_TEST_SPE=str(spe))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "TF_CONFIG"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "tensorflow_distributed_learning_amd.launch"] + args + [str(s), str(tmp_path)],
                       env=env, capture_output=True, text=True, timeout=400, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]


@pytest.fixture(scope="module")
def single(tmp_path_factory):
    d = tmp_path_factory.mktemp("single")
    _run(d, ["--nproc-per-node", "1"])
    return json.load(open(d / "r0_1.json"))


def _check(tmp_path, R, single):
    res = [json.load(open(tmp_path / f"r{i}_{R}.json")) for i in range(R)]
    ws = [np.load(tmp_path / f"w{i}_{R}.npy") for i in range(R)]
    for r in res:
        assert r["engine"] == "generic" and r["comm"] == "gloo" and "xgmi" in r["algorithm"], r
        assert r["bucketed"] and r["buckets"] > 1 and r["fired"] == r["buckets"], r  # every bucket's hook fired
        assert r["graphs"] >= 1, r  # the whole step (incl. the hook-launched exchanges) was captured
    assert all(np.array_equal(ws[0], w) for w in ws[1:]), "replicas diverged"
    np.testing.assert_allclose(res[0]["loss"], single["loss"], rtol=3e-2)
    return res


@pytest.mark.parametrize("R", [2, 4])
def test_generic_bucketed_xgmi_replicas(tmp_path, R, single):
    _run(tmp_path, ["--nproc-per-node", str(R)])
    _check(tmp_path, R, single)


def test_generic_device_execution_graphs_two_replicas(tmp_path, single):
    """steps_per_execution=3 over the device-resident input: each execution is ONE captured graph
    of 3 steps whose bucket exchanges are launched from the backward hooks inside it."""
    _run(tmp_path, ["--nproc-per-node", "2"], spe=3)
    _check(tmp_path, 2, single)


def test_generic_config5_layout_two_workers_two_replicas(tmp_path, single):
    _run(tmp_path, ["--local-workers", "2", "--gpus-per-worker", "2"])
    res = _check(tmp_path, 4, single)
    assert [r["task"] for r in res] == [["worker", 0], ["worker", 0], ["worker", 1], ["worker", 1]]


def test_autotune_decisions_identical_on_every_rank(tmp_path, single):
    """TDL_CONV=auto with two replicas: rank 0 times the candidates and broadcasts every decision
    (ops/conv.py _agree), so both replicas record the same kernel choice for every (direction,
    shape) and stay bit-identical."""
    _run(tmp_path, ["--nproc-per-node", "2"], conv="auto")
    res = [json.load(open(tmp_path / f"r{i}_2.json")) for i in range(2)]
    assert res[0]["choices"], "the autotuner made no decision"
    assert res[0]["choices"] == res[1]["choices"]
    ws = [np.load(tmp_path / f"w{i}_2.npy") for i in range(2)]
    assert np.array_equal(ws[0], ws[1]), "replicas diverged"
