"""Failure semantics on the GPU path (replica processes sharing the box's one GPU, the xGMI
all-reduce kernel between them): a replica killed mid-training ends the whole job within 60 s
instead of leaving the others spinning in the exchange kernel, and a silently corrupted replica is
caught by the periodic consistency check (repaired from rank 0 with the custom all-reduce dropped,
or raised under TDL_REPLICA_MISMATCH=raise)."""
import json
import os
import socket
import subprocess
import sys
import textwrap
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

BODY = """
import json, os, sys, numpy as np, torch
import tensorflow_distributed_learning_amd as tdl
from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn
from tensorflow_distributed_learning_amd.data.tfds import synthetic_mnist
from tensorflow_distributed_learning_amd.parallel.consistency import ReplicaDivergenceError
out = sys.argv[1]
n = int(os.environ.get("JOB_REPLICAS", "2"))
strategy = tdl.distribute.MirroredStrategy(devices=[f"/gpu:{i}" for i in range(n)], spawn=True)
rank = strategy.extended.rank
open(os.path.join(out, f"pid{rank}"), "w").write(str(os.getpid()))
tdl.keras.utils.set_random_seed(5)
x, y = synthetic_mnist(2048, 2)
ds = tdl.data.Dataset.from_tensor_slices((x.reshape(-1, 28, 28, 1), y))
ds = ds.map(lambda i, l: (i.to(torch.float32) / 255, l)).cache().shuffle(2048, seed=9).batch(64 * n).repeat()
with strategy.scope():
    m = build_mnist_cnn()
    m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
              optimizer=tdl.keras.optimizers.SGD(0.01), steps_per_execution=2)
res = {"rank": rank}
try:
    m.fit(ds, epochs=int(os.environ.get("JOB_EPOCHS", "3")), steps_per_epoch=8, verbose=0)
    res["status"] = "ok"
except ReplicaDivergenceError as e:
    res["status"] = "raised"
    res["error"] = str(e)
comm = strategy.extended.communicator
res["algorithm"] = getattr(comm, "algorithm", comm.name)
res["xgmi"] = getattr(comm, "xgmi", None) is not None
res["engine"] = m._trainer.kind
w = np.concatenate([v.ravel() for v in m.get_weights()])
np.save(os.path.join(out, f"w{rank}.npy"), w)
json.dump(res, open(os.path.join(out, f"r{rank}.json"), "w"))
strategy.shutdown()
"""


def _alive(pid):
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split(")")[-1].split()[0] != "Z"
    except OSError:
        return False


def _env(**kw):
    env = dict(os.environ, PYTHONPATH=ROOT, TDL_SHARE_GPU="1", TDL_ABORT_GRACE="10", TDL_HEARTBEAT_INTERVAL="0.5",
               TDL_XGMI_TIMEOUT="15", **kw)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "TF_CONFIG", "TDL_LAUNCHED", "MASTER_ADDR",
              "MASTER_PORT"):
        env.pop(k, None)
    return env


def _script(tmp_path):
    s = tmp_path / "job.py"
    s.write_text(textwrap.dedent(BODY))
    return s


def _pids(tmp_path, n, timeout=120):
    deadline = time.time() + timeout
    while time.time() < deadline:
        ps = [tmp_path / f"pid{r}" for r in range(n)]
        if all(p.exists() and p.read_text() for p in ps):
            return [int(p.read_text()) for p in ps]
        time.sleep(0.2)
    raise AssertionError("replicas did not start")


def test_killed_replica_ends_the_spawned_job(tmp_path):
    """Self-spawned replicas (MirroredStrategy(devices=[2 GPUs]) on the shared GPU): rank 1 dies at
    step 6; rank 0 (its supervisor) exits non-zero at once, nobody keeps spinning in the xGMI kernel."""
    p = subprocess.Popen([sys.executable, str(_script(tmp_path)), str(tmp_path)], cwd=ROOT, env=_env(
        TDL_FAULT_KILL_AT_STEP="1:6", JOB_EPOCHS="50"), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        pids = _pids(tmp_path, 2)
        t0 = time.time()
        _, err = p.communicate(timeout=150)
    finally:
        if p.poll() is None:
            p.kill()
    assert p.returncode != 0 and "fault injection" in err, err[-3000:]
    deadline = time.time() + 20
    while time.time() < deadline and any(_alive(q) for q in pids):
        time.sleep(0.1)
    assert not any(_alive(q) for q in pids)
    assert time.time() - t0 < 60


def test_killed_replica_unsupervised_ranks_exit(tmp_path):
    """Three torchrun-style ranks started independently on the shared GPU: rank 1 dies; ranks 0
    and 2 (blocked in / behind the xGMI exchange) exit non-zero within 60 s (job-liveness watchdog,
    the kernel's bounded wait and the error word checked at entry)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = str(s.getsockname()[1])
    s.close()
    procs = []
    for r in range(3):
        env = _env(TDL_FAULT_KILL_AT_STEP="1:6", JOB_EPOCHS="50", JOB_REPLICAS="3", RANK=str(r), WORLD_SIZE="3",
                   LOCAL_RANK=str(r), LOCAL_WORLD_SIZE="3", MASTER_ADDR="127.0.0.1", MASTER_PORT=port,
                   TDL_LAUNCHED="1")
        procs.append(subprocess.Popen([sys.executable, str(_script(tmp_path)), str(tmp_path)], cwd=ROOT, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    _pids(tmp_path, 3)
    t0 = time.time()
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise AssertionError("a surviving rank hung after the fault")
        outs.append((p.returncode, e))
    assert outs[1][0] == 43, outs[1][1][-2000:]
    for r in (0, 2):
        assert outs[r][0] != 0, outs[r][1][-3000:]
    assert time.time() - t0 < 60


@pytest.mark.parametrize("mode", ["repair", "raise"])
def test_corrupted_replica_is_caught(tmp_path, mode):
    r = subprocess.run([sys.executable, str(_script(tmp_path)), str(tmp_path)], cwd=ROOT, capture_output=True, text=True,
                       timeout=300, env=_env(TDL_FAULT_CORRUPT_AT_STEP="1:4", TDL_CHECK_REPLICAS_EXECUTIONS="1",
                                             TDL_REPLICA_MISMATCH=mode, TDL_CHECK_REPLICAS="0",
                                             TDL_CHECK_REPLICAS_EVERY="0"))
    assert "perturbed" in r.stderr, r.stderr[-3000:]
    assert all((tmp_path / f"r{i}.json").exists() for i in range(2)), r.stderr[-4000:]
    a, b = (json.load(open(tmp_path / f"r{i}.json")) for i in range(2))
    assert a["engine"] == "fused"
    if mode == "repair":
        assert r.returncode == 0, r.stderr[-3000:]
        assert a["status"] == b["status"] == "ok"
        assert "replica divergence detected" in r.stderr
        assert not a["xgmi"] and not b["xgmi"]  # the custom all-reduce path was dropped
        assert np.array_equal(np.load(tmp_path / "w0.npy"), np.load(tmp_path / "w1.npy"))
    else:
        assert a["status"] == b["status"] == "raised", (a, b)


def test_live_rank_out_of_step_ends_the_job(tmp_path):
    """A LIVE replica leaves out one gradient all-reduce (the xGMI bucket exchanges of the generic
    engine on the shared GPU): its peer waits in the exchange kernel while both keep heartbeating.
    The progress watchdog (utils/fault.py) and the bounded collective waits must end EVERY rank
    non-zero -- within 150 s, not the 30 minutes of an unbounded collective."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = str(s.getsockname()[1])
    s.close()
    procs = []
    for r in range(2):
        env = _env(TDL_FAULT_SKIP_ALLREDUCE_AT_STEP="1:1", JOB_EPOCHS="50", JOB_REPLICAS="2", RANK=str(r),
                   WORLD_SIZE="2", LOCAL_RANK=str(r), LOCAL_WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=port,
                   TDL_LAUNCHED="1", TDL_DISABLE_FUSED="1", TDL_GRAPH_STEP="0", TDL_STALL_TIMEOUT="20",
                   TDL_COLLECTIVE_TIMEOUT="40")
        procs.append(subprocess.Popen([sys.executable, str(_script(tmp_path)), str(tmp_path)], cwd=ROOT, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    _pids(tmp_path, 2)
    t0 = time.time()
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=170)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise AssertionError("a rank hung after the out-of-step fault")
        outs.append((p.returncode, e))
    assert "skips its gradient all-reduce" in outs[1][1], outs[1][1][-3000:]
    for r in range(2):
        assert outs[r][0] != 0, outs[r][1][-3000:]
    assert time.time() - t0 < 150
