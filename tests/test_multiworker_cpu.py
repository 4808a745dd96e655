"""Multi-process CPU tests: TF_CONFIG rendezvous, ring all-reduce, MultiWorkerMirroredStrategy
world 2 end-to-end (BASELINE config 1), DATA sharding equivalence, chief-only checkpoints."""
import json
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


def _env(**kw):
    e = dict(os.environ)
    e["PYTHONPATH"] = ROOT
    e["OMP_NUM_THREADS"] = "2"
    e.pop("TF_CONFIG", None)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "TDL_LAUNCHED"):
        e.pop(k, None)
    e["CUDA_VISIBLE_DEVICES"] = ""
    e["HIP_VISIBLE_DEVICES"] = ""
    e.update(kw)
    return e


def _launch(tmp_path, body, args, timeout=240, env=None):
    script = tmp_path / "job.py"
    script.write_text(textwrap.dedent(body))
    cmd = [sys.executable, "-m", "tensorflow_distributed_learning_amd.launch"] + args + [str(script), str(tmp_path)]
    r = subprocess.run(cmd, env=_env(TDL_NO_GPU_PARTITION="1", **(env or {})), cwd=ROOT, capture_output=True,
                       text=True, timeout=timeout)
    return r


def _results(tmp_path, n):
    return [json.load(open(tmp_path / f"out{r}.json")) for r in range(n)]


def test_mwms_world2_trains_identically(tmp_path):
    body = """
    import json, os, sys, numpy as np, torch
    import tensorflow_distributed_learning_amd as tdl
    from tensorflow_distributed_learning_amd.compat import tf, tfds
    from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn
    out = sys.argv[1]
    strategy = tf.distribute.experimental.MultiWorkerMirroredStrategy(
        tf.distribute.experimental.CollectiveCommunication.AUTO)
    R = strategy.num_replicas_in_sync
    (ds, info) = tfds.load('mnist', as_supervised=True, with_info=True)
    def scale(image, label):
        image = tf.cast(image, tf.float32)
        image /= 255
        return image, label
    train = ds['train'].take(2048).map(scale).cache().shuffle(1000).batch(64 * R)
    opts = tf.data.Options()
    opts.experimental_distribute.auto_shard_policy = tf.data.experimental.AutoShardPolicy.OFF
    train = train.with_options(opts)
    with strategy.scope():
        m = build_mnist_cnn()
        m.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tf.keras.optimizers.SGD(learning_rate=0.05),
                  metrics=[tf.keras.metrics.SparseCategoricalAccuracy()])
    h = m.fit(x=train, epochs=3, steps_per_epoch=5, verbose=0)
    ck = os.path.join(out, "ckpt")
    m.save(os.path.join(out, "saved"))
    w = np.concatenate([x.ravel() for x in m.get_weights()])
    json.dump({"rank": strategy.extended.rank, "R": R, "comm": strategy.extended.communicator.name,
               "task": [strategy.extended.task_type, strategy.extended.task_id],
               "hash": float(np.abs(w).sum()), "w0": float(w[0]), "loss": h.history["loss"]},
              open(os.path.join(out, f"out{strategy.extended.rank}.json"), "w"))
    """
    r = _launch(tmp_path, body, ["--local-workers", "2"])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    a, b = _results(tmp_path, 2)
    assert a["R"] == 2 and a["comm"] == "ring" and a["task"] == ["worker", 0] and b["task"] == ["worker", 1]
    assert a["hash"] == b["hash"] and a["w0"] == b["w0"]  # replicas stay bit-identical
    assert a["loss"] == b["loss"]  # logged metrics are cross-replica reduced
    assert a["loss"][-1] < a["loss"][0]
    assert os.path.exists(tmp_path / "saved" / "saved_model.json")  # chief wrote
    assert not any(p.startswith("workertemp") for p in os.listdir(tmp_path))  # non-chief temp removed


def test_data_sharding_equals_single_replica_global_batch(tmp_path):
    body = """
    import json, os, sys, numpy as np, torch
    import tensorflow_distributed_learning_amd as tdl
    from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn
    out = sys.argv[1]
    impl = os.environ.get("IMPL", "AUTO")
    strategy = tdl.distribute.MirroredStrategy(communication=impl)
    R = strategy.num_replicas_in_sync
    tdl.keras.utils.set_random_seed(5)
    from tensorflow_distributed_learning_amd.data.tfds import synthetic_mnist
    x, y = synthetic_mnist(512, 2)
    ds = tdl.data.Dataset.from_tensor_slices((x.reshape(-1, 28, 28, 1).astype(np.float32) / 255, y))
    ds = ds.shuffle(512, seed=9).batch(128)   # AUTO -> DATA sharding: disjoint slices of each global batch
    with strategy.scope():
        m = build_mnist_cnn()
        m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tdl.keras.optimizers.SGD(0.1), metrics=["accuracy"])
    h = m.fit(ds, epochs=2, verbose=0)
    w = np.concatenate([v.ravel() for v in m.get_weights()])
    np.save(os.path.join(out, f"w{strategy.extended.rank}_{R}.npy"), w)
    json.dump({"loss": h.history["loss"], "comm": strategy.extended.communicator.name},
              open(os.path.join(out, f"out{strategy.extended.rank}.json"), "w"))
    """
    r = _launch(tmp_path, body, ["--nproc-per-node", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    single = np.load(tmp_path / "w0_1.npy")
    l1 = _results(tmp_path, 1)[0]["loss"]
    for impl in ("RING", "AUTO"):
        r = _launch(tmp_path, body, ["--nproc-per-node", "2"], env={"IMPL": impl})
        assert r.returncode == 0, r.stderr[-3000:]
        w0, w1 = np.load(tmp_path / "w0_2.npy"), np.load(tmp_path / "w1_2.npy")
        assert np.array_equal(w0, w1)
        np.testing.assert_allclose(w0, single, rtol=1e-4, atol=1e-6)
        res = _results(tmp_path, 2)
        np.testing.assert_allclose(res[0]["loss"], l1, rtol=1e-4)


def test_duplicate_task_rejected_and_ps_refused(tmp_path):
    body = """
    import sys
    import tensorflow_distributed_learning_amd as tdl
    try:
        s = tdl.distribute.MultiWorkerMirroredStrategy(timeout=20)
        print("JOINED", s.extended.rank, flush=True)
        import time; time.sleep(6)  # keep the cluster up while the duplicate tries to join
    except Exception as e:
        print("ERR", type(e).__name__, e)
        sys.exit(3)
    """
    from tensorflow_distributed_learning_amd.parallel.launch import free_ports

    p0, p1 = free_ports(2)
    tfc = json.dumps({"cluster": {"worker": [f"127.0.0.1:{p0}", f"127.0.0.1:{p1}"]}, "task": {"type": "worker", "index": 1}})
    script = tmp_path / "dup.py"
    script.write_text(textwrap.dedent(body))
    chief = json.dumps({"cluster": {"worker": [f"127.0.0.1:{p0}", f"127.0.0.1:{p1}"]}, "task": {"type": "worker", "index": 0}})
    procs = [subprocess.Popen([sys.executable, str(script)], env=_env(TF_CONFIG=c), stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for c in (chief, tfc, tfc)]
    outs = [p.communicate(timeout=120)[0] for p in procs]
    # exactly one of the two processes claiming worker/1 is rejected with a clear message
    assert sum("already taken" in o for o in outs) == 1, outs
    assert "JOINED 0" in outs[0]
    ps = json.dumps({"cluster": {"worker": ["127.0.0.1:1"], "ps": ["127.0.0.1:2"]}, "task": {"type": "ps", "index": 0}})
    r = subprocess.run([sys.executable, str(script)], env=_env(TF_CONFIG=ps), capture_output=True, text=True, timeout=60)
    assert r.returncode == 3 and "ps" in r.stdout


def test_launcher_propagates_failure(tmp_path):
    body = """
    import os, sys, time
    if os.environ["RANK"] == "1":
        sys.exit(7)
    time.sleep(60)
    """
    r = _launch(tmp_path, body, ["--nproc-per-node", "2"], timeout=60)
    assert r.returncode == 7


def test_corrupted_replica_detected_and_repaired(tmp_path):
    """A replica whose weights are silently corrupted mid-training (as a broken fabric hand-off
    would) is detected by fit's periodic fingerprint check, re-synchronised from rank 0, and
    raises instead under TDL_REPLICA_MISMATCH=raise."""
    body = """
    import json, os, sys, warnings, numpy as np, torch
    import tensorflow_distributed_learning_amd as tdl
    from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn
    from tensorflow_distributed_learning_amd.parallel import consistency
    out = sys.argv[1]
    strategy = tdl.distribute.MirroredStrategy(communication="RING")
    rank = strategy.extended.rank
    from tensorflow_distributed_learning_amd.data.tfds import synthetic_mnist
    x, y = synthetic_mnist(512, 2)
    ds = tdl.data.Dataset.from_tensor_slices((x.reshape(-1, 28, 28, 1).astype(np.float32) / 255, y)).batch(64).repeat()
    with strategy.scope():
        m = build_mnist_cnn()
        m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tdl.keras.optimizers.SGD(0.05))

    class Corrupt(tdl.keras.callbacks.Callback):
        def on_epoch_end(self, epoch, logs=None):
            if epoch == 0 and rank == 1:
                with torch.no_grad():
                    m._W.view(-1)[12345] += 1e-3   # one parameter of one replica drifts
    comm = strategy.extended.communicator
    status = {}
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        m.fit(ds, epochs=3, steps_per_epoch=2, verbose=0, callbacks=[Corrupt()])
    status["warned"] = any("replica divergence" in str(w.message) for w in rec)
    status["identical_after"] = consistency.replicas_identical(comm, m._W)
    # strict mode: the same drift raises on every rank
    if rank == 1:
        with torch.no_grad():
            m._W.view(-1)[7] -= 1e-3
    os.environ["TDL_REPLICA_MISMATCH"] = "raise"
    try:
        consistency.check_and_repair(comm, m._W)
        status["raised"] = False
    except consistency.ReplicaDivergenceError:
        status["raised"] = True
    json.dump(status, open(os.path.join(out, f"out{rank}.json"), "w"))
    """
    r = _launch(tmp_path, body, ["--nproc-per-node", "2"], env={"TDL_CHECK_REPLICAS_EVERY": "1"})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    for s in _results(tmp_path, 2):
        assert s["warned"] and s["identical_after"] and s["raised"], s


CORRUPT = """
import json, os, sys, numpy as np, torch
import tensorflow_distributed_learning_amd as tdl
from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn
from tensorflow_distributed_learning_amd.data.tfds import synthetic_mnist
from tensorflow_distributed_learning_amd.parallel.consistency import ReplicaDivergenceError
out = sys.argv[1]
strategy = tdl.distribute.MultiWorkerMirroredStrategy(communication="RING")
rank = strategy.extended.rank
x, y = synthetic_mnist(1024, 3)
ds = tdl.data.Dataset.from_tensor_slices((x.reshape(-1, 28, 28, 1), y))
ds = ds.map(lambda i, l: (i.to(torch.float32) / 255, l)).batch(64).repeat()
with strategy.scope():
    m = build_mnist_cnn()
    m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
              optimizer=tdl.keras.optimizers.SGD(0.05))
res = {"rank": rank}
try:
    m.fit(ds, epochs=2, steps_per_epoch=6, verbose=0)
    res["status"] = "ok"
except ReplicaDivergenceError as e:
    res["status"] = "raised"
    res["error"] = str(e)
w = np.concatenate([v.ravel() for v in m.get_weights()])
res["w"] = [float(w[0]), float(np.abs(w).sum())]
json.dump(res, open(os.path.join(out, f"out{rank}.json"), "w"))
"""


@pytest.mark.parametrize("mode", ["repair", "raise"])
def test_periodic_replica_check_catches_silent_corruption(tmp_path, mode):
    """Rank 1's parameters are silently perturbed after step 2 (TDL_FAULT_CORRUPT_AT_STEP): the
    per-execution consistency check (TDL_CHECK_REPLICAS_EXECUTIONS) repairs them from rank 0 mid-fit,
    or raises on every rank under TDL_REPLICA_MISMATCH=raise."""
    env = {"TDL_FAULT_CORRUPT_AT_STEP": "1:2", "TDL_CHECK_REPLICAS_EXECUTIONS": "1", "TDL_REPLICA_MISMATCH": mode,
           "TDL_CHECK_REPLICAS": "0", "TDL_CHECK_REPLICAS_EVERY": "0"}
    r = _launch(tmp_path, CORRUPT, ["--local-workers", "2"], env=env)
    a, b = _results(tmp_path, 2)
    assert "perturbed" in r.stderr, r.stderr[-2000:]
    if mode == "repair":
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
        assert a["status"] == b["status"] == "ok"
        assert a["w"] == b["w"], (a, b)  # repaired: identical again at the end, with no end-of-fit check
        assert "replica divergence detected" in r.stderr
    else:
        assert a["status"] == b["status"] == "raised", (a, b)
        assert "replica divergence" in a["error"]
