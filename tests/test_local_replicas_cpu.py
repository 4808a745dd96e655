"""Single-process multi-device MirroredStrategy (tf_dist_example.py:13, README.md:15-19): ONE process
drives every device of ``devices=[...]`` (parallel/local_replicas.py), the script body runs once, the
replicas stay bit-identical, and training matches one replica on the same global batches."""
import numpy as np
import pytest
import torch

import tensorflow_distributed_learning_amd as tdl
from tensorflow_distributed_learning_amd.parallel.local_replicas import LocalReplicaGroup
from tensorflow_distributed_learning_amd.parallel.values import PerReplica


def _cnn():
    L = tdl.keras.layers
    return tdl.keras.Sequential([
        L.Conv2D(8, 3, activation="relu", input_shape=(28, 28, 1)), L.MaxPooling2D(),
        L.Flatten(), L.Dense(16, activation="relu"), L.Dense(10)])


def _data(n=256, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(n, 28, 28, 1, generator=g), torch.randint(0, 10, (n,), generator=g)


def _train(strategy, x, y, steps=6):
    tdl.keras.utils.set_random_seed(7)
    ds = tdl.data.Dataset.from_tensor_slices((x, y)).batch(32).repeat()
    with strategy.scope():
        m = _cnn()
        m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tdl.keras.optimizers.SGD(learning_rate=0.05),
                  metrics=[tdl.keras.metrics.SparseCategoricalAccuracy()])
    h = m.fit(ds, epochs=2, steps_per_epoch=steps // 2, verbose=0)
    return m, h


def test_local_group_all_reduce_rank_order_and_broadcast():
    g = LocalReplicaGroup([torch.device("cpu")] * 3)
    xs = [torch.randn(1000, generator=torch.Generator().manual_seed(r)) for r in range(3)]
    want = xs[0] + xs[1] + xs[2]

    def fn(r):
        t = xs[r].clone()
        g.comms[r].all_reduce(t, "sum")
        b = torch.full((4,), float(r))
        g.comms[r].broadcast(b, 2)
        ga = g.comms[r].all_gather(torch.tensor([r]))
        return t, b, ga

    out = g.run(fn)
    for t, b, ga in out:
        assert torch.equal(t, want)  # rank-order sum: bit-identical on every replica
        assert torch.equal(b, torch.full((4,), 2.0))
        assert ga.flatten().tolist() == [0, 1, 2]


def test_local_group_error_in_one_replica_raises_not_hangs():
    g = LocalReplicaGroup([torch.device("cpu")] * 2, timeout=30)

    def fn(r):
        if r == 1:
            raise ValueError("boom")
        g.comms[r].all_reduce(torch.ones(3))

    with pytest.raises(ValueError, match="boom"):
        g.run(fn)


def test_mirrored_two_cpu_devices_one_process_trains_identical_replicas():
    x, y = _data()
    s = tdl.distribute.MirroredStrategy(devices=["/cpu:0", "/cpu:1"])
    assert s.num_replicas_in_sync == 2 and s._local_group is not None
    assert s.extended.rank == 0
    m, h = _train(s, x, y)
    clones = m._local_clones
    assert len(clones) == 1
    for a, b in zip(m.get_weights(), clones[0].get_weights()):
        assert np.array_equal(a, b), "replicas differ"
    assert len(h.history["loss"]) == 2 and np.isfinite(h.history["loss"]).all()
    # the same global batches on ONE replica: the same model up to f32 summation order
    m1, h1 = _train(tdl.distribute.MirroredStrategy(devices=["/cpu:0"]), x, y)
    for a, b in zip(m.get_weights(), m1.get_weights()):
        np.testing.assert_allclose(a, b, rtol=2e-4, atol=2e-5)
    np.testing.assert_allclose(h.history["loss"], h1.history["loss"], rtol=1e-4)
    s.shutdown()


def test_strategy_run_returns_per_replica_values():
    s = tdl.distribute.MirroredStrategy(devices=["/cpu:0", "/cpu:1", "/cpu:2"])

    def step(v):
        ctx = tdl.distribute.get_replica_context()
        rid = ctx.replica_id_in_sync_group
        t = torch.tensor([float(rid + 1)]) * v
        return ctx.all_reduce("SUM", t), torch.tensor([float(rid)])

    tot, ids = s.run(step, args=(torch.tensor([2.0]),))
    assert isinstance(ids, PerReplica)
    assert [float(v) for v in s.experimental_local_results(ids)] == [0.0, 1.0, 2.0]
    assert [float(v) for v in s.experimental_local_results(tot)] == [12.0, 12.0, 12.0]
    assert float(s.reduce("SUM", ids, axis=None)) == 3.0
    assert float(s.reduce("MEAN", ids, axis=None)) == 1.0
    s.shutdown()


def test_script_body_runs_once(tmp_path):
    """The TF semantics the process-per-replica self-spawn could not give: a 2-device script's
    top-level code runs once (one line of output), and fit reports 2 replicas."""
    import os
    import subprocess
    import sys
    import textwrap

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    f = tmp_path / "train.py"
    f.write_text(textwrap.dedent("""
        import torch
        import tensorflow_distributed_learning_amd as tdl
        print("BODY", flush=True)
        s = tdl.distribute.MirroredStrategy(devices=["/cpu:0", "/cpu:1"])
        L = tdl.keras.layers
        x, y = torch.rand(128, 4), torch.randint(0, 3, (128,))
        with s.scope():
            m = tdl.keras.Sequential([L.Dense(8, activation="relu", input_shape=(4,)), L.Dense(3)])
            m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer="sgd")
        m.fit(tdl.data.Dataset.from_tensor_slices((x, y)).batch(32), epochs=1, verbose=0)
        print("REPLICAS", s.num_replicas_in_sync, flush=True)
    """))
    env = dict(os.environ, PYTHONPATH=root, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "TF_CONFIG", "TDL_LAUNCHED"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, str(f)], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("BODY") == 1, r.stdout
    assert "REPLICAS 2" in r.stdout


def _dense_model():
    L = tdl.keras.layers
    return tdl.keras.Sequential([L.Dense(8, activation="relu", input_shape=(8,)), L.Dense(3)])


def _xy(n=256):
    g = torch.Generator().manual_seed(0)
    return torch.rand(n, 8, generator=g), torch.randint(0, 3, (n,), generator=g)


def test_one_training_loop_shares_callbacks_state_with_every_replica():
    """ONE fit loop drives both replicas (engine/mirrored.py): EarlyStopping ends training on every
    replica, a LearningRateScheduler reaches the clone's optimizer, iterations stay in step."""
    x, y = _xy()
    s = tdl.distribute.MirroredStrategy(devices=["/cpu:0", "/cpu:1"])
    with s.scope():
        m = _dense_model()
        m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tdl.keras.optimizers.SGD(0.1))
    ds = tdl.data.Dataset.from_tensor_slices((x, y)).batch(32).repeat()
    cb = [tdl.keras.callbacks.LearningRateScheduler(lambda e, lr: 0.1 * (0.5 ** e)),
          tdl.keras.callbacks.EarlyStopping(monitor="loss", patience=0, min_delta=10.0)]
    h = m.fit(ds, epochs=5, steps_per_epoch=4, verbose=0, callbacks=cb)
    assert len(h.history["loss"]) == 2  # stopped after epoch 1 (no 10.0 improvement), not hung
    assert getattr(m._trainer, "is_group", False)
    (c,) = m._local_clones
    assert c.optimizer.current_lr() == m.optimizer.current_lr() == 0.05
    assert c.optimizer.iterations == m.optimizer.iterations == 8
    for a, b in zip(m.get_weights(), c.get_weights()):
        assert np.array_equal(a, b)
    s.shutdown()


def test_replicas_receive_restored_weights_and_optimizer_state(tmp_path):
    """Weights / optimizer slots set on replica 0 between fits (load_weights, a restored optimizer)
    reach every replica before the next step."""
    x, y = _xy()
    s = tdl.distribute.MirroredStrategy(devices=["/cpu:0", "/cpu:1"])
    with s.scope():
        m = _dense_model()
        m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tdl.keras.optimizers.Adam(0.01))
    ds = tdl.data.Dataset.from_tensor_slices((x, y)).batch(32).repeat()
    m.fit(ds, epochs=1, steps_per_epoch=2, verbose=0)
    (c,) = m._local_clones
    new = [w * 0 + 0.01 for w in m.get_weights()]
    m.set_weights(new)
    m.optimizer.iterations = 100
    for v in m.optimizer.slots().values():
        v.fill_(0.5)
    m._trainer.broadcast_from_primary()
    for a, b in zip(new, c.get_weights()):
        assert np.array_equal(a, b)
    assert c.optimizer.iterations == 100
    assert all(float(v.min()) == 0.5 for v in c.optimizer.slots().values())
    m.fit(ds, epochs=1, steps_per_epoch=2, verbose=0)
    for a, b in zip(m.get_weights(), c.get_weights()):
        assert np.array_equal(a, b)
    s.shutdown()


def test_custom_training_loop_per_replica_inputs_and_merged_update():
    """strategy.experimental_distribute_dataset yields PerReplica slices of ONE pipeline, and
    apply_gradients inside strategy.run is a merge call: the replicas' gradients are summed and the
    variables updated once -- the same as one replica on the whole global batch."""
    from tensorflow_distributed_learning_amd.compat import tf

    x, y = _xy(128)
    s = tdl.distribute.MirroredStrategy(devices=["/cpu:0", "/cpu:1"])
    with s.scope():
        m = _dense_model()
        opt = tdl.keras.optimizers.SGD(0.1)
    loss_fn = tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True, reduction="none")
    dist = s.experimental_distribute_dataset(tdl.data.Dataset.from_tensor_slices((x, y)).batch(64))
    batch = next(iter(dist))
    assert isinstance(batch[0], PerReplica) and [len(v) for v in batch[0].values] == [32, 32]

    def step(b):
        xb, yb = b
        with tf.GradientTape() as tape:
            loss = loss_fn(yb, m(xb, training=True)).sum() / 64.0
        grads = tape.gradient(loss, m.trainable_variables)
        opt.apply_gradients(zip(grads, m.trainable_variables))
        return loss.detach()

    w0 = [w.copy() for w in m.get_weights()]
    s.run(step, args=(batch,))
    ref = _dense_model()
    ref.set_weights(w0)
    ropt = tdl.keras.optimizers.SGD(0.1)
    xb = torch.cat(batch[0].values)
    yb = torch.cat(batch[1].values)
    with tf.GradientTape() as tape:
        loss = loss_fn(yb, ref(xb, training=True)).sum() / 64.0
    ropt.apply_gradients(zip(tape.gradient(loss, ref.trainable_variables), ref.trainable_variables))
    for a, b in zip(m.get_weights(), ref.get_weights()):
        np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-7)
    # distribute_datasets_from_function: consecutive per-replica batches form one step
    ddf = s.distribute_datasets_from_function(
        lambda ctx: tdl.data.Dataset.from_tensor_slices((x, y)).batch(ctx.get_per_replica_batch_size(64)))
    b2 = next(iter(ddf))
    assert isinstance(b2[0], PerReplica) and torch.equal(torch.cat(b2[0].values), x[:64])
    s.shutdown()


def test_replicas_reaching_different_collectives_fail_fast():
    g = LocalReplicaGroup([torch.device("cpu")] * 2, timeout=300)

    def fn(r):
        if r == 0:
            g.comms[r].all_reduce(torch.ones(3))

    import time

    t0 = time.monotonic()
    with pytest.raises(RuntimeError, match="different collectives"):
        g.run(fn)
    assert time.monotonic() - t0 < 30


def test_adam_with_clipping_is_not_graph_safe():
    """A clipped Adam update runs the torch fallback whose lr / step are host values: the whole-step
    graph must not capture it."""
    assert not tdl.keras.optimizers.Adam(0.01, clipnorm=1.0).graph_safe
    assert not tdl.keras.optimizers.Adam(0.01, clipvalue=0.5).graph_safe
