"""compile/fit/evaluate/predict + callbacks + checkpoints on CPU (generic engine) – SURVEY C15-C22."""
import json
import os

import numpy as np
import pytest
import torch

import tensorflow_distributed_learning_amd as tdl
from tensorflow_distributed_learning_amd.data.tfds import synthetic_mnist
from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn

keras = tdl.keras


@pytest.fixture(autouse=True)
def _fresh():
    keras.backend.clear_session()
    keras.utils.set_random_seed(1)


def _ds(n=512, B=64, repeat=True):
    x, y = synthetic_mnist(n, 0)
    ds = tdl.data.Dataset.from_tensor_slices((x.reshape(-1, 28, 28, 1), y))
    ds = ds.map(lambda i, l: (i.to(torch.float32) / 255, l)).cache().shuffle(256, seed=0).batch(B)
    return ds.repeat() if repeat else ds


def _model(lr=0.05, **kw):
    m = build_mnist_cnn()
    m.compile(loss=keras.losses.SparseCategoricalCrossentropy(from_logits=True),
              optimizer=keras.optimizers.SGD(learning_rate=lr, **kw),
              metrics=[keras.metrics.SparseCategoricalAccuracy()])
    return m


def test_fit_learns_and_history():
    m = _model()
    h = m.fit(_ds(), epochs=3, steps_per_epoch=8, verbose=0)
    assert m._trainer.kind == "generic"
    assert set(h.history) == {"loss", "sparse_categorical_accuracy"}
    assert h.history["loss"][-1] < h.history["loss"][0]
    res = m.evaluate(_ds(repeat=False), verbose=0, return_dict=True)
    assert set(res) == {"loss", "sparse_categorical_accuracy"}
    p = m.predict(np.random.rand(5, 28, 28, 1).astype(np.float32))
    assert p.shape == (5, 10)


def test_generic_step_matches_manual_sgd():
    m = _model(lr=0.1)
    x, y = synthetic_mnist(64, 3)
    x = torch.from_numpy(x.reshape(-1, 28, 28, 1)).float() / 255
    y = torch.from_numpy(y)
    w0 = [torch.tensor(w) for w in m.get_weights()]
    ps = [t.clone().double().requires_grad_(True) for t in w0]
    from tensorflow_distributed_learning_amd.models.mnist_cnn import reference_loss

    loss, _, _ = reference_loss(ps, x.double(), y)
    loss.backward()
    m.fit(tdl.data.Dataset.from_tensor_slices((x, y)).batch(64), epochs=1, verbose=0)
    for w, p in zip(m.get_weights(), ps):
        np.testing.assert_allclose(w, (p - 0.1 * p.grad).detach().numpy(), rtol=1e-4, atol=1e-6)


def test_numpy_inputs_validation_split_and_momentum():
    x, y = synthetic_mnist(256, 1)
    m = _model(momentum=0.9, nesterov=True)
    h = m.fit(x.reshape(-1, 28, 28, 1).astype(np.float32) / 255, y, batch_size=32, epochs=2, validation_split=0.25,
              verbose=0)
    assert "val_loss" in h.history and len(h.history["val_loss"]) == 2


def test_steps_per_epoch_exhaustion_warns():
    m = _model()
    with pytest.warns(UserWarning, match="ran out of data"):
        h = m.fit(_ds(n=128, repeat=False), epochs=3, steps_per_epoch=2, verbose=0)
    assert len(h.history["loss"]) == 2  # 4 batches total -> epoch 3 cannot run


def test_steps_per_execution_and_progbar(capsys):
    m = build_mnist_cnn()
    m.compile(loss=keras.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer="sgd",
              metrics=["accuracy"], steps_per_execution=3)
    m.fit(_ds(), epochs=2, steps_per_epoch=7, verbose=1)
    out = capsys.readouterr().out
    assert "Epoch 2/2" in out and "7/7 [" in out and "accuracy:" in out


def test_callbacks(tmp_path):
    seen = []
    m = _model()
    cbs = [keras.callbacks.ModelCheckpoint(str(tmp_path / "ck-{epoch}"), save_weights_only=True),
           keras.callbacks.CSVLogger(str(tmp_path / "log.csv")),
           keras.callbacks.TensorBoard(str(tmp_path / "tb")),
           keras.callbacks.LambdaCallback(on_batch_end=lambda b, logs: seen.append(logs["loss"])),
           keras.callbacks.LearningRateScheduler(lambda e: 0.05 * 0.5 ** e)]
    m.fit(_ds(), epochs=2, steps_per_epoch=3, verbose=0, callbacks=cbs)
    assert len(seen) == 6 and all(np.isfinite(seen))
    assert os.path.exists(str(tmp_path / "ck-2.index"))
    assert open(tmp_path / "log.csv").read().count("\n") == 3
    from tensorflow_distributed_learning_amd.utils.events import read_tfrecords

    ev = [f for f in os.listdir(tmp_path / "tb" / "train") if f.startswith("events.out.tfevents")]
    recs = list(read_tfrecords(str(tmp_path / "tb" / "train" / ev[0])))
    assert len(recs) >= 1 + 2 * 2 and b"epoch_loss" in b"".join(recs)
    assert m.optimizer.current_lr() == pytest.approx(0.025)


def test_early_stopping():
    m = _model(lr=0.0)
    cb = keras.callbacks.EarlyStopping(monitor="loss", patience=1, min_delta=1.0)
    h = m.fit(_ds(), epochs=10, steps_per_epoch=2, verbose=0, callbacks=[cb])
    assert len(h.history["loss"]) == 2


def test_save_load_model_and_weights(tmp_path):
    m = _model()
    m.fit(_ds(), epochs=1, steps_per_epoch=3, verbose=0)
    p = str(tmp_path / "sm")
    m.save(p)
    assert set(os.listdir(p)) >= {"saved_model.json", "variables", "assets"}
    assert sorted(os.listdir(os.path.join(p, "variables"))) == ["variables.data-00000-of-00001", "variables.index"]
    from tensorflow_distributed_learning_amd.ckpt import checkpoint as ck

    idx = dict(ck.list_variables(os.path.join(p, "variables", "variables")))  # TF tensor-bundle index
    assert idx["conv2d/kernel:0"] == (3, 3, 1, 32)
    m2 = keras.models.load_model(p)
    x = torch.rand(4, 28, 28, 1)
    assert torch.allclose(m(x), m2(x), atol=1e-6)
    assert m2.optimizer.iterations == m.optimizer.iterations
    m2.fit(_ds(), epochs=1, steps_per_epoch=2, verbose=0)  # recompiled and trainable
    m.save_weights(str(tmp_path / "w" / "ckpt"))
    keras.backend.clear_session()
    m3 = _model()
    m3.load_weights(str(tmp_path / "w" / "ckpt"))
    assert all(np.array_equal(a, b) for a, b in zip(m.get_weights(), m3.get_weights()))
    assert tdl.train.latest_checkpoint(str(tmp_path / "w")).endswith("ckpt")


def test_checkpoint_manager_and_corruption(tmp_path):
    m = _model()
    m.fit(_ds(), epochs=1, steps_per_epoch=2, verbose=0)
    ck = tdl.train.Checkpoint(model=m, optimizer=m.optimizer)
    mgr = tdl.train.CheckpointManager(ck, str(tmp_path), max_to_keep=2)
    paths = [mgr.save() for _ in range(3)]
    assert mgr.checkpoints == paths[1:] and mgr.latest_checkpoint == paths[-1]
    assert not os.path.exists(paths[0] + ".index")
    w = m.get_weights()
    m.set_weights([np.zeros_like(a) for a in w])
    ck.restore(mgr.latest_checkpoint)
    assert all(np.array_equal(a, b) for a, b in zip(w, m.get_weights()))
    data = bytearray(open(paths[-1] + ".data-00000-of-00001", "rb").read())
    data[100] ^= 0xFF
    open(paths[-1] + ".data-00000-of-00001", "wb").write(bytes(data))
    with pytest.raises(ValueError, match="checksum"):
        ck.restore(paths[-1])


def test_backup_and_restore_resumes(tmp_path):
    d = str(tmp_path / "backup")

    class Boom(keras.callbacks.Callback):
        def on_epoch_end(self, epoch, logs=None):
            if epoch == 1:
                raise RuntimeError("simulated worker failure")

    m = _model()
    with pytest.raises(RuntimeError):
        m.fit(_ds(), epochs=4, steps_per_epoch=2, verbose=0, callbacks=[keras.callbacks.BackupAndRestore(d), Boom()])
    it_after_fail = m.optimizer.iterations
    keras.backend.clear_session()
    m2 = _model()
    h = m2.fit(_ds(), epochs=4, steps_per_epoch=2, verbose=0, callbacks=[keras.callbacks.BackupAndRestore(d)])
    # epoch 1 was backed up (BackupAndRestore runs before Boom raises): resume at epoch 2
    assert len(h.history["loss"]) == 2
    assert m2.optimizer.iterations == 4 + 2 * 2
    assert it_after_fail == 4
    assert not os.path.exists(d)


def test_optimizers_match_torch():
    torch.manual_seed(0)
    w0 = torch.randn(1000)
    gs = [torch.randn(1000) for _ in range(5)]
    for ours, ref in [(keras.optimizers.SGD(0.1, momentum=0.9), lambda p: torch.optim.SGD(p, lr=0.1, momentum=0.9)),
                      (keras.optimizers.Adam(0.01, epsilon=1e-7), None),
                      (keras.optimizers.RMSprop(0.01), None), (keras.optimizers.Adagrad(0.1), None)]:
        W = w0.clone()
        for g in gs:
            ours.apply_flat(W, g.clone())
        assert torch.isfinite(W).all() and not torch.equal(W, w0)
        if ref is not None:
            p = torch.nn.Parameter(w0.clone())
            o = ref([p])
            for g in gs:
                p.grad = g.clone()
                o.step()
            assert torch.allclose(W, p.detach(), atol=1e-5)
    # Keras Adam closed form on step 1: w - lr * g/|g| (approximately)
    a = keras.optimizers.Adam(0.01)
    W = torch.zeros(3)
    a.apply_flat(W, torch.tensor([1.0, -2.0, 0.5]))
    assert torch.allclose(W, torch.tensor([-0.01, 0.01, -0.01]), atol=1e-5)
    s = keras.optimizers.schedules.ExponentialDecay(1.0, 10, 0.5)
    assert s(10) == pytest.approx(0.5)
    assert keras.optimizers.schedules.PiecewiseConstantDecay([5], [1.0, 0.1])(6) == 0.1


def test_bucket_hooks_survive_evaluate_and_predict():
    """evaluate()/predict() rebuild the autograd leaves; the bucketed all-reduce
    hooks must follow them, or the next eager step finds no launched buckets."""
    from tensorflow_distributed_learning_amd.parallel.communicator import LocalCommunicator, _Done

    class FakeRccl(LocalCommunicator):
        name = "rccl"

        def __init__(self):
            super().__init__(torch.device("cpu"))
            self.world_size = 2
            self.launched = 0

        def all_reduce_async(self, t, op="sum"):
            self.launched += 1
            return _Done()

    strategy = tdl.distribute.OneDeviceStrategy("/cpu:0")
    fake = FakeRccl()
    strategy.extended.communicator = fake
    with strategy.scope():
        m = build_mnist_cnn()
        m.compile(loss=keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=keras.optimizers.SGD(0.05), bucket_bytes=64 << 10)
    m.fit(_ds(), epochs=1, steps_per_epoch=2, verbose=0)
    nb = len(m._trainer._bucket_ranges)
    assert nb > 1 and fake.launched == 2 * nb
    m.evaluate(_ds(n=128, repeat=False), verbose=0)
    m.predict(np.random.rand(3, 28, 28, 1).astype(np.float32))
    m.fit(_ds(), epochs=1, steps_per_epoch=2, verbose=0)
    assert fake.launched == 4 * nb
