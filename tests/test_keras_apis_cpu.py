"""Offline Keras / tfds API surface around the reference script: tf.keras.applications.resnet50
preprocessing helpers ('caffe' mode), tf.keras.datasets.mnist.load_data (npz file, else IDX / synthetic),
tfds.as_numpy / builder / list_builders."""
import json

import numpy as np
import torch

import tensorflow_distributed_learning_amd as tdl
from tensorflow_distributed_learning_amd.compat import tfds


def test_resnet50_preprocess_input_caffe_mode():
    app = tdl.keras.applications.resnet50
    x = np.arange(2 * 3 * 3 * 3, dtype=np.uint8).reshape(2, 3, 3, 3)
    y = app.preprocess_input(x)
    assert y.dtype == np.float32 and y.shape == x.shape
    ref = x[..., ::-1].astype(np.float32) - np.array([103.939, 116.779, 123.68], np.float32)
    np.testing.assert_allclose(y, ref, rtol=0, atol=1e-5)
    t = app.preprocess_input(torch.from_numpy(x).permute(0, 3, 1, 2), data_format="channels_first")
    np.testing.assert_allclose(t.permute(0, 2, 3, 1).numpy(), ref, atol=1e-5)


def test_resnet50_decode_predictions(tmp_path, monkeypatch):
    app = tdl.keras.applications
    preds = np.array([[0.1, 0.7, 0.2], [0.5, 0.25, 0.25]], np.float32)
    monkeypatch.setenv("KERAS_HOME", str(tmp_path))
    monkeypatch.setattr(app, "_CLASS_INDEX", None)
    out = app.resnet50.decode_predictions(preds, top=2)
    assert out[0] == [("1", "class_1", np.float32(0.7)), ("2", "class_2", np.float32(0.2))]
    assert [c[0] for c in out[1]] == ["0", "1"]  # ties: lower index first
    (tmp_path / "models").mkdir()
    (tmp_path / "models" / "imagenet_class_index.json").write_text(
        json.dumps({"0": ["n0", "zero"], "1": ["n1", "one"], "2": ["n2", "two"]}))
    monkeypatch.setattr(app, "_CLASS_INDEX", None)
    out = app.resnet50.decode_predictions(torch.from_numpy(preds), top=1)
    assert out == [[("n1", "one", np.float32(0.7))], [("n0", "zero", np.float32(0.5))]]


def test_mnist_load_data_npz_then_fallback(tmp_path, monkeypatch):
    monkeypatch.setenv("KERAS_HOME", str(tmp_path))
    (xtr, ytr), (xte, yte) = tdl.keras.datasets.mnist.load_data()
    assert xtr.shape == (60000, 28, 28) and xtr.dtype == np.uint8 and ytr.dtype == np.uint8
    assert xte.shape == (10000, 28, 28) and ytr.max() <= 9
    (tmp_path / "datasets").mkdir()
    g = np.random.default_rng(0)
    arrs = dict(x_train=g.integers(0, 255, (5, 28, 28), dtype=np.uint8), y_train=np.arange(5, dtype=np.uint8),
                x_test=g.integers(0, 255, (2, 28, 28), dtype=np.uint8), y_test=np.arange(2, dtype=np.uint8))
    np.savez(tmp_path / "datasets" / "mnist.npz", **arrs)
    (a, b), (c, d) = tdl.keras.datasets.mnist.load_data()
    assert np.array_equal(a, arrs["x_train"]) and np.array_equal(b, arrs["y_train"])
    assert np.array_equal(c, arrs["x_test"]) and np.array_equal(d, arrs["y_test"])


def test_tfds_as_numpy_builder_list():
    assert tfds.list_builders() == ["mnist"]
    b = tfds.builder("mnist")
    assert b.info.splits["train"].num_examples == 60000
    ds = b.as_dataset(split="test", as_supervised=True).take(3).batch(3)
    (x, y), = list(tfds.as_numpy(ds))
    assert isinstance(x, np.ndarray) and x.shape == (3, 28, 28, 1) and y.shape == (3,)
    both = tfds.as_numpy({"a": ds})
    assert set(both) == {"a"}
    try:
        tfds.builder("cifar10")
    except ValueError as e:
        assert "mnist" in str(e)
    else:
        raise AssertionError("unknown builder accepted")
