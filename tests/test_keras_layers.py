"""Keras layers: TF layouts/semantics vs plain PyTorch references."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import tensorflow_distributed_learning_amd as tdl
from tensorflow_distributed_learning_amd.keras import layers as L
from tensorflow_distributed_learning_amd.models import mnist_cnn as M

keras = tdl.keras


@pytest.fixture(autouse=True)
def _fresh():
    keras.backend.clear_session()


def test_reference_model_names_shapes_params():
    m = M.build_mnist_cnn()
    assert m.count_params() == M.MNIST_NUM_PARAMS
    assert [(w.name, w.shape) for w in m.weights] == [(n, s) for n, s in M.MNIST_CNN_VARIABLES]
    x = torch.rand(3, 28, 28, 1)
    ref = M.reference_logits([w.read_value() for w in m.weights], x)
    assert torch.allclose(m(x), ref, atol=1e-6)
    lines = []
    m.summary(print_fn=lines.append)
    assert any("225,034" in l for l in lines)


def test_glorot_uniform_bounds():
    keras.utils.set_random_seed(0)
    m = M.build_mnist_cnn()
    k = m.weights[4].numpy()  # dense/kernel [1600,128]
    lim = math.sqrt(6 / (1600 + 128))
    assert k.max() <= lim and k.min() >= -lim and k.std() > lim / 3
    assert np.all(m.weights[1].numpy() == 0)


@pytest.mark.parametrize("stride,pad", [(1, "valid"), (2, "same"), (1, "same"), (2, "valid")])
def test_conv2d_tf_padding(stride, pad):
    c = L.Conv2D(5, 3, strides=stride, padding=pad)
    x = torch.randn(2, 9, 10, 3)
    y = c(x)
    # reference: explicit TF 'same' padding (extra pad at the end) then valid conv
    h = x.permute(0, 3, 1, 2)
    if pad == "same":
        def pads(n):
            out = -(-n // stride)
            tot = max((out - 1) * stride + 3 - n, 0)
            return tot // 2, tot - tot // 2
        ph, pw = pads(9), pads(10)
        h = F.pad(h, (pw[0], pw[1], ph[0], ph[1]))
    ref = F.conv2d(h, c.kernel.value.permute(3, 2, 0, 1), c.bias.value, stride=stride).permute(0, 2, 3, 1)
    assert y.shape == ref.shape and torch.allclose(y, ref, atol=1e-5)
    assert c.compute_output_shape((None, 9, 10, 3)) == (None,) + tuple(y.shape[1:])


def test_pooling_and_flatten_order():
    x = torch.randn(2, 5, 5, 3)
    assert L.MaxPooling2D()(x).shape == (2, 2, 2, 3)
    assert L.MaxPooling2D(3, strides=2, padding="same")(x).shape == (2, 3, 3, 3)
    ap = L.AveragePooling2D(2, padding="same")(x)
    assert torch.allclose(ap[:, 2, 2], x[:, 4, 4])  # edge window averages only valid elements
    f = L.Flatten()(x)
    assert torch.equal(f[0, :3], x[0, 0, 0])  # HWC order
    assert L.GlobalAveragePooling2D()(x).shape == (2, 3)


def test_batchnorm_train_and_moving_stats():
    bn = L.BatchNormalization(momentum=0.9, epsilon=1e-3)
    x = torch.randn(64, 4, 4, 3) * 2 + 1
    y = bn(x, training=True)
    assert torch.allclose(y.mean(dim=(0, 1, 2)), torch.zeros(3), atol=1e-5)
    mm = bn.moving_mean.numpy()
    assert np.allclose(mm, 0.1 * x.mean(dim=(0, 1, 2)).numpy(), atol=1e-5)
    y2 = bn(x, training=False)
    assert y2.shape == x.shape


def test_functional_model_and_config_roundtrip():
    inp = keras.Input(shape=(8,))
    a = L.Dense(4, activation="relu")(inp)
    b = L.Dense(4)(inp)
    out = L.Dense(2)(L.Add()([a, b]))
    m = keras.Model(inp, out)
    x = torch.randn(5, 8)
    y = m(x)
    assert y.shape == (5, 2)
    m2 = keras.models.model_from_config(m.get_config_full())
    m2.set_weights(m.get_weights())
    assert torch.allclose(m2(x), y, atol=1e-6)


def test_sequential_config_roundtrip():
    m = M.build_mnist_cnn()
    m2 = keras.models.model_from_config(m.get_config_full())
    m2.set_weights(m.get_weights())
    x = torch.rand(2, 28, 28, 1)
    assert torch.allclose(m(x), m2(x), atol=1e-6)


def test_resnet50_param_count():
    m = keras.applications.ResNet50(weights=None, input_shape=(64, 64, 3), classes=1000)
    assert m.count_params() == 25_636_712
    assert sum(int(np.prod(w.shape)) for w in m.trainable_weights) == 25_583_592
    y = m(torch.randn(2, 64, 64, 3))
    assert y.shape == (2, 1000) and torch.allclose(y.sum(1), torch.ones(2), atol=1e-4)


def test_misc_layers():
    x = torch.randn(2, 3, 4)
    assert L.Reshape((12,))(x).shape == (2, 12)
    assert L.Reshape((-1, 2))(x).shape == (2, 6, 2)
    assert L.Concatenate()([x, x]).shape == (2, 3, 8)
    assert L.Dropout(0.5)(x, training=False).equal(x)
    assert L.ZeroPadding2D(1)(torch.zeros(1, 2, 2, 1)).shape == (1, 4, 4, 1)
    assert L.Embedding(10, 3)(torch.tensor([[1, 2]])).shape == (1, 2, 3)
    assert L.LayerNormalization()(x).shape == x.shape
    assert L.Activation("softmax")(x).sum(-1).allclose(torch.ones(2, 3))
