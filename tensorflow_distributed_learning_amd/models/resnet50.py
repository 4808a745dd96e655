"""ResNet-50 (Keras ``applications.ResNet50`` layout) – BASELINE configs 4/5.

Built with this framework's functional Keras API: ZeroPadding + 7x7/2 conv + BN + ReLU +
3x3/2 max-pool, then 3/4/6/3 bottleneck blocks (1x1 -> 3x3 -> 1x1, 4x expansion, projection
shortcut on the first block of each stage, stride on the first 1x1 as Keras v1 does), global
average pool, Dense(classes).  25,636,712 parameters including BatchNorm moving statistics
(25,583,592 trainable), matching tf.keras.applications.ResNet50(weights=None).
"""
from __future__ import annotations

from typing import Optional


def _block(x, filters, L, stride=1, conv_shortcut=True, name=""):
    bn_eps = 1.001e-5
    if conv_shortcut:
        sc = L.Conv2D(4 * filters, 1, strides=stride, name=name + "_0_conv")(x)
        sc = L.BatchNormalization(axis=3, epsilon=bn_eps, name=name + "_0_bn")(sc)
    else:
        sc = x
    x = L.Conv2D(filters, 1, strides=stride, name=name + "_1_conv")(x)
    x = L.BatchNormalization(axis=3, epsilon=bn_eps, name=name + "_1_bn")(x)
    x = L.Activation("relu", name=name + "_1_relu")(x)
    x = L.Conv2D(filters, 3, padding="same", name=name + "_2_conv")(x)
    x = L.BatchNormalization(axis=3, epsilon=bn_eps, name=name + "_2_bn")(x)
    x = L.Activation("relu", name=name + "_2_relu")(x)
    x = L.Conv2D(4 * filters, 1, name=name + "_3_conv")(x)
    x = L.BatchNormalization(axis=3, epsilon=bn_eps, name=name + "_3_bn")(x)
    x = L.Add(name=name + "_add")([sc, x])
    return L.Activation("relu", name=name + "_out")(x)


def _stack(x, filters, blocks, L, stride1=2, name=""):
    x = _block(x, filters, L, stride=stride1, name=name + "_block1")
    for i in range(2, blocks + 1):
        x = _block(x, filters, L, conv_shortcut=False, name=name + "_block" + str(i))
    return x


def ResNet50(include_top: bool = True, weights=None, input_tensor=None, input_shape=None, pooling=None,  # noqa: N802
             classes: int = 1000, classifier_activation: Optional[str] = "softmax", keras_module=None, **kw):
    if weights not in (None, "none"):
        raise ValueError("pretrained weights are not available offline; use weights=None")
    if keras_module is None:
        from .. import keras as keras_module
    L = keras_module.layers
    inp = input_tensor if input_tensor is not None else L.Input(shape=input_shape or (224, 224, 3), name="input_1")
    x = L.ZeroPadding2D(padding=((3, 3), (3, 3)), name="conv1_pad")(inp)
    x = L.Conv2D(64, 7, strides=2, name="conv1_conv")(x)
    x = L.BatchNormalization(axis=3, epsilon=1.001e-5, name="conv1_bn")(x)
    x = L.Activation("relu", name="conv1_relu")(x)
    x = L.ZeroPadding2D(padding=((1, 1), (1, 1)), name="pool1_pad")(x)
    x = L.MaxPooling2D(3, strides=2, name="pool1_pool")(x)
    x = _stack(x, 64, 3, L, stride1=1, name="conv2")
    x = _stack(x, 128, 4, L, name="conv3")
    x = _stack(x, 256, 6, L, name="conv4")
    x = _stack(x, 512, 3, L, name="conv5")
    if include_top:
        x = L.GlobalAveragePooling2D(name="avg_pool")(x)
        x = L.Dense(classes, activation=classifier_activation, name="predictions")(x)
    elif pooling == "avg":
        x = L.GlobalAveragePooling2D(name="avg_pool")(x)
    elif pooling == "max":
        x = L.GlobalMaxPooling2D(name="max_pool")(x)
    return keras_module.Model(inp, x, name="resnet50")
