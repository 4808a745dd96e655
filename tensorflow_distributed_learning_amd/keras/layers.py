"""Keras layers (tf_dist_example.py:40-48 and what ResNet-50 needs), NHWC / TF weight layouts.

Layers hold *specs* (variables with TF names and layouts: Conv2D kernels HWIO, Dense kernels
[in, out], Flatten in HWC order) and a plain-PyTorch ``call`` used by the generic training path
and for inference.  On MI355X the reference's layer stack is not executed layer by layer at all:
the engine compiles it into the fused HIP train step (engine/fused.py).

Functional API: calling a layer on a :class:`KerasTensor` (from :func:`Input`) records a graph node
instead of computing; ``keras.Model(inputs, outputs)`` executes that graph.
"""
from __future__ import annotations

import math
import re
from collections import defaultdict
from typing import Any, Dict, List, Optional, Sequence, Tuple, Union

import torch
import torch.nn.functional as F

from ..parallel.values import Variable, VariableAggregation, VariableSynchronization, create_variable
from ..ops import conv as _conv
from ..ops import conv_f32 as _conv_f32
from ..ops import dense as _dense
from . import activations as _act
from . import initializers as _init

_UIDS: Dict[str, int] = defaultdict(int)


def _snake(name: str) -> str:
    s = re.sub(r"(.)([A-Z][a-z]+)", r"\1_\2", name)
    s = re.sub(r"([a-z0-9])([A-Z])", r"\1_\2", s).lower()
    return s.replace("2_d", "2d").replace("1_d", "1d").replace("3_d", "3d")


def unique_name(prefix: str) -> str:
    n = _UIDS[prefix]
    _UIDS[prefix] += 1
    return prefix if n == 0 else f"{prefix}_{n}"


def reset_uids():
    _UIDS.clear()


def _pair(v) -> Tuple[int, int]:
    if isinstance(v, int):
        return (v, v)
    v = tuple(v)
    return (int(v[0]), int(v[1]))


# ------------------------------------------------------------------------------------------------
class KerasTensor:
    """Symbolic tensor of the functional API (shape includes the batch dim as None)."""

    def __init__(self, shape, dtype=torch.float32, node=None, index=0, name=None):
        self.shape = tuple(shape)
        self.dtype = dtype
        self._node = node
        self._index = index
        self.name = name

    def __repr__(self):
        return f"<KerasTensor shape={self.shape}>"


class Node:
    def __init__(self, layer, inputs, kwargs):
        self.layer = layer
        self.inputs = inputs  # structure of KerasTensors
        self.kwargs = kwargs
        self.outputs = None


def _flat(x) -> List[Any]:
    if isinstance(x, (list, tuple)):
        out = []
        for v in x:
            out += _flat(v)
        return out
    return [x]


def _map(fn, x):
    if isinstance(x, (list, tuple)):
        return type(x)(_map(fn, v) for v in x)
    return fn(x)


class Layer:
    """Base layer (tf.keras.layers.Layer)."""

    def __init__(self, name: Optional[str] = None, trainable: bool = True, dtype=None, input_shape=None,
                 batch_input_shape=None, input_dim=None, **kwargs):
        self.name = name or unique_name(_snake(type(self).__name__))
        self.trainable = trainable
        self.dtype = dtype or torch.float32
        self.built = False
        self._weights: List[Variable] = []
        self._layers: List["Layer"] = []
        if input_dim is not None and input_shape is None:
            input_shape = (input_dim,)
        self._batch_input_shape = (tuple(batch_input_shape) if batch_input_shape is not None else
                                   ((None,) + tuple(input_shape) if input_shape is not None else None))
        self._inbound_nodes: List[Node] = []
        self.input_spec = None
        unknown = set(kwargs) - {"autocast", "dynamic", "weights", "activity_regularizer"}
        if unknown:
            raise TypeError(f"{type(self).__name__}: unexpected keyword arguments {sorted(unknown)}")

    # ------------------------------------------------------------------ weights
    def add_weight(self, name: str, shape, dtype=None, initializer="glorot_uniform", trainable: bool = True,
                   regularizer=None, constraint=None, synchronization=VariableSynchronization.AUTO,
                   aggregation=VariableAggregation.NONE):
        init = _init.get(initializer)
        dtype = dtype or torch.float32
        v = create_variable(lambda: init(tuple(shape), dtype), name=f"{self.name}/{name}", trainable=trainable,
                            synchronization=synchronization, aggregation=aggregation, dtype=dtype)
        v._regularizer = regularizer
        self._weights.append(v)
        return v

    @property
    def weights(self) -> List[Variable]:
        out = list(self._weights)
        for l in self._layers:
            out += l.weights
        return out

    variables = weights

    @property
    def trainable_weights(self) -> List[Variable]:
        if not self.trainable:
            return []
        return [w for w in self.weights if w.trainable]

    trainable_variables = trainable_weights

    @property
    def non_trainable_weights(self) -> List[Variable]:
        if not self.trainable:
            return self.weights
        return [w for w in self.weights if not w.trainable]

    non_trainable_variables = non_trainable_weights

    def get_weights(self):
        return [w.numpy() for w in self.weights]

    def set_weights(self, weights):
        ws = self.weights
        if len(weights) != len(ws):
            raise ValueError(f"{self.name}: expected {len(ws)} weight arrays, got {len(weights)}")
        for v, a in zip(ws, weights):
            if tuple(v.shape) != tuple(getattr(a, "shape", ())):
                raise ValueError(f"{v.name}: shape {tuple(getattr(a, 'shape', ()))} != {v.shape}")
            v.assign(a)

    def count_params(self) -> int:
        return int(sum(math.prod(w.shape) for w in self.weights))

    # ------------------------------------------------------------------ build / call
    def build(self, input_shape):
        self.built = True

    def _maybe_build(self, input_shape):
        if not self.built:
            self.build(input_shape)
            self.built = True

    def call(self, inputs, training=None):
        return inputs

    def compute_output_shape(self, input_shape):
        """Default: run call on a tiny dummy batch (batch 1) to infer the shape."""
        def dummy(s):
            return torch.zeros((1,) + tuple(d if d is not None else 1 for d in s[1:]))

        with torch.no_grad():
            x = _map(dummy, input_shape) if isinstance(input_shape, list) else dummy(input_shape)
            y = self.call(x, training=False)
        return _map(lambda t: (None,) + tuple(t.shape[1:]), y)

    def __call__(self, inputs, training=None, **kwargs):
        flat = _flat(inputs)
        if any(isinstance(t, KerasTensor) for t in flat):
            shapes = _map(lambda t: t.shape, inputs)
            self._maybe_build(shapes)
            node = Node(self, inputs, dict(kwargs, training=training) if training is not None else kwargs)
            out_shape = self.compute_output_shape(shapes)
            if isinstance(out_shape, list) and out_shape and isinstance(out_shape[0], tuple):
                outs = [KerasTensor(s, node=node, index=i) for i, s in enumerate(out_shape)]
            else:
                outs = KerasTensor(out_shape, node=node, index=0)
            node.outputs = outs
            self._inbound_nodes.append(node)
            return outs
        shapes = _map(lambda t: tuple(t.shape), inputs)
        self._maybe_build(shapes)
        if kwargs:
            return self.call(inputs, training=training, **kwargs)
        return self.call(inputs, training=training)

    def get_config(self) -> Dict[str, Any]:
        cfg = {"name": self.name, "trainable": self.trainable}
        if self._batch_input_shape is not None:
            cfg["batch_input_shape"] = list(self._batch_input_shape)
        return cfg

    @classmethod
    def from_config(cls, config):
        return cls(**config)

    def __repr__(self):
        return f"<{type(self).__name__} name={self.name}>"


class InputLayer(Layer):
    def __init__(self, input_shape=None, batch_size=None, dtype=None, name=None, **kw):
        super().__init__(name=name or unique_name("input"), dtype=dtype,
                         batch_input_shape=(batch_size,) + tuple(input_shape) if input_shape is not None else None, **kw)


def Input(shape=None, batch_size=None, name=None, dtype=None, **kwargs) -> KerasTensor:  # noqa: N802
    layer = InputLayer(input_shape=shape, batch_size=batch_size, name=name, dtype=dtype)
    node = Node(layer, None, {})
    t = KerasTensor((batch_size,) + tuple(shape), dtype=dtype or torch.float32, node=node, name=layer.name)
    node.outputs = t
    return t


# ------------------------------------------------------------------------------------------------
class Dense(Layer):
    def __init__(self, units, activation=None, use_bias=True, kernel_initializer="glorot_uniform",
                 bias_initializer="zeros", kernel_regularizer=None, bias_regularizer=None,
                 activity_regularizer=None, kernel_constraint=None, bias_constraint=None, **kw):
        super().__init__(**kw)
        self.units = int(units)
        self.activation = _act.get(activation)
        self.use_bias = use_bias
        self.kernel_initializer = _init.get(kernel_initializer)
        self.bias_initializer = _init.get(bias_initializer)
        self.kernel_regularizer = kernel_regularizer
        self.bias_regularizer = bias_regularizer

    def build(self, input_shape):
        d = int(input_shape[-1])
        self.kernel = self.add_weight("kernel", (d, self.units), initializer=self.kernel_initializer,
                                      regularizer=self.kernel_regularizer)
        self.bias = self.add_weight("bias", (self.units,), initializer=self.bias_initializer,
                                    regularizer=self.bias_regularizer) if self.use_bias else None
        self.built = True

    def call(self, x, training=None):
        x = _autocast_input(x)
        if _dense.dense_supported(x, self.units):
            # bf16 on the GPU: hand-written MFMA GEMMs (ops/dense.py), gradients straight into the
            # trainer's slab when it is bound
            gw = self.kernel.grad_target()
            gb = self.bias.grad_target() if self.bias is not None else None
            if gw is not None and (self.bias is None or gb is not None):
                w = self.kernel.compute_view(x.dtype)
                w = w if w is not None else self.kernel.value.detach().to(x.dtype)
                b = self.bias.value.detach() if self.bias is not None else None
                return self.activation(_dense.dense_bf16(x, w, b, (gw, gb), anchor=self.kernel.value))
            b = self.bias.value if self.bias is not None else None
            return self.activation(_dense.dense_bf16(x, self.kernel.cast(x.dtype), b))
        low = x.is_cuda and x.dtype == torch.bfloat16 and self.kernel.value.dtype == torch.float32
        if (_conv_f32.dense_supported(x) or low) and self.kernel.value.dtype == torch.float32:
            # f32 on the GPU: the f32-MFMA GEMM of csrc/kernels/gemm_f32.hip (no hipBLASLt); also a bf16
            # input whose shape the bf16 GEMM does not tile (a 10-class head under mixed_bfloat16):
            # f32 math on the f32 master weights, bf16 out (the layer's compute dtype)
            xf = x.float() if low else x
            gw = self.kernel.grad_target()
            gb = self.bias.grad_target() if self.bias is not None else None
            act = _fused_act(self.activation)  # ReLU inside the GEMMs (forward epilogue, backward masks)
            if gw is not None and gw.is_contiguous() and (self.bias is None or gb is not None):
                b = self.bias.value.detach() if self.bias is not None else None
                y = _conv_f32.dense(xf, self.kernel.value.detach(), b, (gw, gb), anchor=self.kernel.value, act=act)
            else:
                b = self.bias.value if self.bias is not None else None
                y = _conv_f32.dense(xf, self.kernel.value, b, act=act)
            y = y.to(torch.bfloat16) if low else y
            return y if act else self.activation(y)
        y = torch.matmul(x, self.kernel.cast(x.dtype))
        if self.bias is not None:
            y = y + self.bias.value.to(y.dtype)
        return self.activation(y)

    def compute_output_shape(self, s):
        return tuple(s[:-1]) + (self.units,)

    def get_config(self):
        return dict(super().get_config(), units=self.units, activation=_act.serialize(self.activation),
                    use_bias=self.use_bias, kernel_initializer=_init.serialize(self.kernel_initializer),
                    bias_initializer=_init.serialize(self.bias_initializer))


def _fused_act(fn) -> int:
    """1 when the layer's activation is the plain ReLU the f32 GEMM kernels fuse (gemm_f32.hip), else 0."""
    import os

    return 1 if fn is _act.relu and os.environ.get("TDL_FUSE_ACT", "1") == "1" else 0


def _autocast_input(x):
    """Keras mixed precision: a layer casts its floating-point inputs to its compute dtype.  Under
    the ``mixed_bfloat16`` policy (bf16 autocast on the GPU) an f32 batch straight from the input
    pipeline therefore reaches the first Conv2D as bf16 and runs on the hand-written kernels.
    Without this cast it went to MIOpen under autocast, whose find-mode solver choice depends on
    timing: the first layer's output -- and, amplified over BN steps, the whole training run --
    then differed between runs and between asynchronous and HIP_LAUNCH_BLOCKING=1 execution
    (scripts/diag_checksums.py, profiles/generic_determinism_r4.txt)."""
    if (isinstance(x, torch.Tensor) and x.is_cuda and x.dtype == torch.float32 and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        return x.to(torch.bfloat16)
    return x


def _same_pads(in_size, k, s, d=1):
    out = -(-in_size // s)
    total = max((out - 1) * s + (k - 1) * d + 1 - in_size, 0)
    return total // 2, total - total // 2


class Conv2D(Layer):
    """2-D convolution, channels_last (NHWC), kernel HWIO, TF 'same'/'valid' padding."""

    def __init__(self, filters, kernel_size, strides=(1, 1), padding="valid", data_format=None, dilation_rate=(1, 1),
                 groups=1, activation=None, use_bias=True, kernel_initializer="glorot_uniform",
                 bias_initializer="zeros", kernel_regularizer=None, bias_regularizer=None,
                 activity_regularizer=None, kernel_constraint=None, bias_constraint=None, **kw):
        super().__init__(**kw)
        if data_format not in (None, "channels_last"):
            raise ValueError("only channels_last (NHWC) is supported – the TF default")
        self.filters = int(filters)
        self.kernel_size = _pair(kernel_size)
        self.strides = _pair(strides)
        self.padding = padding.lower()
        if self.padding not in ("valid", "same"):
            raise ValueError(f"padding must be 'valid' or 'same', got {padding!r}")
        self.dilation_rate = _pair(dilation_rate)
        self.groups = int(groups)
        self.activation = _act.get(activation)
        self.use_bias = use_bias
        self.kernel_initializer = _init.get(kernel_initializer)
        self.bias_initializer = _init.get(bias_initializer)
        self.kernel_regularizer = kernel_regularizer
        self.bias_regularizer = bias_regularizer

    def build(self, input_shape):
        cin = int(input_shape[-1])
        if cin % self.groups:
            raise ValueError("input channels must be divisible by groups")
        kh, kw = self.kernel_size
        self.kernel = self.add_weight("kernel", (kh, kw, cin // self.groups, self.filters),
                                      initializer=self.kernel_initializer, regularizer=self.kernel_regularizer)
        self.bias = self.add_weight("bias", (self.filters,), initializer=self.bias_initializer,
                                    regularizer=self.bias_regularizer) if self.use_bias else None
        self.built = True

    def call(self, x, training=None, _pool=None, **kw):
        """``_pool``: the 2x2 / stride-2 'valid' MaxPooling2D layer that follows this conv in a Sequential
        model (models.Sequential.call): on the generic f32 path the pool runs in the convolution's own
        launch (ops/conv_f32.conv2d_pool); elsewhere it is simply applied after the conv."""
        if _pool is None:
            return self._conv_call(x, training=training, **kw)
        out = self._conv_call(x, training=training, _pool_try=True, **kw)
        if isinstance(out, _Pooled):
            return out.t
        return _pool(out, training=training)

    def _conv_call(self, x, training=None, _fold_bias=False, _grad_box=None, _bn_stats=False, _zero_pad=None,
                   _pool_try=False):
        """``_fold_bias``: the functional executor folded this bias into the following training-mode
        BatchNormalization (keras/fusion.py), so the convolution runs without it.  ``_grad_box``:
        the input's other consumer's gradient is summed into this conv's input gradient.
        ``_zero_pad``: ((top, bottom), (left, right)) of a ZeroPadding2D folded in front (a <= 4-channel
        stride-2 'valid' conv: the ResNet stem, csrc/kernels/stem.hip)."""
        if _zero_pad is not None:
            (pt, pb), (pl, pr) = _zero_pad
            if self.padding == "valid" and _conv.stem_supported(x, self.kernel.value, self.strides, self.groups,
                                                                self.dilation_rate):
                gt = self.kernel.grad_target()
                k_hwio = (self.kernel.compute_view(torch.bfloat16) if gt is not None else None)
                if k_hwio is None:
                    k_hwio = self.kernel.value.detach().to(torch.bfloat16) if gt is not None else \
                        self.kernel.cast(torch.bfloat16)
                y = _conv.stem_conv2d_nhwc(x, k_hwio, (pt, pb, pl, pr), self.strides, grad_out=gt, bn_stats=_bn_stats,
                                           anchor=self.kernel.value if gt is not None else None)
                if self.bias is not None and not _fold_bias:
                    y = y + self.bias.value.to(y.dtype)
                return self.activation(y)
            x = F.pad(x, (0, 0, pl, pr, pt, pb))
        x = _autocast_input(x)
        gt = None
        if _conv.supported(x, self.kernel.value, self.groups, self.dilation_rate):
            gt = self.kernel.grad_target()
        # with a slab target the weight gradient kernel adds dW straight into the f32 slab view
        if gt is not None:
            k_hwio = self.kernel.compute_view(x.dtype)
            if k_hwio is None:
                k_hwio = self.kernel.value.detach().to(x.dtype)
        else:
            k_hwio = self.kernel.cast(x.dtype)
        w = k_hwio.permute(3, 2, 0, 1)  # HWIO -> OIHW
        h = x.permute(0, 3, 1, 2)  # NHWC data viewed as NCHW (channels_last memory format)
        pad = 0
        symmetric = True
        if self.padding == "same":
            ph = _same_pads(h.shape[2], self.kernel_size[0], self.strides[0], self.dilation_rate[0])
            pw = _same_pads(h.shape[3], self.kernel_size[1], self.strides[1], self.dilation_rate[1])
            if ph[0] == ph[1] and pw[0] == pw[1]:
                pad = (ph[0], pw[0])
            else:
                symmetric = False
                h = F.pad(h, (pw[0], pw[1], ph[0], ph[1]))
        b = self.bias.value.to(x.dtype) if (self.bias is not None and not _fold_bias) else None
        if gt is not None and not symmetric:  # (asymmetric "same" padding: undo the detached fast path)
            gt, k_hwio = None, self.kernel.cast(x.dtype)
            w = k_hwio.permute(3, 2, 0, 1)
        if symmetric and _conv.supported(x, k_hwio, self.groups, self.dilation_rate):
            # hand-written implicit-GEMM MFMA kernels (csrc/kernels/conv.hip), autotuned against MIOpen
            y = _conv.conv2d_nhwc(x, k_hwio, self.strides, pad if pad else (0, 0), grad_out=gt,
                                  w_ohwi=self.kernel.compute_view_ohwi(x.dtype) if gt is not None else None,
                                  grad_box=_grad_box, bn_stats=_bn_stats, bn_src=getattr(x, "_tdl_bn_src", None),
                                  bn_src2=getattr(x, "_tdl_bn_src2", None),
                                  bn_stats_src=getattr(x, "_tdl_bn_stats", None),
                                  anchor=self.kernel.value if gt is not None else None,
                                  bn_in=getattr(x, "_tdl_bn_in", None))
            if b is not None:
                y = y + b
            return self.activation(y)
        if getattr(x, "_tdl_bn_in", None) is not None:  # (keras/fusion.py plans it only where the kernels run)
            raise RuntimeError("Conv2D: a deferred BN -> ReLU input needs the hand-written 1x1 kernels")
        if _conv_f32.supported(x, self.groups) and _conv.mode() != "miopen":
            # every other conv -- f32 layers, asymmetric 'same' padding, dilation, channel counts the bf16
            # kernels do not tile: the generic f32-MFMA implicit GEMM (ops/conv_f32.py)
            pads = (0, 0, 0, 0)
            if self.padding == "same":
                ph = _same_pads(x.shape[1], self.kernel_size[0], self.strides[0], self.dilation_rate[0])
                pw = _same_pads(x.shape[2], self.kernel_size[1], self.strides[1], self.dilation_rate[1])
                pads = (ph[0], ph[1], pw[0], pw[1])
            gt = self.kernel.grad_target()
            gb = None
            if gt is not None and gt.is_contiguous():
                wv, anchor = self.kernel.value.detach(), self.kernel.value
                if b is not None:
                    gb = self.bias.grad_target()
                    if gb is not None:  # the bias gradient from the weight-gradient kernel, into the slab
                        b = self.bias.value.detach().to(x.dtype)
            else:
                gt, wv, anchor = None, self.kernel.cast(x.dtype), None
            act = _fused_act(self.activation)  # ReLU inside the GEMMs (forward epilogue, backward masks)
            if _pool_try and act == 1:
                oh = _conv_f32.out_size(x.shape[1], self.kernel_size[0], self.strides[0], self.dilation_rate[0],
                                        pads[0], pads[1])
                ow = _conv_f32.out_size(x.shape[2], self.kernel_size[1], self.strides[1], self.dilation_rate[1],
                                        pads[2], pads[3])
                if _conv_f32.conv_pool_supported(x, oh, ow, self.filters):
                    return _Pooled(_conv_f32.conv2d_pool(x, wv, b, self.strides, pads, self.dilation_rate, grad_out=gt,
                                                         anchor=anchor, act=act, gb_out=gb))
            y = _conv_f32.conv2d(x, wv, b, self.strides, pads, self.dilation_rate, grad_out=gt, anchor=anchor, act=act,
                                 gb_out=gb)
            return y if act else self.activation(y)
        if x.is_cuda:  # no hand-written kernel covers this conv: library path, counted (ops/conv.py)
            _conv._lib("conv2d", f"{str(x.dtype).replace('torch.', '')} C={x.shape[-1]} K={w.shape[0]} "
                       f"{self.kernel_size[0]}x{self.kernel_size[1]}/{self.strides[0]} {self.padding}")
        y = F.conv2d(h, w, b, stride=self.strides, padding=pad, dilation=self.dilation_rate, groups=self.groups)
        return self.activation(y.permute(0, 2, 3, 1))

    def compute_output_shape(self, s):
        n, h, w, _ = s

        def o(i, k, st, d):
            if i is None:
                return None
            if self.padding == "same":
                return -(-i // st)
            return (i - (k - 1) * d - 1) // st + 1

        return (n, o(h, self.kernel_size[0], self.strides[0], self.dilation_rate[0]),
                o(w, self.kernel_size[1], self.strides[1], self.dilation_rate[1]), self.filters)

    def get_config(self):
        return dict(super().get_config(), filters=self.filters, kernel_size=list(self.kernel_size),
                    strides=list(self.strides), padding=self.padding, dilation_rate=list(self.dilation_rate),
                    groups=self.groups, activation=_act.serialize(self.activation), use_bias=self.use_bias,
                    kernel_initializer=_init.serialize(self.kernel_initializer),
                    bias_initializer=_init.serialize(self.bias_initializer))


class _Pooled:
    """Conv2D._conv_call's result when the following max pool already ran in the conv's launch."""

    __slots__ = ("t",)

    def __init__(self, t):
        self.t = t


def conv_pool_pair(conv, pool) -> bool:
    """``Conv2D -> MaxPooling2D(2, 2, 'valid')``: the pair the generic engine can run as one forward launch
    (TDL_FUSE_CONV_POOL=0 keeps them apart)."""
    import os

    return (type(conv) is Conv2D and type(pool) is MaxPooling2D and pool.pool_size == (2, 2)
            and pool.strides == (2, 2) and pool.padding == "valid"
            and os.environ.get("TDL_FUSE_CONV_POOL", "1") == "1")


class _Pool2D(Layer):
    def __init__(self, pool_size=(2, 2), strides=None, padding="valid", data_format=None, **kw):
        super().__init__(**kw)
        self.pool_size = _pair(pool_size)
        self.strides = _pair(strides) if strides is not None else self.pool_size
        self.padding = padding.lower()

    def compute_output_shape(self, s):
        n, h, w, c = s

        def o(i, k, st):
            if i is None:
                return None
            return -(-i // st) if self.padding == "same" else (i - k) // st + 1

        return (n, o(h, self.pool_size[0], self.strides[0]), o(w, self.pool_size[1], self.strides[1]), c)

    def _pads(self, h):
        ph = _same_pads(h.shape[2], self.pool_size[0], self.strides[0])
        pw = _same_pads(h.shape[3], self.pool_size[1], self.strides[1])
        return ph, pw

    def get_config(self):
        return dict(super().get_config(), pool_size=list(self.pool_size), strides=list(self.strides),
                    padding=self.padding)


class MaxPooling2D(_Pool2D):
    def call(self, x, training=None, _zero_pad=None):
        """``_zero_pad``: padding of a ZeroPadding2D fused in front (keras/fusion.py)."""
        from ..ops import pooling as _pool

        if _zero_pad is not None or _pool.supported(x):
            pads = ((0, 0), (0, 0))
            if self.padding == "same":
                pads = (_same_pads(x.shape[1], self.pool_size[0], self.strides[0]),
                        _same_pads(x.shape[2], self.pool_size[1], self.strides[1]))
            if _zero_pad is not None:
                if self.padding == "same":
                    x = F.pad(x, (0, 0, _zero_pad[1][0], _zero_pad[1][1], _zero_pad[0][0], _zero_pad[0][1]))
                else:
                    return _pool.max_pool_nhwc(x, self.pool_size, self.strides, _zero_pad, pad_zero=True)
            return _pool.max_pool_nhwc(x, self.pool_size, self.strides, pads, pad_zero=False)
        h = x.permute(0, 3, 1, 2)
        if self.padding == "same":
            ph, pw = self._pads(h)
            h = F.pad(h, (pw[0], pw[1], ph[0], ph[1]), value=float("-inf"))
        return F.max_pool2d(h, self.pool_size, self.strides).permute(0, 2, 3, 1)


class AveragePooling2D(_Pool2D):
    def call(self, x, training=None):
        h = x.permute(0, 3, 1, 2)
        if self.padding == "same":
            ph, pw = self._pads(h)
            ones = torch.ones_like(h[:, :1])
            hp = F.pad(h, (pw[0], pw[1], ph[0], ph[1]))
            cnt = F.avg_pool2d(F.pad(ones, (pw[0], pw[1], ph[0], ph[1])), self.pool_size, self.strides)
            y = F.avg_pool2d(hp, self.pool_size, self.strides) / cnt
        else:
            y = F.avg_pool2d(h, self.pool_size, self.strides)
        return y.permute(0, 2, 3, 1)


MaxPool2D = MaxPooling2D
AvgPool2D = AveragePooling2D


class GlobalAveragePooling2D(Layer):
    def __init__(self, data_format=None, keepdims=False, **kw):
        super().__init__(**kw)
        self.keepdims = keepdims

    def call(self, x, training=None):
        if not self.keepdims and type(self) is GlobalAveragePooling2D and _dense.gap_supported(x):
            return _dense.gap_nhwc(x)  # hand-written NHWC kernel (ops/dense.py)
        return x.mean(dim=(1, 2), keepdim=self.keepdims)

    def compute_output_shape(self, s):
        return (s[0], 1, 1, s[3]) if self.keepdims else (s[0], s[3])


class GlobalMaxPooling2D(GlobalAveragePooling2D):
    def call(self, x, training=None):
        return x.amax(dim=(1, 2), keepdim=self.keepdims)


GlobalAvgPool2D = GlobalAveragePooling2D
GlobalMaxPool2D = GlobalMaxPooling2D


class Flatten(Layer):
    def __init__(self, data_format=None, **kw):
        super().__init__(**kw)

    def call(self, x, training=None):
        return x.reshape(x.shape[0], -1)  # NHWC -> HWC order, as Keras channels_last

    def compute_output_shape(self, s):
        rest = s[1:]
        return (s[0], None if any(d is None for d in rest) else int(math.prod(rest)))


class Reshape(Layer):
    def __init__(self, target_shape, **kw):
        super().__init__(**kw)
        self.target_shape = tuple(target_shape)

    def call(self, x, training=None):
        return x.reshape((x.shape[0],) + self.target_shape)

    def compute_output_shape(self, s):
        ts = list(self.target_shape)
        if -1 in ts and all(d is not None for d in s[1:]):
            known = math.prod(d for d in ts if d != -1)
            ts[ts.index(-1)] = int(math.prod(s[1:])) // known
        return (s[0],) + tuple(ts)

    def get_config(self):
        return dict(super().get_config(), target_shape=list(self.target_shape))


class Activation(Layer):
    def __init__(self, activation, **kw):
        super().__init__(**kw)
        self.activation = _act.get(activation)

    def call(self, x, training=None):
        return self.activation(x)

    def compute_output_shape(self, s):
        return s

    def get_config(self):
        return dict(super().get_config(), activation=_act.serialize(self.activation))


class ReLU(Layer):
    def __init__(self, max_value=None, negative_slope=0.0, threshold=0.0, **kw):
        super().__init__(**kw)
        self.max_value, self.negative_slope, self.threshold = max_value, negative_slope, threshold

    def call(self, x, training=None):
        return _act.relu(x, self.negative_slope, self.max_value, self.threshold)

    def compute_output_shape(self, s):
        return s


class Softmax(Layer):
    def __init__(self, axis=-1, **kw):
        super().__init__(**kw)
        self.axis = axis

    def call(self, x, training=None):
        return torch.softmax(x, dim=self.axis)

    def compute_output_shape(self, s):
        return s


class Dropout(Layer):
    def __init__(self, rate, noise_shape=None, seed=None, **kw):
        super().__init__(**kw)
        self.rate = float(rate)

    def call(self, x, training=None):
        return F.dropout(x, self.rate, training=bool(training))

    def compute_output_shape(self, s):
        return s


class Rescaling(Layer):
    def __init__(self, scale, offset=0.0, **kw):
        super().__init__(**kw)
        self.scale, self.offset = scale, offset

    def call(self, x, training=None):
        return x.to(torch.float32) * self.scale + self.offset

    def compute_output_shape(self, s):
        return s


class ZeroPadding2D(Layer):
    def __init__(self, padding=(1, 1), data_format=None, **kw):
        super().__init__(**kw)
        if isinstance(padding, int):
            padding = ((padding, padding), (padding, padding))
        elif isinstance(padding[0], int):
            padding = ((padding[0], padding[0]), (padding[1], padding[1]))
        self.padding = tuple(tuple(p) for p in padding)

    def call(self, x, training=None):
        (t, b), (l, r) = self.padding
        return F.pad(x, (0, 0, l, r, t, b))

    def compute_output_shape(self, s):
        (t, b), (l, r) = self.padding
        return (s[0], None if s[1] is None else s[1] + t + b, None if s[2] is None else s[2] + l + r, s[3])


class BatchNormalization(Layer):
    """Keras BatchNormalization: per-replica batch statistics (not synchronised, the Keras default);
    moving mean/variance are ON_READ variables averaged across replicas when read."""

    def __init__(self, axis=-1, momentum=0.99, epsilon=1e-3, center=True, scale=True, beta_initializer="zeros",
                 gamma_initializer="ones", moving_mean_initializer="zeros", moving_variance_initializer="ones",
                 beta_regularizer=None, gamma_regularizer=None, synchronized=False, **kw):
        super().__init__(**kw)
        self.axis = axis
        self.momentum, self.epsilon = float(momentum), float(epsilon)
        self.center, self.scale = center, scale
        self.beta_initializer = _init.get(beta_initializer)
        self.gamma_initializer = _init.get(gamma_initializer)
        self.mm_init = _init.get(moving_mean_initializer)
        self.mv_init = _init.get(moving_variance_initializer)
        self.synchronized = synchronized

    def build(self, input_shape):
        c = int(input_shape[self.axis])
        self.gamma = self.add_weight("gamma", (c,), initializer=self.gamma_initializer) if self.scale else None
        self.beta = self.add_weight("beta", (c,), initializer=self.beta_initializer) if self.center else None
        self.moving_mean = self.add_weight("moving_mean", (c,), initializer=self.mm_init, trainable=False,
                                           synchronization=VariableSynchronization.ON_READ,
                                           aggregation=VariableAggregation.MEAN)
        self.moving_variance = self.add_weight("moving_variance", (c,), initializer=self.mv_init, trainable=False,
                                               synchronization=VariableSynchronization.ON_READ,
                                               aggregation=VariableAggregation.MEAN)
        self.built = True

    def call(self, x, training=None):
        axis = self.axis % x.dim()
        if training and self.trainable and axis == x.dim() - 1 and x.is_cuda:
            # NHWC training on the GPU: hand-written batch-norm kernels (ops/batchnorm.py)
            from ..ops import batchnorm as _bn

            if _bn.supported(x):
                return _bn.batch_norm_train(x, self.gamma.value if self.gamma is not None else None,
                                            self.beta.value if self.beta is not None else None,
                                            self.moving_mean.value, self.moving_variance.value, self.momentum,
                                            self.epsilon, grad_out=self._grad_targets())
        perm = None
        if axis != 1:
            perm = [0, axis] + [i for i in range(1, x.dim()) if i != axis]
            h = x.permute(*perm)
        else:
            h = x
        g = self.gamma.value if self.gamma is not None else None
        b = self.beta.value if self.beta is not None else None
        y = F.batch_norm(h, self.moving_mean.value, self.moving_variance.value,
                         g.to(h.dtype) if g is not None else None, b.to(h.dtype) if b is not None else None,
                         training=bool(training) and self.trainable, momentum=1.0 - self.momentum, eps=self.epsilon)
        if perm is not None:
            inv = [0] * len(perm)
            for i, p in enumerate(perm):
                inv[p] = i
            y = y.permute(*inv)
        return y

    def _grad_targets(self):
        """(gamma, beta) slab views the BN backward kernel adds into directly, or None."""
        t = tuple(v.grad_target() if v is not None else None for v in (self.gamma, self.beta))
        if any(tt is None and v is not None for tt, v in zip(t, (self.gamma, self.beta))):
            return None
        return t

    def compute_output_shape(self, s):
        return s

    def get_config(self):
        return dict(super().get_config(), axis=self.axis, momentum=self.momentum, epsilon=self.epsilon,
                    center=self.center, scale=self.scale)


class LayerNormalization(Layer):
    def __init__(self, axis=-1, epsilon=1e-3, center=True, scale=True, **kw):
        super().__init__(**kw)
        self.axis, self.epsilon, self.center, self.scale = axis, epsilon, center, scale

    def build(self, input_shape):
        c = int(input_shape[-1])
        self.gamma = self.add_weight("gamma", (c,), initializer="ones") if self.scale else None
        self.beta = self.add_weight("beta", (c,), initializer="zeros") if self.center else None
        self.built = True

    def call(self, x, training=None):
        return F.layer_norm(x, (x.shape[-1],), self.gamma.value if self.gamma else None,
                            self.beta.value if self.beta else None, self.epsilon)

    def compute_output_shape(self, s):
        return s


class Embedding(Layer):
    def __init__(self, input_dim, output_dim, embeddings_initializer="uniform", **kw):
        super().__init__(**kw)
        self.input_dim, self.output_dim = int(input_dim), int(output_dim)
        self.emb_init = _init.get("random_uniform" if embeddings_initializer == "uniform" else embeddings_initializer)

    def build(self, input_shape):
        self.embeddings = self.add_weight("embeddings", (self.input_dim, self.output_dim), initializer=self.emb_init)
        self.built = True

    def call(self, x, training=None):
        return F.embedding(x.long(), self.embeddings.value)

    def compute_output_shape(self, s):
        return tuple(s) + (self.output_dim,)


class _Merge(Layer):
    def compute_output_shape(self, shapes):
        return shapes[0]


class Add(_Merge):
    def call(self, xs, training=None):
        y = xs[0]
        for t in xs[1:]:
            y = y + t
        return y


class Subtract(_Merge):
    def call(self, xs, training=None):
        return xs[0] - xs[1]


class Multiply(_Merge):
    def call(self, xs, training=None):
        y = xs[0]
        for t in xs[1:]:
            y = y * t
        return y


class Average(_Merge):
    def call(self, xs, training=None):
        return sum(xs) / len(xs)


class Maximum(_Merge):
    def call(self, xs, training=None):
        y = xs[0]
        for t in xs[1:]:
            y = torch.maximum(y, t)
        return y


class Concatenate(Layer):
    def __init__(self, axis=-1, **kw):
        super().__init__(**kw)
        self.axis = axis

    def call(self, xs, training=None):
        return torch.cat(list(xs), dim=self.axis)

    def compute_output_shape(self, shapes):
        ax = self.axis % len(shapes[0])
        s = list(shapes[0])
        s[ax] = None if any(x[ax] is None for x in shapes) else sum(x[ax] for x in shapes)
        return tuple(s)


class Lambda(Layer):
    def __init__(self, function, output_shape=None, **kw):
        super().__init__(**kw)
        self.function = function
        self._out_shape = output_shape

    def call(self, x, training=None):
        return self.function(x)


def add(inputs, **kw):
    return Add(**kw)(inputs)


def concatenate(inputs, axis=-1, **kw):
    return Concatenate(axis=axis, **kw)(inputs)


def multiply(inputs, **kw):
    return Multiply(**kw)(inputs)


LAYER_CLASSES = {c.__name__: c for c in (
    InputLayer, Dense, Conv2D, MaxPooling2D, AveragePooling2D, GlobalAveragePooling2D, GlobalMaxPooling2D, Flatten,
    Reshape, Activation, ReLU, Softmax, Dropout, Rescaling, ZeroPadding2D, BatchNormalization, LayerNormalization,
    Embedding, Add, Subtract, Multiply, Average, Maximum, Concatenate)}
