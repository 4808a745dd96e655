"""``import tensorflow as tf`` stand-in covering every API the reference uses
plus the common neighbours (tensor helpers on torch tensors, GradientTape, tf.train, tf.config).
Tensors are ``torch.Tensor``s."""
from __future__ import annotations

import numpy as np
import torch

from .. import data, keras  # noqa: F401
from .. import parallel as distribute  # noqa: F401
from ..ckpt import checkpoint as _ck
from ..data import dataset as _D
from ..parallel import values as _values
from ..parallel.values import Variable as _Var
from ..parallel.values import create_variable as _create_variable

float16, float32, float64 = torch.float16, torch.float32, torch.float64
bfloat16 = torch.bfloat16
int8, int16, int32, int64, uint8 = torch.int8, torch.int16, torch.int32, torch.int64, torch.uint8
bool = torch.bool  # noqa: A001
string = str
Tensor = torch.Tensor
__version__ = "2.99.0-tdl"


def cast(x, dtype):
    """Always returns a NEW tensor (TF tensors are immutable; the reference does ``image /= 255``
    on the result of cast, which must not write back into the dataset)."""
    return torch.as_tensor(x).to(dtype, copy=True)


def constant(value, dtype=None, shape=None, name=None):
    t = torch.as_tensor(np.asarray(value) if not isinstance(value, torch.Tensor) else value)
    if dtype is not None:
        t = t.to(dtype)
    if shape is not None:
        t = t.expand(shape) if t.numel() == 1 else t.reshape(shape)
    return t.clone()


convert_to_tensor = constant


def zeros(shape, dtype=float32):
    return torch.zeros(shape, dtype=dtype)


def ones(shape, dtype=float32):
    return torch.ones(shape, dtype=dtype)


def reshape(x, shape):
    return torch.as_tensor(x).reshape(shape)


def shape(x):
    return torch.tensor(tuple(torch.as_tensor(x).shape))


def reduce_sum(x, axis=None, keepdims=False):
    x = torch.as_tensor(x)
    return x.sum() if axis is None else x.sum(dim=axis, keepdim=keepdims)


def reduce_mean(x, axis=None, keepdims=False):
    x = torch.as_tensor(x)
    return x.mean() if axis is None else x.mean(dim=axis, keepdim=keepdims)


def reduce_max(x, axis=None, keepdims=False):
    x = torch.as_tensor(x)
    return x.max() if axis is None else x.amax(dim=axis, keepdim=keepdims)


def argmax(x, axis=None):
    return torch.as_tensor(x).argmax(dim=axis)


def square(x):
    return torch.as_tensor(x) ** 2


def sqrt(x):
    return torch.sqrt(torch.as_tensor(x))


def exp(x):
    return torch.exp(torch.as_tensor(x))


def matmul(a, b):
    return torch.matmul(a, b)


def concat(values, axis):
    return torch.cat(list(values), dim=axis)


def stack(values, axis=0):
    return torch.stack(list(values), dim=axis)


def expand_dims(x, axis):
    return torch.as_tensor(x).unsqueeze(axis)


def squeeze(x, axis=None):
    x = torch.as_tensor(x)
    return x.squeeze() if axis is None else x.squeeze(axis)


def one_hot(indices, depth, dtype=float32):
    return torch.nn.functional.one_hot(torch.as_tensor(indices).long(), depth).to(dtype)


def identity(x):
    return torch.as_tensor(x).clone()


def function(fn=None, **kw):
    """tf.function: eager here (the engine captures hipGraphs itself)."""
    if fn is None:
        return lambda f: f
    return fn


def Variable(initial_value, trainable=True, name="Variable", dtype=None, **kw):  # noqa: N802
    return _create_variable(initial_value, name=name, trainable=trainable, dtype=dtype)


class nn:  # noqa: N801
    relu = staticmethod(torch.relu)
    softmax = staticmethod(lambda x, axis=-1: torch.softmax(x, axis))
    sparse_softmax_cross_entropy_with_logits = staticmethod(
        lambda labels, logits: torch.nn.functional.cross_entropy(logits, labels.long(), reduction="none"))

    @staticmethod
    def compute_average_loss(per_example_loss, sample_weight=None, global_batch_size=None):
        from ..parallel.strategy import get_strategy

        l = torch.as_tensor(per_example_loss)
        if sample_weight is not None:
            l = l * sample_weight
        gbs = global_batch_size or l.shape[0] * get_strategy().num_replicas_in_sync
        return l.sum() / gbs


class random:  # noqa: N801
    @staticmethod
    def set_seed(seed):
        from ..keras.utils import set_random_seed

        set_random_seed(seed)

    @staticmethod
    def normal(shape, mean=0.0, stddev=1.0, dtype=float32, seed=None):
        return torch.randn(shape, dtype=dtype) * stddev + mean

    @staticmethod
    def uniform(shape, minval=0.0, maxval=1.0, dtype=float32, seed=None):
        return torch.rand(shape, dtype=dtype) * (maxval - minval) + minval


class _PhysicalDevice:
    def __init__(self, name, device_type):
        self.name, self.device_type = name, device_type

    def __repr__(self):
        return f"PhysicalDevice(name='{self.name}', device_type='{self.device_type}')"


class config:  # noqa: N801
    @staticmethod
    def list_physical_devices(device_type=None):
        out = [_PhysicalDevice("/physical_device:CPU:0", "CPU")]
        out += [_PhysicalDevice(f"/physical_device:GPU:{i}", "GPU") for i in range(torch.cuda.device_count())]
        return [d for d in out if device_type is None or d.device_type == device_type]

    list_logical_devices = list_physical_devices

    class experimental:  # noqa: N801
        @staticmethod
        def set_memory_growth(device, enable):
            return None

        @staticmethod
        def list_physical_devices(device_type=None):
            return config.list_physical_devices(device_type)


class train:  # noqa: N801
    Checkpoint = _ck.Checkpoint
    CheckpointManager = _ck.CheckpointManager
    latest_checkpoint = staticmethod(_ck.latest_checkpoint)
    list_variables = staticmethod(_ck.list_variables)


class saved_model:  # noqa: N801
    @staticmethod
    def save(obj, export_dir, signatures=None, options=None):
        obj.save(export_dir)

    @staticmethod
    def load(export_dir, tags=None, options=None):
        return keras.models.load_model(export_dir)


_TAPES = []


class GradientTape:
    """Eager autograd tape over framework Variables (custom training loops)."""

    def __init__(self, persistent=False, watch_accessed_variables=True):
        self.persistent = persistent

    def __enter__(self):
        _TAPES.append(self)
        _values.TAPE_DEPTH[0] += 1
        return self

    def __exit__(self, *a):
        _TAPES.pop()
        _values.TAPE_DEPTH[0] -= 1

    def watch(self, t):
        if isinstance(t, torch.Tensor):
            t.requires_grad_(True)

    def gradient(self, target, sources, output_gradients=None, unconnected_gradients=None):
        single = not isinstance(sources, (list, tuple))
        srcs = [sources] if single else list(sources)
        ts = []
        for s in srcs:
            if isinstance(s, _Var):
                if s._leaf is None or not s._leaf.requires_grad:
                    raise ValueError(f"{s.name} was not used under this tape")
                ts.append(s._leaf)
            else:
                ts.append(s)
        gs = torch.autograd.grad(target, ts, grad_outputs=output_gradients, allow_unused=True,
                                 retain_graph=self.persistent)
        gs = [g if g is not None else torch.zeros_like(t) for g, t in zip(gs, ts)]
        return gs[0] if single else gs
