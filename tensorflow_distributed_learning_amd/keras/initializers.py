"""Keras initializers (defaults of tf_dist_example.py:41-47: glorot_uniform kernels, zero biases)."""
from __future__ import annotations

import math
from typing import Optional, Sequence

import torch

_GEN = torch.Generator()
_GEN.manual_seed(torch.initial_seed() % (1 << 62))


def set_seed(seed: int):
    _GEN.manual_seed(int(seed))


def generator() -> torch.Generator:
    return _GEN


def _fans(shape: Sequence[int]):
    shape = tuple(shape)
    if len(shape) < 1:
        return 1, 1
    if len(shape) == 1:
        return shape[0], shape[0]
    if len(shape) == 2:
        return shape[0], shape[1]
    rf = int(math.prod(shape[:-2]))  # HWIO conv kernels: receptive field = kh*kw
    return shape[-2] * rf, shape[-1] * rf


class Initializer:
    def __call__(self, shape, dtype=torch.float32) -> torch.Tensor:
        raise NotImplementedError

    def get_config(self):
        return {}


class Zeros(Initializer):
    def __call__(self, shape, dtype=torch.float32):
        return torch.zeros(tuple(shape), dtype=dtype)


class Ones(Initializer):
    def __call__(self, shape, dtype=torch.float32):
        return torch.ones(tuple(shape), dtype=dtype)


class Constant(Initializer):
    def __init__(self, value=0.0):
        self.value = value

    def __call__(self, shape, dtype=torch.float32):
        return torch.full(tuple(shape), float(self.value), dtype=dtype)

    def get_config(self):
        return {"value": self.value}


class RandomUniform(Initializer):
    def __init__(self, minval=-0.05, maxval=0.05, seed=None):
        self.minval, self.maxval, self.seed = minval, maxval, seed

    def __call__(self, shape, dtype=torch.float32):
        g = torch.Generator().manual_seed(self.seed) if self.seed is not None else _GEN
        return (torch.rand(tuple(shape), generator=g) * (self.maxval - self.minval) + self.minval).to(dtype)


class RandomNormal(Initializer):
    def __init__(self, mean=0.0, stddev=0.05, seed=None):
        self.mean, self.stddev, self.seed = mean, stddev, seed

    def __call__(self, shape, dtype=torch.float32):
        g = torch.Generator().manual_seed(self.seed) if self.seed is not None else _GEN
        return (torch.randn(tuple(shape), generator=g) * self.stddev + self.mean).to(dtype)


def _truncated_normal(shape, stddev, g):
    t = torch.randn(tuple(shape), generator=g)
    bad = t.abs() > 2
    while bad.any():
        t[bad] = torch.randn(int(bad.sum()), generator=g)
        bad = t.abs() > 2
    return t * stddev


class TruncatedNormal(Initializer):
    def __init__(self, mean=0.0, stddev=0.05, seed=None):
        self.mean, self.stddev, self.seed = mean, stddev, seed

    def __call__(self, shape, dtype=torch.float32):
        g = torch.Generator().manual_seed(self.seed) if self.seed is not None else _GEN
        return (_truncated_normal(shape, self.stddev, g) + self.mean).to(dtype)


class VarianceScaling(Initializer):
    def __init__(self, scale=1.0, mode="fan_in", distribution="truncated_normal", seed=None):
        self.scale, self.mode, self.distribution, self.seed = scale, mode, distribution, seed

    def __call__(self, shape, dtype=torch.float32):
        fan_in, fan_out = _fans(shape)
        n = {"fan_in": fan_in, "fan_out": fan_out, "fan_avg": (fan_in + fan_out) / 2.0}[self.mode]
        s = self.scale / max(1.0, n)
        g = torch.Generator().manual_seed(self.seed) if self.seed is not None else _GEN
        if self.distribution == "uniform":
            lim = math.sqrt(3.0 * s)
            return ((torch.rand(tuple(shape), generator=g) * 2 - 1) * lim).to(dtype)
        if self.distribution in ("truncated_normal", "normal"):
            std = math.sqrt(s) / (0.87962566103423978 if self.distribution == "truncated_normal" else 1.0)
            if self.distribution == "truncated_normal":
                return _truncated_normal(shape, std, g).to(dtype)
            return (torch.randn(tuple(shape), generator=g) * std).to(dtype)
        if self.distribution == "untruncated_normal":
            return (torch.randn(tuple(shape), generator=g) * math.sqrt(s)).to(dtype)
        raise ValueError(f"unknown distribution {self.distribution}")

    def get_config(self):
        return {"scale": self.scale, "mode": self.mode, "distribution": self.distribution, "seed": self.seed}


class _Preset(VarianceScaling):
    def get_config(self):
        return {"seed": self.seed}


class GlorotUniform(_Preset):
    def __init__(self, seed=None):
        super().__init__(1.0, "fan_avg", "uniform", seed)


class GlorotNormal(_Preset):
    def __init__(self, seed=None):
        super().__init__(1.0, "fan_avg", "truncated_normal", seed)


class HeNormal(_Preset):
    def __init__(self, seed=None):
        super().__init__(2.0, "fan_in", "truncated_normal", seed)


class HeUniform(_Preset):
    def __init__(self, seed=None):
        super().__init__(2.0, "fan_in", "uniform", seed)


class LecunNormal(_Preset):
    def __init__(self, seed=None):
        super().__init__(1.0, "fan_in", "truncated_normal", seed)


_ALIASES = {
    "zeros": Zeros, "ones": Ones, "constant": Constant, "random_uniform": RandomUniform,
    "random_normal": RandomNormal, "truncated_normal": TruncatedNormal, "glorot_uniform": GlorotUniform,
    "glorot_normal": GlorotNormal, "he_normal": HeNormal, "he_uniform": HeUniform, "lecun_normal": LecunNormal,
    "variance_scaling": VarianceScaling,
}


def get(identifier) -> Optional[Initializer]:
    if identifier is None:
        return None
    if isinstance(identifier, Initializer):
        return identifier
    if isinstance(identifier, str):
        key = identifier.lower()
        if key not in _ALIASES:
            raise ValueError(f"unknown initializer {identifier!r}")
        return _ALIASES[key]()
    if isinstance(identifier, dict):
        return _ALIASES[identifier["class_name"].lower()](**identifier.get("config", {}))
    if callable(identifier):
        class _Fn(Initializer):
            def __call__(self, shape, dtype=torch.float32):
                return torch.as_tensor(identifier(shape, dtype=dtype), dtype=dtype)
        return _Fn()
    raise ValueError(f"could not interpret initializer {identifier!r}")


def serialize(init: Initializer):
    name = {v: k for k, v in _ALIASES.items()}.get(type(init), type(init).__name__)
    return {"class_name": name, "config": init.get_config()}
