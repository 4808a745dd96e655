"""tf.keras.optimizers.schedules: step -> learning rate."""
from __future__ import annotations

import math


class LearningRateSchedule:
    def __call__(self, step):
        raise NotImplementedError

    def get_config(self):
        return {}


class ExponentialDecay(LearningRateSchedule):
    def __init__(self, initial_learning_rate, decay_steps, decay_rate, staircase=False, name=None):
        self.initial_learning_rate, self.decay_steps = initial_learning_rate, decay_steps
        self.decay_rate, self.staircase = decay_rate, staircase

    def __call__(self, step):
        p = step / self.decay_steps
        if self.staircase:
            p = math.floor(p)
        return self.initial_learning_rate * self.decay_rate ** p

    def get_config(self):
        return {"initial_learning_rate": self.initial_learning_rate, "decay_steps": self.decay_steps,
                "decay_rate": self.decay_rate, "staircase": self.staircase}


class InverseTimeDecay(LearningRateSchedule):
    def __init__(self, initial_learning_rate, decay_steps, decay_rate, staircase=False, name=None):
        self.initial_learning_rate, self.decay_steps = initial_learning_rate, decay_steps
        self.decay_rate, self.staircase = decay_rate, staircase

    def __call__(self, step):
        p = step / self.decay_steps
        if self.staircase:
            p = math.floor(p)
        return self.initial_learning_rate / (1 + self.decay_rate * p)

    def get_config(self):
        return {"initial_learning_rate": self.initial_learning_rate, "decay_steps": self.decay_steps,
                "decay_rate": self.decay_rate, "staircase": self.staircase}


class PiecewiseConstantDecay(LearningRateSchedule):
    def __init__(self, boundaries, values, name=None):
        if len(values) != len(boundaries) + 1:
            raise ValueError("len(values) must be len(boundaries) + 1")
        self.boundaries, self.values = list(boundaries), list(values)

    def __call__(self, step):
        for b, v in zip(self.boundaries, self.values):
            if step <= b:
                return v
        return self.values[-1]

    def get_config(self):
        return {"boundaries": self.boundaries, "values": self.values}


class PolynomialDecay(LearningRateSchedule):
    def __init__(self, initial_learning_rate, decay_steps, end_learning_rate=0.0001, power=1.0, cycle=False, name=None):
        self.a, self.n, self.e, self.p, self.cycle = initial_learning_rate, decay_steps, end_learning_rate, power, cycle

    def __call__(self, step):
        n = self.n
        if self.cycle:
            n = n * max(1, math.ceil(step / n))
        s = min(step, n)
        return (self.a - self.e) * (1 - s / n) ** self.p + self.e

    def get_config(self):
        return {"initial_learning_rate": self.a, "decay_steps": self.n, "end_learning_rate": self.e,
                "power": self.p, "cycle": self.cycle}


class CosineDecay(LearningRateSchedule):
    def __init__(self, initial_learning_rate, decay_steps, alpha=0.0, warmup_target=None, warmup_steps=0, name=None):
        self.a, self.n, self.alpha = initial_learning_rate, decay_steps, alpha
        self.warmup_target, self.warmup_steps = warmup_target, warmup_steps

    def __call__(self, step):
        if self.warmup_target is not None and step < self.warmup_steps:
            return self.a + (self.warmup_target - self.a) * step / max(1, self.warmup_steps)
        base = self.warmup_target if self.warmup_target is not None else self.a
        s = min(max(step - self.warmup_steps, 0), self.n)
        cos = 0.5 * (1 + math.cos(math.pi * s / self.n))
        return base * ((1 - self.alpha) * cos + self.alpha)

    def get_config(self):
        return {"initial_learning_rate": self.a, "decay_steps": self.n, "alpha": self.alpha,
                "warmup_target": self.warmup_target, "warmup_steps": self.warmup_steps}


_ALL = {c.__name__: c for c in (ExponentialDecay, InverseTimeDecay, PiecewiseConstantDecay, PolynomialDecay,
                                 CosineDecay)}


def serialize(s: LearningRateSchedule):
    return {"class_name": type(s).__name__, "config": s.get_config()}


def deserialize(d):
    return _ALL[d["class_name"]](**d["config"])
