"""Keras optimizers over the flat parameter slab.

Every replica applies the optimizer to its whole slab in ONE update after the gradient
all-reduce (TF applies ``ResourceApplyGradientDescent`` once per variable).  On the GPU every
optimizer is one hand-written gfx950 kernel over the slab (``_C.sgd`` / ``_C.sgd_momentum``,
``_C.adam`` (AdamW's decay in the same pass), ``_C.rmsprop``, ``_C.adagrad``; csrc/kernels/optim.hip),
with the learning rate and Adam's step count read from device memory so the update can sit inside
a captured hipGraph.  Gradient clipping keeps its torch ops (a global norm).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch

from . import schedules as _sched


class Optimizer:
    def __init__(self, learning_rate=0.001, name="Optimizer", clipnorm=None, clipvalue=None, global_clipnorm=None,
                 weight_decay=None, **kwargs):
        self.name = name
        self._lr = learning_rate
        self.clipnorm, self.clipvalue, self.global_clipnorm = clipnorm, clipvalue, global_clipnorm
        self.weight_decay = weight_decay
        self.iterations = 0
        self._slots: Dict[str, torch.Tensor] = {}
        self._n = None
        self._device = None
        self.lr_dev: Optional[torch.Tensor] = None
        self._lr_synced = None  # (value, lr_dev address) last written by _sync_lr
        # device copy of ``iterations`` at the start of the next step / execution (Adam's bias
        # correction on the device: a captured step graph reads it, each step adds its offset)
        self.t_dev: Optional[torch.Tensor] = None
        self._t_synced = None
        unknown = set(kwargs) - {"decay", "amsgrad_legacy", "jit_compile", "is_legacy_optimizer",
                                 "use_ema", "ema_momentum", "ema_overwrite_frequency"}
        if unknown:
            raise TypeError(f"{type(self).__name__}: unexpected arguments {sorted(unknown)}")

    # ------------------------------------------------------------------ learning rate
    @property
    def learning_rate(self):
        return self._lr

    @learning_rate.setter
    def learning_rate(self, v):
        self._lr = v

    lr = learning_rate

    def current_lr(self, step: Optional[int] = None) -> float:
        lr = self._lr
        if isinstance(lr, _sched.LearningRateSchedule):
            return float(lr(self.iterations if step is None else step))
        if callable(lr):
            return float(lr())
        return float(lr)

    def _sync_lr(self, step: Optional[int] = None):
        # one fill kernel only when the value changes: a constant learning rate costs no launch in
        # front of every graph replay (the device copy is written nowhere else)
        if self.lr_dev is not None:
            v = self.current_lr(step)
            if self._lr_synced != (v, self.lr_dev.data_ptr()):
                self.lr_dev.fill_(v)
                self._lr_synced = (v, self.lr_dev.data_ptr())
        if self.t_dev is not None and self._needs_step:
            t = float(self.iterations if step is None else step)
            if self._t_synced != (t, self.t_dev.data_ptr()):
                self.t_dev.fill_(t)
                self._t_synced = (t, self.t_dev.data_ptr())

    _needs_step = False  # the device update reads t_dev (Adam's bias correction)

    def device_update(self, W: torch.Tensor, G: torch.Tensor, t_add: int = 0) -> bool:
        """One hand-written flat-slab update kernel (learning rate and step count read from the
        device: capturable) when this optimizer has one and the slab is on the GPU; False
        otherwise (the caller then uses apply_flat).  ``t_add``: the step's offset inside an
        execution whose first step is t_dev (Adam)."""
        return False

    # ------------------------------------------------------------------ slots
    def build(self, n: int, device: torch.device):
        if self._n == n and self._device == device:
            return
        self._n, self._device = n, device
        self.lr_dev = torch.full((1,), self.current_lr(), dtype=torch.float32, device=device)
        self._lr_synced = (self.current_lr(), self.lr_dev.data_ptr())
        self.t_dev = torch.full((1,), float(self.iterations), dtype=torch.float32, device=device)
        self._t_synced = (float(self.iterations), self.t_dev.data_ptr())
        for k in self._slot_names():
            old = self._slots.get(k)
            self._slots[k] = old.to(device) if (old is not None and old.numel() == n) else torch.zeros(
                n, dtype=torch.float32, device=device)

    def _slot_names(self) -> List[str]:
        return []

    def slots(self) -> Dict[str, torch.Tensor]:
        return self._slots

    # ------------------------------------------------------------------ update
    def _clip(self, G: torch.Tensor):
        if self.clipvalue is not None:
            G.clamp_(-self.clipvalue, self.clipvalue)
        norm = self.global_clipnorm or self.clipnorm
        if norm is not None:
            n = torch.linalg.vector_norm(G)
            G.mul_(torch.clamp(norm / (n + 1e-12), max=1.0))

    def apply_flat(self, W: torch.Tensor, G: torch.Tensor, sync_lr: bool = True, t_add: int = 0):
        """w <- update(w, g) over the whole slab (gradients already all-reduced).  ``t_add``: this
        step's offset from ``t_dev`` inside a multi-step execution (only Adam reads a step count)."""
        if self._n != W.numel() or self._device != W.device:
            self.build(W.numel(), W.device)
        if sync_lr:
            self._sync_lr()
        self._clip(G)
        if self.weight_decay:
            W.mul_(1.0 - self.current_lr() * self.weight_decay)
        with torch.no_grad():
            self._update(W, G)
        self.iterations += 1

    def _update(self, W, G):
        raise NotImplementedError

    def apply_gradients(self, grads_and_vars):
        """Eager per-variable path for custom training loops (tf.GradientTape style).

        Called from the replica functions of a single-process multi-device MirroredStrategy
        (``strategy.run``), this is TF's merge call: the replicas' gradients are summed across
        replicas in rank order and the variables are updated ONCE, by the last replica to arrive
        (parallel/local_replicas.py rendezvous)."""
        gv = [(g, v) for g, v in grads_and_vars if g is not None]
        from ..parallel.strategy import get_strategy, has_strategy

        grp = getattr(get_strategy(), "_local_group", None) if has_strategy() else None
        if grp is not None and grp.in_region():
            def merge(per_replica):
                n = len(per_replica[0])
                if any(len(p) != n for p in per_replica):
                    raise ValueError("apply_gradients: replicas passed different variable lists")
                # (custom-loop path, not the fit engine: full device syncs order the replicas'
                # gradient producers on their streams against this thread's update)
                if grp.device_comm().gpu:
                    grp.device_comm().synchronize()
                summed = []
                for i in range(n):
                    v = per_replica[0][i][1]
                    dev = v.read_value().device
                    acc = torch.as_tensor(per_replica[0][i][0]).to(dev, copy=True)
                    for p in per_replica[1:]:
                        acc += torch.as_tensor(p[i][0]).to(dev)
                    summed.append((acc, v))
                self._apply_gradients_now(summed)
                if grp.device_comm().gpu:
                    grp.device_comm().synchronize()

            grp.rendezvous(gv, merge)
            return
        self._apply_gradients_now(gv)

    def _apply_gradients_now(self, gv):
        if not gv:
            return
        flat_g = torch.cat([torch.as_tensor(g).reshape(-1).float() for g, _ in gv])
        flat_w = torch.cat([v.read_value().reshape(-1).float() for _, v in gv])
        key = "_eager"
        if getattr(self, key, None) is None or self._n != flat_w.numel():
            self.build(flat_w.numel(), flat_w.device)
            setattr(self, key, True)
        self.apply_flat(flat_w, flat_g.to(flat_w.device))
        off = 0
        for _, v in gv:
            n = int(math.prod(v.shape))
            v.assign(flat_w[off : off + n].reshape(v.shape))
            off += n

    def variables(self):
        return [self.iterations] + list(self._slots.values())

    def get_config(self):
        lr = self._lr
        if isinstance(lr, _sched.LearningRateSchedule):
            lr = _sched.serialize(lr)
        return {"name": self.name, "learning_rate": lr, "clipnorm": self.clipnorm, "clipvalue": self.clipvalue,
                "global_clipnorm": self.global_clipnorm}

    @classmethod
    def from_config(cls, cfg):
        cfg = dict(cfg)
        if isinstance(cfg.get("learning_rate"), dict):
            cfg["learning_rate"] = _sched.deserialize(cfg["learning_rate"])
        return cls(**cfg)

    def state_dict(self):
        return {"iterations": self.iterations, "slots": {k: v.detach().cpu() for k, v in self._slots.items()}}

    def load_state_dict(self, st):
        self.iterations = int(st.get("iterations", 0))
        for k, v in st.get("slots", {}).items():
            self._slots[k] = v.to(self._device) if self._device is not None else v.clone()


def _kernel_present(kernel: str) -> bool:
    from .. import ops

    return ops.hip_available() and hasattr(ops.hip(), kernel)


def _hip_ok(t: torch.Tensor, kernel: str = "sgd") -> bool:
    if t.device.type != "cuda" or t.dtype != torch.float32:
        return False
    from .. import ops

    return hasattr(ops.hip(), kernel)  # ops.hip() raises loudly if the HIP kernels are missing on a GPU box


class SGD(Optimizer):
    """tf.keras.optimizers.SGD(learning_rate=0.01, momentum=0.0, nesterov=False) (ex:51)."""

    # the GPU update reads the learning rate from ``lr_dev`` (refreshed before every step), so a
    # captured step graph stays correct under learning-rate schedules
    graph_safe = True

    def __init__(self, learning_rate=0.01, momentum=0.0, nesterov=False, name="SGD", **kw):
        super().__init__(learning_rate, name, **kw)
        if not 0.0 <= momentum <= 1.0:
            raise ValueError("momentum must be in [0, 1]")
        self.momentum, self.nesterov = float(momentum), bool(nesterov)

    def _slot_names(self):
        return ["momentum"] if self.momentum > 0 else []

    def device_update(self, W, G, t_add=0):
        if not _hip_ok(W) or self.weight_decay:
            return False
        from .. import ops

        C = ops.hip()
        # (the generic trainer's request: zero G after its use, so its next step needs no fill launch)
        zero = bool(getattr(self, "_zero_grad_after", False))
        if self.momentum > 0:
            C.sgd_momentum(W, G, self._slots["momentum"], self.lr_dev, self.momentum, self.nesterov, zero_grad=zero)
        else:
            C.sgd(W, G, self.lr_dev, zero_grad=zero)
        self._zeroed_grad = zero
        return True

    def _update(self, W, G):
        if self.device_update(W, G):
            return
        lr = self.current_lr()
        if self.momentum > 0:
            v = self._slots["momentum"]
            v.mul_(self.momentum).add_(G, alpha=-lr)
            if self.nesterov:
                W.add_(v, alpha=self.momentum).add_(G, alpha=-lr)
            else:
                W.add_(v)
        else:
            W.add_(G, alpha=-lr)

    def get_config(self):
        return dict(super().get_config(), momentum=self.momentum, nesterov=self.nesterov)


class Adam(Optimizer):
    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-7, amsgrad=False, name="Adam", **kw):
        super().__init__(learning_rate, name, **kw)
        self.beta_1, self.beta_2, self.epsilon, self.amsgrad = beta_1, beta_2, epsilon, amsgrad

    def _slot_names(self):
        return ["m", "v"] + (["vhat"] if self.amsgrad else [])

    @property
    def graph_safe(self) -> bool:
        """Whether a captured step replays this update correctly: only the kernel path reads the
        learning rate and the step count from device memory (t_dev); the clipping fallback
        (_update) bakes the capture-time values into the graph."""
        if self.clipvalue is not None or self.clipnorm or self.global_clipnorm:
            return False
        return _kernel_present("adam")

    _needs_step = True

    def device_update(self, W, G, t_add=0):
        """csrc/kernels/optim.hip k_adam (AdamW's decoupled decay inside the same pass)."""
        if not _hip_ok(W, "adam"):
            return False
        from .. import ops

        ops.hip().adam(W, G, self._slots["m"], self._slots["v"], self._slots.get("vhat"), self.lr_dev, self.t_dev,
                       int(t_add), self.beta_1, self.beta_2, self.epsilon, float(self.weight_decay or 0.0))
        return True

    def apply_flat(self, W, G, sync_lr: bool = True, t_add: int = 0):
        if self._n != W.numel() or self._device != W.device:
            self.build(W.numel(), W.device)
        if sync_lr:
            self._sync_lr()
        if (self.clipvalue is None and not (self.global_clipnorm or self.clipnorm)
                and self.device_update(W, G, t_add)):  # decay + update in one kernel
            self.iterations += 1
            return
        super().apply_flat(W, G, sync_lr=False)

    def _update(self, W, G):
        t = self.iterations + 1
        lr = self.current_lr()
        m, v = self._slots["m"], self._slots["v"]
        m.mul_(self.beta_1).add_(G, alpha=1 - self.beta_1)
        v.mul_(self.beta_2).addcmul_(G, G, value=1 - self.beta_2)
        lr_t = lr * math.sqrt(1 - self.beta_2 ** t) / (1 - self.beta_1 ** t)
        vv = v
        if self.amsgrad:
            torch.maximum(self._slots["vhat"], v, out=self._slots["vhat"])
            vv = self._slots["vhat"]
        W.addcdiv_(m, vv.sqrt().add_(self.epsilon), value=-lr_t)

    def get_config(self):
        return dict(super().get_config(), beta_1=self.beta_1, beta_2=self.beta_2, epsilon=self.epsilon,
                    amsgrad=self.amsgrad)


class AdamW(Adam):
    def __init__(self, learning_rate=0.001, weight_decay=0.004, beta_1=0.9, beta_2=0.999, epsilon=1e-7, amsgrad=False,
                 name="AdamW", **kw):
        super().__init__(learning_rate, beta_1, beta_2, epsilon, amsgrad, name, weight_decay=weight_decay, **kw)


class RMSprop(Optimizer):
    def __init__(self, learning_rate=0.001, rho=0.9, momentum=0.0, epsilon=1e-7, centered=False, name="RMSprop", **kw):
        super().__init__(learning_rate, name, **kw)
        self.rho, self.momentum, self.epsilon, self.centered = rho, momentum, epsilon, centered

    def _slot_names(self):
        return ["rms"] + (["mom"] if self.momentum > 0 else []) + (["mg"] if self.centered else [])

    graph_safe = property(lambda self: _kernel_present("rmsprop"))  # (the torch fallback bakes lr)

    def device_update(self, W, G, t_add=0):
        """csrc/kernels/optim.hip k_rmsprop."""
        if not _hip_ok(W, "rmsprop") or self.weight_decay:
            return False
        from .. import ops

        ops.hip().rmsprop(W, G, self._slots["rms"], self._slots.get("mom"), self._slots.get("mg"), self.lr_dev,
                          self.rho, self.momentum, self.epsilon)
        return True

    def _update(self, W, G):
        if self.device_update(W, G):
            return
        lr = self.current_lr()
        rms = self._slots["rms"]
        rms.mul_(self.rho).addcmul_(G, G, value=1 - self.rho)
        denom = rms
        if self.centered:
            mg = self._slots["mg"]
            mg.mul_(self.rho).add_(G, alpha=1 - self.rho)
            denom = rms - mg * mg
        step = G / (denom.sqrt() + self.epsilon)
        if self.momentum > 0:
            mom = self._slots["mom"]
            mom.mul_(self.momentum).add_(step, alpha=lr)
            W.sub_(mom)
        else:
            W.add_(step, alpha=-lr)


class Adagrad(Optimizer):
    def __init__(self, learning_rate=0.001, initial_accumulator_value=0.1, epsilon=1e-7, name="Adagrad", **kw):
        super().__init__(learning_rate, name, **kw)
        self.init_acc, self.epsilon = initial_accumulator_value, epsilon

    def _slot_names(self):
        return ["acc"]

    def build(self, n, device):
        fresh = "acc" not in self._slots
        super().build(n, device)
        if fresh:
            self._slots["acc"].fill_(self.init_acc)

    graph_safe = property(lambda self: _kernel_present("adagrad"))

    def device_update(self, W, G, t_add=0):
        """csrc/kernels/optim.hip k_adagrad."""
        if not _hip_ok(W, "adagrad") or self.weight_decay:
            return False
        from .. import ops

        ops.hip().adagrad(W, G, self._slots["acc"], self.lr_dev, self.epsilon)
        return True

    def _update(self, W, G):
        if self.device_update(W, G):
            return
        acc = self._slots["acc"]
        acc.addcmul_(G, G)
        W.addcdiv_(G, acc.sqrt().add_(self.epsilon), value=-self.current_lr())


_ALIASES = {"sgd": SGD, "adam": Adam, "adamw": AdamW, "rmsprop": RMSprop, "adagrad": Adagrad}


def get(identifier) -> Optimizer:
    if isinstance(identifier, Optimizer):
        return identifier
    if isinstance(identifier, str):
        k = identifier.lower()
        if k not in _ALIASES:
            raise ValueError(f"unknown optimizer {identifier!r}")
        return _ALIASES[k]()
    if isinstance(identifier, dict):
        return _ALIASES[identifier["class_name"].lower()].from_config(identifier.get("config", {}))
    raise ValueError(f"could not interpret optimizer {identifier!r}")


def serialize(opt: Optimizer):
    return {"class_name": type(opt).__name__, "config": opt.get_config()}


schedules = _sched


class legacy:  # noqa: N801 - tf.keras.optimizers.legacy
    SGD = SGD
    Adam = Adam
    RMSprop = RMSprop
    Adagrad = Adagrad
