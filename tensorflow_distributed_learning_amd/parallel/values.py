"""Distributed variables (README.md:15 "MirroredVariable").

Under a strategy every model variable is a :class:`MirroredVariable`: one logical variable whose
per-replica copy lives in that replica's flat parameter slab (engine/slab.py).  All replicas start
from the chief's initial values (broadcast at build time) and apply identical all-reduced updates,
so the copies stay bit-identical.  Metric accumulators and BatchNorm moving statistics are
:class:`SyncOnReadVariable`: each replica updates its own copy; reading aggregates across replicas.
"""
from __future__ import annotations

import enum
from typing import Optional

import numpy as np
import torch


TAPE_DEPTH = [0]  # > 0 while a compat GradientTape is recording


_CURRENT = []


def _replica_device():
    if not _CURRENT:
        from .local_replicas import CURRENT

        _CURRENT.append(CURRENT)
    return getattr(_CURRENT[0], "device", None)
CAST_ACCUMULATE = [0]  # > 0 while GenericTrainer.train_step runs its forward (Variable.cast fast path)


class VariableSynchronization(enum.Enum):
    AUTO = 0
    NONE = 1
    ON_WRITE = 2
    ON_READ = 3


class VariableAggregation(enum.Enum):
    NONE = 0
    SUM = 1
    MEAN = 2
    ONLY_FIRST_REPLICA = 3


class _CastAccumulate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, leaf, gview, dtype, cview=None):
        ctx.gview = gview
        # cview: this variable's view of the trainer's compute-dtype weight slab (cast once per step)
        return cview.view_as(cview) if cview is not None else leaf.detach().to(dtype)

    @staticmethod
    def backward(ctx, g):
        ctx.gview.add_(g.reshape(ctx.gview.shape))
        return None, None, None, None


class Variable:
    """A named tensor whose storage may be a view into a replica slab."""

    def __init__(self, initial_value, name: str = "Variable", trainable: bool = True,
                 synchronization=VariableSynchronization.AUTO, aggregation=VariableAggregation.NONE,
                 dtype: Optional[torch.dtype] = None, strategy=None):
        t = torch.as_tensor(initial_value() if callable(initial_value) else initial_value)
        if dtype is not None:
            t = t.to(dtype)
        self._value = t.clone()
        self._leaf: Optional[torch.Tensor] = None  # autograd leaf sharing storage with the slab view
        self.name = name if name.endswith(":0") else name + ":0"
        self.trainable = trainable
        self.synchronization = synchronization
        self.aggregation = aggregation
        self._strategy = strategy

    # ------------------------------------------------------------------ storage binding
    def _bind(self, view: torch.Tensor, copy: bool = True):
        if copy:
            view.copy_(self._value.to(view.device, view.dtype).reshape(view.shape))
        self._value = view
        self._leaf = None

    @property
    def value(self) -> torch.Tensor:
        if TAPE_DEPTH[0] > 0 and self.trainable and (self._leaf is None or not self._leaf.requires_grad):
            # inside a GradientTape: expose an autograd leaf sharing this variable's storage
            self._leaf = self._value.detach().requires_grad_(True)
        t = self._leaf if self._leaf is not None else self._value
        dev = _replica_device()
        if dev is not None and t.device != dev:
            # read inside replica r's function of a single-process multi-device MirroredStrategy:
            # replica r's (mirrored) copy on its device; differentiable, so a tape's gradient
            # arrives at the variable (parallel/local_replicas.py)
            t = t.to(dev)
        return t

    def cast(self, dtype: torch.dtype) -> torch.Tensor:
        """``value.to(dtype)`` for a compute-dtype copy (mixed_bfloat16). When the generic trainer
        bound the leaf's gradient to a slab view (``_tdl_gview``), the backward adds the bf16
        gradient straight into that f32 view in one mixed-dtype kernel, instead of a bf16->f32
        cast kernel followed by AccumulateGrad's f32 add (ResNet-50: 53 conv kernels per step)."""
        t = self.value
        if t.dtype == dtype:
            return t
        g = getattr(t, "_tdl_gview", None)
        # only inside the trainer's own step: a GradientTape loop (or any other autograd user) on
        # the same leaves must see an ordinary differentiable cast, not a gradient routed into G
        if (g is not None and CAST_ACCUMULATE[0] > 0 and TAPE_DEPTH[0] == 0 and t.requires_grad and
                torch.is_grad_enabled()):
            return _CastAccumulate.apply(t, g, dtype, self.compute_view(dtype))
        return t.to(dtype)

    def compute_view(self, dtype: torch.dtype) -> Optional[torch.Tensor]:
        """This variable's view of the trainer's compute-dtype copy of the weight slab (refreshed by
        ONE cast kernel at the start of every GenericTrainer step), or None outside such a step."""
        cv = getattr(self.value, "_tdl_cview", None)
        if cv is not None and cv.dtype == dtype and CAST_ACCUMULATE[0] > 0:
            return cv
        return None

    def compute_view_ohwi(self, dtype: torch.dtype) -> Optional[torch.Tensor]:
        """Conv kernels: the step's OHWI [K,KH,KW,C] compute-dtype copy (see :meth:`compute_view`)."""
        tv = getattr(self.value, "_tdl_tview", None)
        if tv is not None and tv.dtype == dtype and CAST_ACCUMULATE[0] > 0:
            return tv
        return None

    def grad_target(self) -> Optional[torch.Tensor]:
        """The f32 slab view a hand-written kernel may ADD this variable's gradient into directly
        (skipping autograd's accumulate kernel), or None.  Same conditions as the :meth:`cast`
        fast path: inside GenericTrainer.train_step, no GradientTape, gradient slab bound (no
        bucket all-reduce hooks waiting on this leaf)."""
        t = self.value
        g = getattr(t, "_tdl_gview", None)
        if (g is not None and CAST_ACCUMULATE[0] > 0 and TAPE_DEPTH[0] == 0 and t.requires_grad and
                torch.is_grad_enabled()):
            return g
        return None

    def read_value(self) -> torch.Tensor:
        return self._value

    def numpy(self) -> np.ndarray:
        return self.read_value().detach().cpu().numpy().copy()

    def __array__(self, dtype=None):
        a = self.numpy()
        return a.astype(dtype) if dtype is not None else a

    @property
    def shape(self):
        return tuple(self._value.shape)

    @property
    def dtype(self):
        return self._value.dtype

    @property
    def device(self):
        return self._value.device

    @property
    def values(self):
        return (self,)

    def assign(self, v, read_value=True):
        with torch.no_grad():
            self._value.copy_(torch.as_tensor(np.asarray(v) if not isinstance(v, torch.Tensor) else v)
                              .to(self._value.device, self._value.dtype).reshape(self._value.shape))
        return self

    def assign_add(self, v):
        with torch.no_grad():
            self._value.add_(torch.as_tensor(v).to(self._value.device, self._value.dtype))
        return self

    def assign_sub(self, v):
        with torch.no_grad():
            self._value.sub_(torch.as_tensor(v).to(self._value.device, self._value.dtype))
        return self

    def __repr__(self):
        return f"<{type(self).__name__} '{self.name}' shape={self.shape} dtype={self.dtype}>"


class MirroredVariable(Variable):
    """Replicated variable, synchronised on write (every replica applies the same update)."""


class SyncOnReadVariable(Variable):
    """Per-replica variable aggregated across replicas when read (metrics, BN moving stats)."""

    def read_value(self) -> torch.Tensor:
        s = self._strategy
        if s is None or s.num_replicas_in_sync == 1:
            return self._value
        from .strategy import in_cross_replica_context

        if not in_cross_replica_context():
            return self._value
        op = "MEAN" if self.aggregation == VariableAggregation.MEAN else "SUM"
        if self.aggregation == VariableAggregation.ONLY_FIRST_REPLICA:
            t = self._value.clone()
            s.extended.broadcast(t, 0)
            return t
        return s.extended.all_reduce(op, self._value)


class PerReplica:
    """Values of one logical tensor, one per local replica (one per process here)."""

    def __init__(self, values):
        self.values = tuple(values)

    def __repr__(self):
        return f"PerReplica({self.values})"


def create_variable(initial_value, name, trainable=True, synchronization=VariableSynchronization.AUTO,
                    aggregation=VariableAggregation.NONE, dtype=None):
    """Variable creator honouring the current strategy scope (variable_creator_scope equivalent)."""
    from .strategy import get_strategy, has_strategy

    strategy = get_strategy() if has_strategy() else None
    if synchronization == VariableSynchronization.ON_READ:
        cls = SyncOnReadVariable
    elif strategy is not None:
        cls = MirroredVariable
    else:
        cls = Variable
    return cls(initial_value, name=name, trainable=trainable, synchronization=synchronization,
               aggregation=aggregation, dtype=dtype, strategy=strategy)
