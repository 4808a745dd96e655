"""Flat parameter / gradient slabs.

Every replica keeps ALL of a model's variables in one contiguous f32 buffer per device (the
"slab"); Keras-style variables (MirroredVariable) are named views into it.  Gradients live in a
second slab with the same layout, so the cross-replica all-reduce and the optimizer update are
single operations over one buffer (SURVEY.md §2.3 C7/C9, §7.1 principle 2).  Buckets for
overlapped all-reduce are contiguous sub-ranges of the slab.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Sequence, Tuple

import torch

ALIGN = 64  # floats (256 B): every variable starts on a 256-byte boundary (16-B vector access)


@dataclass
class VarSpec:
    name: str
    shape: Tuple[int, ...]
    trainable: bool = True

    @property
    def size(self) -> int:
        return int(math.prod(self.shape)) if self.shape else 1


@dataclass
class SlabLayout:
    specs: List[VarSpec]
    align: int = ALIGN
    offsets: List[int] = field(default_factory=list)
    total: int = 0

    def __post_init__(self):
        off = 0
        self.offsets = []
        for s in self.specs:
            self.offsets.append(off)
            off += s.size
            off = (off + self.align - 1) // self.align * self.align
        self.total = max(off, self.align)

    @classmethod
    def from_shapes(cls, items: Sequence[Tuple[str, Sequence[int]]], align: int = ALIGN) -> "SlabLayout":
        return cls([VarSpec(n, tuple(int(d) for d in s)) for n, s in items], align=align)

    def index(self, name: str) -> int:
        for i, s in enumerate(self.specs):
            if s.name == name:
                return i
        raise KeyError(name)

    def view(self, flat: torch.Tensor, i: int) -> torch.Tensor:
        s = self.specs[i]
        o = self.offsets[i]
        return flat[o : o + s.size].view(s.shape)

    def views(self, flat: torch.Tensor) -> List[torch.Tensor]:
        return [self.view(flat, i) for i in range(len(self.specs))]

    def named_views(self, flat: torch.Tensor) -> Dict[str, torch.Tensor]:
        return {s.name: self.view(flat, i) for i, s in enumerate(self.specs)}

    @property
    def num_params(self) -> int:
        return sum(s.size for s in self.specs)

    def pack(self, tensors: Sequence[torch.Tensor], device=None, dtype=torch.float32) -> torch.Tensor:
        flat = torch.zeros(self.total, dtype=dtype, device=device)
        for i, t in enumerate(tensors):
            self.view(flat, i).copy_(torch.as_tensor(t).reshape(self.specs[i].shape))
        return flat

    def buckets(self, bucket_bytes: int, elem_bytes: int = 4) -> List[Tuple[int, int]]:
        """Contiguous [start, end) slab ranges of ~bucket_bytes, cut at variable boundaries,
        ordered from the END of the slab (the last layers' gradients are produced first in the
        backward pass, so their bucket can be all-reduced while earlier layers still compute)."""
        if bucket_bytes <= 0:
            return [(0, self.total)]
        cap = max(1, bucket_bytes // elem_bytes)
        bounds = self.offsets[1:] + [self.total]
        out: List[Tuple[int, int]] = []
        end = self.total
        start = end
        for i in range(len(self.specs) - 1, -1, -1):
            start = self.offsets[i]
            if end - start >= cap:
                out.append((start, end))
                end = start
        if end > 0:
            out.append((0, end))
        del bounds
        return out
