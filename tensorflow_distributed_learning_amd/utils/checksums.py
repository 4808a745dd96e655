"""Per-op checksums of one training step (``TDL_DEBUG_CHECKSUMS=1``): a bisection tool for
run-to-run or async-vs-launch-blocking differences in the generic engine.

Every forward output of the functional executor (one entry per node or fused group), every
gradient that reaches such an output in the backward, the whole gradient slab after backward
(per variable) and the weight slab after the optimizer are reduced on the device to
``(float64 sum, float64 abs-sum, bit hash)`` and kept as device tensors (no host sync inside the
step, so the recorder does not serialise what it observes).  :func:`dump` moves them to the host
once, in recording order; ``scripts/diag_checksums.py`` diffs two dumps and names the first tag
that differs.
"""
from __future__ import annotations

import json
import os
from typing import List, Tuple

import torch

_ON = [os.environ.get("TDL_DEBUG_CHECKSUMS", "0") == "1"]
_REC: List[Tuple[str, torch.Tensor]] = []


def enabled() -> bool:
    return _ON[0]


def enable(on: bool = True) -> None:
    _ON[0] = bool(on)


def reset() -> None:
    _REC.clear()


def _digest(t: torch.Tensor) -> torch.Tensor:
    t = t.detach()
    d = t.double()
    # bit hash: integer view of the raw bits, position-weighted so a permutation shows up too
    if t.dtype in (torch.float32, torch.int32):
        bits = t.contiguous().view(torch.int32).long()
    elif t.dtype in (torch.bfloat16, torch.float16, torch.int16):
        bits = t.contiguous().view(torch.int16).long()
    else:
        bits = d.view(torch.int64)
    w = torch.arange(1, bits.numel() + 1, device=t.device, dtype=torch.int64) % 1000003
    h = (bits.reshape(-1) * w).sum().double()
    return torch.stack([d.sum(), d.abs().sum(), h])


def record(tag: str, t) -> None:
    if not _ON[0] or not isinstance(t, torch.Tensor) or t.numel() == 0:
        return
    if t.is_cuda and torch.cuda.is_current_stream_capturing():
        return  # a captured step records once, not per replay: leave graphs alone
    _REC.append((tag, _digest(t)))


def record_tree(tag: str, ts) -> None:
    if isinstance(ts, (list, tuple)):
        for i, t in enumerate(ts):
            record_tree(f"{tag}[{i}]", t)
    else:
        record(tag, ts)


def hook_grad(tag: str, t) -> None:
    """Record the gradient that reaches ``t`` in the backward (a no-op hook otherwise)."""
    if not _ON[0] or not isinstance(t, torch.Tensor) or not t.requires_grad:
        return

    def h(g, tag=tag):
        record("grad:" + tag, g)

    t.register_hook(h)


def dump(path: str) -> List[dict]:
    out = []
    for tag, d in _REC:
        v = d.cpu().tolist()
        out.append({"tag": tag, "sum": v[0], "abs": v[1], "hash": v[2]})
    with open(path, "w") as f:
        json.dump(out, f)
    return out


def first_difference(a: List[dict], b: List[dict], key: str = "hash"):
    """(index, tag_a, tag_b, entry_a, entry_b) of the first entry whose ``key`` differs, or None."""
    for i, (x, y) in enumerate(zip(a, b)):
        if x["tag"] != y["tag"] or x[key] != y[key]:
            return i, x["tag"], y["tag"], x, y
    if len(a) != len(b):
        return min(len(a), len(b)), None, None, None, None
    return None
