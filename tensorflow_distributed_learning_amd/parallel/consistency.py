"""Run-time replica-consistency checks for mirrored variables (README.md:15-17).

A MirroredVariable is only "mirrored" while every replica applies bit-identical updates.  The
all-reduce paths here are deterministic by construction (rank-order sums, no float atomics), but a
broken fabric hand-off or a silently dropped collective would let replicas drift without any error.
These helpers make that observable:

* :func:`fingerprint` hashes a flat parameter slab on its own device into two int64 words (a
  position-weighted sum of the raw float bits, so permutations and single-ulp flips both change
  it) without a host copy of the slab;
* :func:`replicas_identical` compares the fingerprints of every replica with ONE small collective
  (max of ``[h, -h]`` equals ``[h, -h]`` on every rank iff all ``h`` are equal);
* :func:`check_and_repair` is what ``fit`` runs periodically (``TDL_CHECK_REPLICAS_EVERY``
  executions, and at the end of ``fit``): on a mismatch it warns, re-synchronises the slab from
  rank 0 over the communicator's library path and reports it, or raises under
  ``TDL_REPLICA_MISMATCH=raise``.
"""
from __future__ import annotations

import os
import warnings

import torch


class ReplicaDivergenceError(RuntimeError):
    pass


_WEIGHTS = {}


def _weights(n: int, device: torch.device) -> torch.Tensor:
    key = (n, str(device))
    w = _WEIGHTS.get(key)
    if w is None:
        # odd multipliers from a 31-bit LCG over the position: distinct, order-sensitive weights
        i = torch.arange(n, dtype=torch.int64, device=device)
        w = ((i * 1103515245 + 12345) % (1 << 31)) | 1
        _WEIGHTS[key] = w
    return w


def fingerprint(t: torch.Tensor) -> torch.Tensor:
    """[2] int64 fingerprint of a contiguous f32/bf16/f16 tensor (on its own device)."""
    flat = t.detach().reshape(-1)
    if flat.dtype == torch.float32:
        bits = flat.view(torch.int32).to(torch.int64)
    elif flat.dtype in (torch.bfloat16, torch.float16):
        bits = flat.view(torch.int16).to(torch.int64)
    else:
        bits = flat.to(torch.float64).view(torch.int64)
    w = _weights(bits.numel(), bits.device)
    lo = (bits & 0xFFFF) * w
    hi = (bits >> 16) * w
    # int64 sums wrap; the wrap is identical on every rank, so equality is preserved
    return torch.stack([lo.sum(), hi.sum()])


def replicas_identical(comm, t: torch.Tensor) -> bool:
    """True iff ``t`` is bit-identical on every replica of ``comm`` (one small collective)."""
    if comm.world_size == 1:
        return True
    h = fingerprint(t)
    ctrl = t.device if getattr(comm, "name", "") == "rccl" else torch.device("cpu")
    v = torch.cat([h, -h]).to(ctrl)
    m = v.clone()
    comm.all_reduce(m, "max")
    return bool(torch.equal(m, v))


def check_and_repair(comm, slab: torch.Tensor, what: str = "parameters") -> bool:
    """Collective: verify ``slab`` is identical on all replicas; on mismatch broadcast rank 0's
    copy (or raise with ``TDL_REPLICA_MISMATCH=raise``).  Returns True if it was consistent."""
    if comm.world_size == 1:
        return True
    ok = replicas_identical(comm, slab)
    if ok:
        return True
    msg = (f"replica divergence detected: the {what} differ across the {comm.world_size} replicas "
           f"(communicator {getattr(comm, 'algorithm', comm.name)})")
    if os.environ.get("TDL_REPLICA_MISMATCH", "repair") == "raise":
        raise ReplicaDivergenceError(msg)
    warnings.warn(msg + "; re-synchronising from rank 0")
    comm.broadcast(slab, 0) if slab.device.type == "cpu" or getattr(comm, "name", "") == "rccl" else \
        _broadcast_staged(comm, slab)
    return False


def _broadcast_staged(comm, slab: torch.Tensor) -> None:
    h = slab.detach().cpu()
    comm.broadcast(h, 0)
    slab.copy_(h)
