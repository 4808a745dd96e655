"""Tracing ranges for ROCm profilers (tracing row).

``TDL_TRACE=1`` turns on roctx ranges (``torch.cuda.nvtx`` is roctx on ROCm builds) around each
``fit`` execution and each generic train-step phase (forward, backward, all-reduce, optimizer), so a
``rocprofv3 --marker-trace --kernel-trace`` timeline shows which kernels belong to which phase.
Off by default: a disabled range costs one attribute lookup.
"""
from __future__ import annotations

import contextlib
import os

import torch

ENABLED = os.environ.get("TDL_TRACE", "0") == "1"


def _push(name: str):
    try:
        torch.cuda.nvtx.range_push(name)
        return True
    except Exception:  # no roctx in this build / no GPU
        return False


@contextlib.contextmanager
def trace_range(name: str):
    """roctx range ``name`` when tracing is enabled, else a no-op."""
    if not ENABLED:
        yield
        return
    pushed = _push(name)
    try:
        yield
    finally:
        if pushed:
            torch.cuda.nvtx.range_pop()


def set_enabled(on: bool) -> None:
    global ENABLED
    ENABLED = bool(on)
