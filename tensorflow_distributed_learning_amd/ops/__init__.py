"""Loader for the in-tree native extensions.

``_C``      hand-written gfx950 HIP kernels (csrc/kernels/*.hip) – the GPU compute path.
``_native`` C++ runtime (csrc/native/*.cpp) – rendezvous / KV store, TCP ring all-reduce.

Both are built in place by ``python build_native.py`` (or ``__graft_entry__.build()``).  On a
machine with a GPU the HIP path is mandatory: :func:`hip` raises instead of silently falling back
to eager PyTorch ops, so a missing or stale extension is loud.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_cache: dict = {}


class NativeExtensionMissing(ImportError):
    pass


def _load(name: str):
    with _lock:
        if name in _cache:
            return _cache[name]
        try:
            import torch  # noqa: F401  (the extensions link against libtorch)

            mod = importlib.import_module(f"tensorflow_distributed_learning_amd.{name}")
        except ImportError as e:  # pragma: no cover - exercised when not built
            mod = e
        _cache[name] = mod
        return mod


def hip():
    """The HIP kernel module; raises :class:`NativeExtensionMissing` if it is not built."""
    mod = _load("_C")
    if isinstance(mod, Exception):
        raise NativeExtensionMissing(
            "tensorflow_distributed_learning_amd._C (gfx950 HIP kernels) is not built or failed to load: "
            f"{mod}. Run `python build_native.py` in the repository root."
        ) from mod
    return mod


def native():
    """The C++ runtime module (rendezvous, TCP ring); raises if it is not built."""
    mod = _load("_native")
    if isinstance(mod, Exception):
        raise NativeExtensionMissing(
            "tensorflow_distributed_learning_amd._native (C++ runtime) is not built or failed to load: "
            f"{mod}. Run `python build_native.py` in the repository root."
        ) from mod
    return mod


def hip_available() -> bool:
    return not isinstance(_load("_C"), Exception)


def native_available() -> bool:
    return not isinstance(_load("_native"), Exception)


def loaded_paths() -> dict:
    out = {}
    for n in ("_C", "_native"):
        m = _cache.get(n)
        if m is not None and not isinstance(m, Exception):
            out[n] = os.path.abspath(m.__file__)
    return out
