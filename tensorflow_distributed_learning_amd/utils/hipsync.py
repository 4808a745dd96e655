"""How the host thread waits for the GPU (the HIP runtime's device schedule flag).

A short training execution ends in a host-side wait (``torch.cuda.synchronize``, a metrics read,
the end of ``fit``).  HIP's default schedule lets that thread yield / block, and waking it after
the GPU's completion signal costs microseconds that a 20-step MNIST execution (0.5 ms) feels.
``TDL_HIP_SCHEDULE=spin`` makes the waiting thread poll the completion signal instead (one CPU
core busy while it waits), ``yield`` forces the blocking form, ``auto`` the runtime heuristic.
The flag must be set before the device's context is created: the strategy applies it to its
replica's own device only, when that device is chosen (parallel/strategy.py StrategyExtended), through
the runtime's C API (no GPU work is issued).  Launchers and parents of replica processes, which never
touch a GPU, never reach it.
"""
import ctypes
import os

_FLAGS = {"auto": 0, "spin": 1, "yield": 2}
applied = None  # (mode, [per-device return codes]) once configure() ran


_done = set()


def configure(mode: str = "", devices=None) -> bool:
    """Set hipDeviceSchedule<mode> on ``devices`` (indices; default: every visible device), once
    per device and process; False if unset / unsupported."""
    global applied
    mode = (mode or os.environ.get("TDL_HIP_SCHEDULE", "")).strip().lower()
    if mode not in _FLAGS:
        return False
    try:
        lib = ctypes.CDLL("libamdhip64.so")
    except OSError:
        return False
    n = ctypes.c_int(0)
    if lib.hipGetDeviceCount(ctypes.byref(n)) != 0 or n.value == 0:
        return False
    cur = ctypes.c_int(0)
    lib.hipGetDevice(ctypes.byref(cur))
    rcs = []
    for d in (range(n.value) if devices is None else [int(i) for i in devices if 0 <= int(i) < n.value]):
        if d in _done:
            continue
        _done.add(d)
        lib.hipSetDevice(d)
        rcs.append(int(lib.hipSetDeviceFlags(_FLAGS[mode])))
    lib.hipSetDevice(cur.value)
    applied = (mode, rcs)
    return all(rc == 0 for rc in rcs)
