"""Collective implementation selection (README.md:21-29, tf_dist_example.py:12).

TF offers ``CollectiveCommunication.{AUTO, RING, NCCL}`` (TF 2.0-2.3 spelling, used by the
reference) and ``CommunicationImplementation`` + ``CommunicationOptions`` (TF >= 2.4).  Both are
accepted.  Mapping on this framework:

* ``NCCL`` -> RCCL over xGMI through ``torch.distributed`` (backend ``"nccl"``); GPU replicas only.
* ``RING`` -> the native C++ TCP ring (csrc/native/ring.cpp); GPU tensors are staged via host.
* ``AUTO`` -> RCCL when every replica is a GPU, otherwise the native ring (gloo if the native
  runtime is unavailable).
"""
from __future__ import annotations

import enum
import os
from dataclasses import dataclass
from typing import Optional


def default_timeout() -> float:
    """Seconds a collective may wait for its peers before the job fails (process-group timeout,
    the xGMI kernels' bounded waits, the progress watchdog's base threshold).  TF's collectives wait
    for ever; a synchronous job whose peer is live but out of step should end in minutes, not the 30
    of torch's default -- but a healthy job must never hit it (a slow first step, a long execution, a
    chief-only checkpoint), hence 10 minutes.  ``TDL_COLLECTIVE_TIMEOUT`` overrides;
    ``CommunicationOptions.timeout_seconds`` overrides per strategy."""
    return float(os.environ.get("TDL_COLLECTIVE_TIMEOUT", "600"))


def collective_timeout(opts) -> float:
    t = getattr(opts, "timeout_seconds", None)
    return float(t) if t else default_timeout()


class CommunicationImplementation(enum.Enum):
    AUTO = "AUTO"
    RING = "RING"
    NCCL = "NCCL"


# TF 2.0-2.3 name used by tf_dist_example.py:12
CollectiveCommunication = CommunicationImplementation


@dataclass
class CommunicationOptions:
    """tf.distribute.experimental.CommunicationOptions."""

    bytes_per_pack: int = 0
    timeout_seconds: Optional[float] = None
    implementation: CommunicationImplementation = CommunicationImplementation.AUTO
    # extension (not in TF): dtype of the gradient on the wire; "bfloat16" halves the all-reduce
    # bytes of an f32 gradient (cast before, cast back after; summation error of bf16)
    all_reduce_dtype: Optional[str] = None

    def __post_init__(self):
        if isinstance(self.implementation, str):
            self.implementation = CommunicationImplementation(self.implementation.upper())
        if self.bytes_per_pack < 0:
            raise ValueError("bytes_per_pack must be >= 0")
        if self.all_reduce_dtype not in (None, "float32", "bfloat16", "float16"):
            raise ValueError(f"all_reduce_dtype must be float32, bfloat16 or float16, got {self.all_reduce_dtype!r}")


def normalize_options(communication=None, communication_options=None) -> CommunicationOptions:
    if communication_options is not None and communication is not None:
        raise ValueError("pass either `communication` or `communication_options`, not both")
    if communication_options is not None:
        if isinstance(communication_options, CommunicationImplementation):
            return CommunicationOptions(implementation=communication_options)
        return communication_options
    if communication is None:
        return CommunicationOptions()
    if isinstance(communication, CommunicationOptions):
        return communication
    if isinstance(communication, str):
        communication = CommunicationImplementation(communication.upper())
    return CommunicationOptions(implementation=communication)
