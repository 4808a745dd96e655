"""Which GPU kernels a piece of training code really launches (hand-written vs library).

The framework's hot path is meant to be hand-written gfx950 kernels (namespace ``tdl``, csrc/kernels)
plus PyTorch's own elementwise / reduction / pooling kernels (``at::native``) -- never a vendor
library's GEMM or convolution (hipBLASLt / rocBLAS / Tensile ``Cijk_*``, MIOpen, composable_kernel
instances).  :func:`audit` runs a callable under the PyTorch profiler (roctracer device activity),
demangles nothing, and sorts every device kernel name into ``tdl`` / ``torch`` / ``library`` /
``other``.  Kernels launched from a replayed hipGraph may not be reported by the tracer, so callers
audit eager runs (``TDL_GRAPH=0`` / ``TDL_GRAPH_STEP=0``).
"""
from __future__ import annotations

import re
from collections import Counter
from typing import Callable, Dict

LIBRARY_PATTERNS = re.compile(
    r"Cijk_|rocblas|hipblaslt|hipblas|tensile|miopen|MIOpen|naive_conv|igemm|gridwise_|device_gemm|"
    r"DeviceGemm|DeviceConv|ck::|batched_transpose|SubTensorOpWithScalar|Op2dTensorGeneric|"
    r"MIOpenBatchNorm|MIOpenConv|conv2d_grouped|winograd|sp3AsmConv|gcnAsmConv|conv1x1u|implicitgemm",
    re.IGNORECASE)


def classify(name: str) -> str:
    if "tdl::" in name or name.startswith("tdl_") or re.search(r"\bk_(fwd|finalize|xgmi|sgd|adam)", name):
        return "tdl"
    if LIBRARY_PATTERNS.search(name):
        return "library"
    if ("at::native" in name or "at::" in name or "c10::" in name or "rocprim" in name or "hipcub" in name or
            "softmax_warp_" in name):  # (PyTorch's persistent softmax kernels live in an anonymous namespace)
        return "torch"
    return "other"


def audit(fn: Callable[[], object], sync: bool = True) -> Dict[str, Counter]:
    """Run ``fn`` under the profiler; {category: Counter(kernel name -> launches)}."""
    import torch
    from torch.profiler import ProfilerActivity, profile

    if sync:
        torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        fn()
        if sync:
            torch.cuda.synchronize()
    out: Dict[str, Counter] = {"tdl": Counter(), "torch": Counter(), "library": Counter(), "other": Counter()}
    for ev in prof.events():
        dt = getattr(ev, "device_type", None)
        if dt is None or "CUDA" not in str(dt):
            continue
        name = ev.name
        if name.startswith(("Memcpy", "Memset", "hipMemcpy", "hipMemset", "[memory]")) or "Memcpy" in name[:12]:
            continue
        out[classify(name)][name] += 1
    return out
