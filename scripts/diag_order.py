"""In-process order dependence of the fused-BN comparison (diagnostic)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from diag_bnfuse import run, worst  # noqa: E402
from tensorflow_distributed_learning_amd.parallel import values as V  # noqa: E402

seq = sys.argv[1].split(",")
flags = {"F": (False, False, False), "T": (True, True, True), "O": (True, False, False)}
ms = []
for s in seq:
    print(s, "CAST_ACCUMULATE", V.CAST_ACCUMULATE, "TAPE_DEPTH", getattr(V, "TAPE_DEPTH", None), flush=True)
    ms.append(run(*flags[s], 2))
for i in range(1, len(ms)):
    print(seq[i], "vs", seq[0], worst(ms[i], ms[0]), flush=True)
