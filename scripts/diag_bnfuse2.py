"""Run the projection-shortcut test model once (fused or not) and save its weights (diagnostic)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from diag_bnfuse import run  # noqa: E402

mode, out = sys.argv[1], sys.argv[2]
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
flags = {"F": (False, False, False), "T": (True, True, True), "S2": (True, True, False), "SC": (True, False, True)}[mode]
from tensorflow_distributed_learning_amd.ops import batchnorm as B  # noqa: E402

m = run(*flags, steps)
np.savez(out, *m.get_weights())
print("fused_modes", B.FUSED_BWD_MODES, flush=True)
print("saved", out, flush=True)
