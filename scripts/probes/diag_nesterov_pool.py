"""Diagnostic: the reference CNN with Nesterov SGD (tests/test_fit_gpu.py optimizer case) on the fused
engine vs the generic engine with and without the fused Conv2D -> MaxPooling2D forward: per-tensor
fraction of weights outside (rtol 5e-3, atol 5e-4), and the loss histories."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import test_fit_gpu as T  # noqa: E402
import tensorflow_distributed_learning_amd as tdl  # noqa: E402

mk = lambda: tdl.keras.optimizers.SGD(learning_rate=0.05, momentum=0.9, nesterov=True)  # noqa: E731
runs = {}
mf, hf = T._train_opt(True, mk)
runs["fused"] = (mf.get_weights(), hf.history["loss"])
for fuse in ("1", "0"):
    os.environ["TDL_FUSE_CONV_POOL"] = fuse
    mg, hg = T._train_opt(False, mk)
    runs[f"generic_pool{fuse}"] = (mg.get_weights(), hg.history["loss"])
for k, (w, l) in runs.items():
    print(k, "loss", np.round(l, 5))
for a, b in (("fused", "generic_pool1"), ("fused", "generic_pool0"), ("generic_pool1", "generic_pool0")):
    offs = [float((~np.isclose(x, y, rtol=5e-3, atol=5e-4)).mean()) for x, y in zip(runs[a][0], runs[b][0])]
    mx = [float(np.abs(x - y).max()) for x, y in zip(runs[a][0], runs[b][0])]
    print(a, "vs", b, "off", np.round(offs, 4).tolist(), "max", np.round(mx, 5).tolist())
