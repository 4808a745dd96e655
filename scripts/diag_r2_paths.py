#!/usr/bin/env python3
"""Diagnostics: the fused MNIST engine at R=2 (two replica processes sharing one GPU) over each
communicator path, compared with R=1 on the same global batch and with each other.

    python scripts/diag_r2_paths.py OUTDIR
"""
import json
import os
import subprocess
import sys
import textwrap

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.test_multiproc_gpu import BODY  # noqa: E402


def run(out, tag, n, comm, extra=None):
    d = os.path.join(out, tag)
    os.makedirs(d, exist_ok=True)
    s = os.path.join(d, "job.py")
    open(s, "w").write(textwrap.dedent(BODY))
    env = dict(os.environ, PYTHONPATH=ROOT, TDL_SHARE_GPU="1", JOB_COMM=comm, **(extra or {}))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "TF_CONFIG"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "tensorflow_distributed_learning_amd.launch", "--nproc-per-node", str(n),
                        s, d], env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    if r.returncode != 0:
        print(tag, "FAILED", r.stdout[-1500:], r.stderr[-2500:], flush=True)
        return None
    w = np.load(os.path.join(d, f"w0_{n}.npy"))
    meta = json.load(open(os.path.join(d, f"r0_{n}.json")))
    print(f"{tag}: algo={meta['algorithm']} graph={meta['graph']} loss={meta['loss']}", flush=True)
    return w


def main():
    out = sys.argv[1]
    ws = {}
    ws["r1"] = run(out, "r1", 1, "")
    ws["ring"] = run(out, "ring", 2, "RING")
    ws["auto"] = run(out, "auto", 2, "")
    ws["auto_noover"] = run(out, "auto_noover", 2, "", {"TDL_OVERLAP_ALLREDUCE": "0"})
    ws["auto_nocap"] = run(out, "auto_nocap", 2, "", {"TDL_CAPTURE_ALLREDUCE": "0"})
    ws["nccl"] = run(out, "nccl", 2, "NCCL")
    ref = ws["ring"]
    names = ["w1", "b1", "w2", "b2", "w3", "b3", "w4", "b4"]
    sizes = [288, 32, 18432, 64, 204800, 128, 1280, 10]
    for k, w in ws.items():
        if w is None or ref is None:
            continue
        diff = np.abs(w - ref)
        parts, o = [], 0
        for nm, sz in zip(names, sizes):
            parts.append(f"{nm}={diff[o:o + sz].max():.2e}")
            o += sz
        print(f"{k} vs ring: max {diff.max():.3e} identical={np.array_equal(w, ref)}  " + " ".join(parts), flush=True)


if __name__ == "__main__":
    main()
