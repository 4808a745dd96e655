#!/bin/bash
set -o pipefail
O=gpurun_out/bnfuse
mkdir -p $O
for m in F T; do for r in 1 2 3; do
  timeout -k 10 120 python -u scripts/diag_bnfuse2.py $m $O/w_${m}$r.npz > $O/d_${m}$r.log 2>&1 || { tail -5 $O/d_${m}$r.log; exit 1; }
done; done
python - <<'PY'
import numpy as np
O = "gpurun_out/bnfuse"
ref = np.load(f"{O}/w_F1.npz")
for m in ["F2", "F3", "T1", "T2", "T3"]:
    d = np.load(f"{O}/w_{m}.npz")
    w = max(float(np.abs(d[k] - ref[k]).max()) / max(float(np.abs(ref[k]).max()), 1e-3) for k in ref.files)
    print(m, "worst rel diff vs F1:", round(w, 5))
PY
