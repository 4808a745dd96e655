#!/bin/bash
set -o pipefail
O=gpurun_out/bnfuse
mkdir -p $O
for v in 1 2; do
TDL_DEBUG_POISON=$v timeout -k 10 120 python -u scripts/diag_bnfuse2.py F $O/w_P$v.npz > $O/d_P$v.log 2>&1 || { tail -20 $O/d_P$v.log; exit 1; }
done
timeout -k 10 120 python -u scripts/diag_bnfuse2.py F $O/w_F.npz > $O/d_F.log 2>&1 || exit 1
python - <<'PY'
import numpy as np
O = "gpurun_out/bnfuse"
ref = np.load(f"{O}/w_F.npz")
for m in ("P1", "P2"):
    d = np.load(f"{O}/w_{m}.npz")
    bad = [k for k in ref.files if not np.isfinite(d[k]).all()]
    print(m, "non-finite weights:", len(bad), "of", len(ref.files), bad[:5])
    print(m, "vs F", max(float(np.nan_to_num(np.abs(d[k] - ref[k]), nan=9)).max() / max(float(np.abs(ref[k]).max()), 1e-3) for k in ref.files))
PY
