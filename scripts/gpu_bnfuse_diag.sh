#!/bin/bash
set -o pipefail
O=gpurun_out/bnfuse
mkdir -p $O
for m in F T S2 SC; do
  timeout -k 10 120 python -u scripts/diag_bnfuse2.py $m $O/w_$m.npz > $O/d_$m.log 2>&1 || { tail -5 $O/d_$m.log; exit 1; }
  AMD_SERIALIZE_KERNEL=3 timeout -k 10 120 python -u scripts/diag_bnfuse2.py $m $O/w_${m}_ser.npz > $O/d_${m}_ser.log 2>&1 || { tail -5 $O/d_${m}_ser.log; exit 1; }
done
python - <<'PY'
import numpy as np
O = "gpurun_out/bnfuse"
ref = np.load(f"{O}/w_F.npz")
for m in ["F_ser", "T", "T_ser", "S2", "S2_ser", "SC", "SC_ser"]:
    d = np.load(f"{O}/w_{m}.npz")
    w = max(float(np.abs(d[k] - ref[k]).max()) / max(float(np.abs(ref[k]).max()), 1e-3) for k in ref.files)
    print(m, "worst rel diff vs F:", round(w, 5))
PY
