#!/bin/bash
# F vs F under kernel serialization, after the pageable non_blocking copy fix
set -o pipefail
O=gpurun_out/bnfuse
mkdir -p $O
timeout -k 10 120 python -u scripts/diag_bnfuse2.py F $O/w_F.npz > $O/d_F.log 2>&1 || exit 1
AMD_SERIALIZE_KERNEL=3 timeout -k 10 120 python -u scripts/diag_bnfuse2.py F $O/w_F_ser.npz > $O/d_F_ser.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/diag_order.py T,F > $O/o_TF.log 2>&1; grep "vs" $O/o_TF.log
python - <<'PY'
import numpy as np
O = "gpurun_out/bnfuse"
ref = np.load(f"{O}/w_F.npz")
d = np.load(f"{O}/w_F_ser.npz")
print("F_ser vs F", max(float(np.abs(d[k] - ref[k]).max()) / max(float(np.abs(ref[k]).max()), 1e-3) for k in ref.files))
PY
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_slab_grad_gpu.py > $O/ts.log 2>&1; tail -1 $O/ts.log
