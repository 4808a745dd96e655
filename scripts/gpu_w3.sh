#!/bin/bash
set -o pipefail
O=gpurun_out/w3
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_conv_gpu.py -k "wgrad3x3" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 200 python -u - > $O/time.log 2>&1 <<'PY'
import torch
from tensorflow_distributed_learning_amd.ops import hip
from tensorflow_distributed_learning_amd.ops.conv import _time, _miopen_bwd
C = hip()
x = torch.randn(256, 56, 56, 64, device="cuda").bfloat16(); dy = torch.randn(256, 56, 56, 64, device="cuda").bfloat16()
w = torch.zeros(64, 64, 3, 3, device="cuda", dtype=torch.bfloat16)
t_mi = _time(lambda: _miopen_bwd(dy.permute(0, 3, 1, 2), x.permute(0, 3, 1, 2), w, [1, 1], [1, 1], [False, True, False]))
res = {"miopen_ms": t_mi}
for rows in (0, 14, 28, 56, 112):
    C.conv_wgrad3x3_set_rows(rows)
    res[f"row_kernel_rows{rows}_ms"] = _time(lambda: C.conv_wgrad(x, dy, 3, 3, 1, 1, 1, 1, plan=[0, 0, 0]))
C.conv_wgrad3x3_set_rows(0)
p = C.conv_wgrad_plans(list(x.shape), list(dy.shape), 3, 3, 1, 1, 1, 1, 3)[1]
res["splitk_best_model_ms"] = _time(lambda: C.conv_wgrad(x, dy, 3, 3, 1, 1, 1, 1, plan=[p[0], p[1], p[3]]))
print(res)
PY
cat $O/time.log | tail -1
scripts/gpu_resnet_window.sh rn_r3d
