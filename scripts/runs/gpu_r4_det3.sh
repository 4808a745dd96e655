#!/bin/bash
# Round 4: the fused-config (T) async vs HIP_LAUNCH_BLOCKING=1 checksums (a 1-ulp difference seen once
# in tests/test_slab_grad_gpu.py), then the BN -> ReLU -> max-pool fusion tests and the ResNet window.
set -o pipefail
O=gpurun_out/r4det3
mkdir -p $O
export TMPDIR=/tmp
for run in a1 a2; do
  timeout -k 10 200 python -u scripts/diag_checksums.py run T $O/T_$run.json 2 > $O/T_$run.log 2>&1 || { echo "RUN $run FAILED"; tail -30 $O/T_$run.log; exit 1; }
done
HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 python -u scripts/diag_checksums.py run T $O/T_b1.json 2 > $O/T_b1.log 2>&1 || { echo "RUN b1 FAILED"; tail -30 $O/T_b1.log; exit 1; }
for p in "a1 a2" "a1 b1"; do
  set -- $p
  echo "== T $1 vs $2"
  python scripts/diag_checksums.py compare $O/T_$1.json $O/T_$2.json | head -20 || true
done
timeout -k 10 400 python -u -m pytest tests/test_bn_gpu.py tests/test_stem_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
bash scripts/gpu_resnet_window.sh rnw_bnpool
