#!/bin/bash
# XCD-aware (image, quarter) placement of k_fwd_conv (TDL_MNIST_VARIANT bit 8) vs the default map:
# numerics under the variant, then a same-box interleaved A/B (K=1000 and K=20) and step stamps.
set -o pipefail
O=gpurun_out/${1:-r6xcd}
mkdir -p $O
export TMPDIR=/tmp
TDL_MNIST_VARIANT=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mnist_fused_gpu.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/runs/ab_arms.sh ${1:-r6xcd}/ab ${REPS:-3} cur=.:0 xcd=.:8
