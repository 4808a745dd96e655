#!/bin/bash
# adopted write-through dW3 W stores: MNIST GPU tests; then A/B of write-through P2 stores in the fused kernel (variant 8)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5p2wt
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_mnist_fused_gpu.py tests/test_fit_gpu.py tests/test_mnist_exchange_gpu.py tests/test_eval_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error" $O/tests.log | tail -20; tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
bash scripts/runs/ab_arms.sh r5p2wt_ab 3 v0=.:0 p2wt=.:8
