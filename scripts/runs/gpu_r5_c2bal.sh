#!/bin/bash
# dW3 finalize tasks with quad-transposed 16-B operand loads / stores: MNIST GPU tests, then same-box A/B vs the snapshot ab/base8
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5c2bal
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_mnist_fused_gpu.py tests/test_fit_gpu.py tests/test_mnist_exchange_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error" $O/tests.log | tail -20; tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
bash scripts/runs/ab_arms.sh r5c2bal_ab 3 base=ab/base8:0 qt=.:0
