#!/bin/bash
# A/B: the fused kernel's conv1-wgrad partials as 16-B write-through stores (variant 8) vs 4-B plain; numerics test of the variant
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5p1wt
mkdir -p $O
TDL_MNIST_VARIANT=8 timeout -k 10 600 python -u -m pytest tests/test_mnist_fused_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error" $O/tests.log | tail -20; tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
bash scripts/runs/ab_arms.sh r5p1wt_ab 3 v0=.:0 p1wt=.:8
