#!/bin/bash
# MNIST round harness: fused-engine GPU tests (+ $TESTS), fused-kernel phase stamps, then the same-box
# interleaved A/B of ab_arms.sh over $ARMS (name=dir:variant ...), $REPS reps, into gpurun_out/$OUT and /$AB.
set -o pipefail
O=gpurun_out/${OUT:-r5v6}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mnist_fused_gpu.py ${TESTS:-} > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python scripts/stamps_mnist.py > $O/phases.log 2>&1 || { echo PH FAILED; tail -20 $O/phases.log; exit 1; }
grep -v amdgpu $O/phases.log | head -5
bash scripts/runs/ab_arms.sh ${AB:-r5v6ab} ${REPS:-2} ${ARMS:-base=ab/base:0 cur=.:0}
