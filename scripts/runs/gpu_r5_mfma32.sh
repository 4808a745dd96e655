#!/bin/bash
# 32x32x16 vs 16x16x32 MFMA form of the dma1 conv main loop: correctness tests + same-box A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5mf32
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_gpu.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 500 python scripts/bench_conv_mfma32.py > $O/ab.log 2>&1 || { echo AB FAILED; tail -20 $O/ab.log; exit 1; }
grep "{" $O/ab.log
