#!/bin/bash
# Halo conv main loop: correctness tests, then the per-shape A/B against the default kernels
# (scripts/bench_conv_halo.py).  Usage: OUTDIR
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6halo}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_conv_halo_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
timeout -k 10 300 python -u scripts/bench_conv_halo.py 256 > $O/bench.log 2>&1 || { echo BENCH FAILED; tail -20 $O/bench.log; exit 1; }
cat $O/bench.log
