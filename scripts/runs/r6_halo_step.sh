#!/bin/bash
# Halo conv: tests, per-shape A/B, then ResNet-50 b=256 step A/B (TDL_CONV_HALO=0 vs the default
# selection), interleaved.  Usage: OUTDIR
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6halostep}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_conv_halo_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
timeout -k 10 300 python -u scripts/bench_conv_halo.py 256 > $O/bench.log 2>&1 || { echo BENCH FAILED; tail -20 $O/bench.log; exit 1; }
grep -o '"dir": "[a-z]*", "shape": \[[0-9, ]*\], "default_us": [0-9.]*, "halo_us": [0-9.]*' $O/bench.log
for r in 1 2; do
  for h in 0 2; do
    TDL_CONV_HALO=$h timeout -k 10 400 python -u scripts/bench_resnet50.py > $O/rn_h${h}_$r.log 2>&1 || { echo RN FAILED; tail -20 $O/rn_h${h}_$r.log; exit 1; }
    echo "halo=$h run $r: $(grep -o '"value": [0-9.]*' $O/rn_h${h}_$r.log | tail -1)"
  done
done
