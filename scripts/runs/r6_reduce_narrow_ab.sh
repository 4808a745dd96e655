#!/bin/bash
# few-slice f32 split-K reduce issuing only 4 / 8 loads when the slices fit vs 16 clamped loads: f32 conv /
# fused-pair / fit tests, then the generic bench interleaved (TDL_F32_REDUCE_NARROW=1 default vs 0).  Usage: OUTDIR
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6narrow}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_conv_f32_gpu.py tests/test_conv_pool_f32_gpu.py tests/test_fit_gpu.py tests/test_generic_device_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
for r in 1 2 3; do
for arm in 1 0; do
  TDL_F32_REDUCE_NARROW=$arm timeout -k 10 300 python bench.py --engine generic --steps 200 --warmup 25 > $O/w${arm}_$r.json 2> $O/w${arm}_$r.err || { tail -20 $O/w${arm}_$r.err; exit 1; }
  echo "narrow=$arm $r $(grep -o '"ms_per_step": [0-9.]*' $O/w${arm}_$r.json)"
done
done
