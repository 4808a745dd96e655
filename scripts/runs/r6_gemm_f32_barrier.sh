#!/bin/bash
# f32 GEMM main loop with LDS-only barriers (no vmcnt(0) drain of the 4-deep register ring per slice):
# f32 conv / dense tests, then the generic-engine bench (reference CNN, K=200 W=25).  Usage: OUTDIR
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6gbar}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_conv_f32_gpu.py tests/test_generic_device_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
for r in 1 2; do
for v in reference same dropout; do
  timeout -k 10 300 python bench.py --engine generic --variant $v --steps 200 --warmup 25 > $O/generic_${v}_$r.json 2> $O/generic_${v}_$r.err || { tail -20 $O/generic_${v}_$r.err; exit 1; }
  echo "$v $r $(grep -o '"value": [0-9.]*' $O/generic_${v}_$r.json) $(grep -o '"ms_per_step": [0-9.]*' $O/generic_${v}_$r.json)"
done
done
