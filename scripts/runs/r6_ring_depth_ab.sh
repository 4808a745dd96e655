#!/bin/bash
# f32 GEMM register-ring depth 6 vs 4 (two prebuilt copies of the extension under abso/, swapped between
# runs): f32 tests on the depth-6 build, then the generic bench interleaved.  Usage: OUTDIR
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6ring}
SO=tensorflow_distributed_learning_amd/_C.cpython-310-x86_64-linux-gnu.so
mkdir -p $O
cp abso/C_kd6.so $SO
timeout -k 10 600 python -u -m pytest tests/test_conv_f32_gpu.py tests/test_conv_pool_f32_gpu.py tests/test_fit_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
for r in 1 2 3; do
for arm in kd6 kd4; do
  cp abso/C_$arm.so $SO
  timeout -k 10 300 python bench.py --engine generic --steps 200 --warmup 25 > $O/${arm}_$r.json 2> $O/${arm}_$r.err || { tail -20 $O/${arm}_$r.err; exit 1; }
  echo "$arm $r $(grep -o '"ms_per_step": [0-9.]*' $O/${arm}_$r.json)"
done
done
