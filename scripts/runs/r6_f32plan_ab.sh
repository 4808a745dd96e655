#!/bin/bash
# Generic engine: f32 GEMM split-K plan A/B (TDL_F32_SPLIT=kmin,cap): 128,256 (round-5 plan) vs 64,1024,
# interleaved, plus the f32 kernel / generic-device tests.  Usage: OUTDIR
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6plan}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_conv_f32_gpu.py tests/test_generic_device_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for p in 128,256 64,1024 32,1024; do
    TDL_F32_SPLIT=$p timeout -k 10 300 python bench.py --engine generic --steps 200 --warmup 25 > $O/g_${p/,/_}_$r.json 2> $O/g_${p/,/_}_$r.err || { tail -5 $O/g_${p/,/_}_$r.err; exit 1; }
    echo "$p rep$r $(grep -o '"ms_per_step": [0-9.]*' $O/g_${p/,/_}_$r.json)"
  done
done
