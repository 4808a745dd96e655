#!/bin/bash
# Fused Conv2D -> MaxPooling2D forward on the generic f32 path: tests, then the generic-engine bench
# (fused pair vs TDL_FUSE_CONV_POOL=0, interleaved) and rocprofv3 kernel stats.  Usage: OUTDIR
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6cpool}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_conv_pool_f32_gpu.py tests/test_conv_f32_gpu.py tests/test_generic_device_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
for r in 1 2; do
for f in 1 0; do
for v in reference same dropout; do
  TDL_FUSE_CONV_POOL=$f timeout -k 10 300 python bench.py --engine generic --variant $v --steps 200 --warmup 25 > $O/g_${v}_f${f}_$r.json 2> $O/g_${v}_f${f}_$r.err || { tail -20 $O/g_${v}_f${f}_$r.err; exit 1; }
  echo "fuse=$f $v $r $(grep -o '"ms_per_step": [0-9.]*' $O/g_${v}_f${f}_$r.json)"
done
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --engine generic --steps 100 --warmup 10 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/prof_summary.py $O/prof/run_kernel_stats.csv > $O/prof_summary.txt 2>&1; head -24 $O/prof_summary.txt
