#!/bin/bash
# Generic engine: f32 tests + the reference-CNN bench (3 interleaved repeats of the three variants) +
# rocprofv3 kernel stats.  Usage: OUTDIR
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6gab}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_conv_f32_gpu.py tests/test_generic_device_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
for r in 1 2; do
for v in reference same dropout; do
  timeout -k 10 300 python bench.py --engine generic --variant $v --steps 200 --warmup 25 > $O/generic_${v}_$r.json 2> $O/generic_${v}_$r.err || { tail -20 $O/generic_${v}_$r.err; exit 1; }
  echo "$v $r $(grep -o '"ms_per_step": [0-9.]*' $O/generic_${v}_$r.json)"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --engine generic --steps 100 --warmup 10 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/prof_summary.py $O/prof/run_kernel_stats.csv > $O/prof_summary.txt 2>&1; head -18 $O/prof_summary.txt
