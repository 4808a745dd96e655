#!/bin/bash
# Generic engine on device-resident multi-step execution graphs: tests, bench (3 variants), kernel profile.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6gdev}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_conv_f32_gpu.py tests/test_generic_device_gpu.py tests/test_hot_path_kernels_gpu.py tests/test_fit_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -60 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
for v in reference same dropout; do
  timeout -k 10 300 python bench.py --engine generic --variant $v --steps 200 --warmup 25 > $O/generic_$v.json 2> $O/generic_$v.err || { tail -20 $O/generic_$v.err; exit 1; }
  tail -1 $O/generic_$v.json | cut -c1-220
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --engine generic --steps 100 --warmup 25 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/prof_summary.py $O/prof/run_kernel_stats.csv > $O/prof_summary.txt 2>&1; head -40 $O/prof_summary.txt
