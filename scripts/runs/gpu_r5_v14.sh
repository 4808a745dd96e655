#!/bin/bash
# v14: f32 conv reduce / stride-1 dgrad speedups (tests + bench), MNIST rocprof kernel stats of the current build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5v14
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_f32_gpu.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python scripts/bench_conv_f32.py > $O/conv_f32.log 2>&1 || { echo CONVF32 FAILED; tail -20 $O/conv_f32.log; exit 1; }
grep "{" $O/conv_f32.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 1000 --warmup 20 > $O/prof.log 2>&1 || { echo PROF FAILED; tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs head -8
