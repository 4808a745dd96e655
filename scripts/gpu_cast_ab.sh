#!/bin/bash
# GPU-box: generic-engine GPU tests + ResNet-50 A/B of the fused bf16 weight-gradient accumulation
# (TDL_CAST_ACCUMULATE=1, default) against cast + AccumulateGrad (=0), then a kernel-stats profile.
set -o pipefail
OUT=gpurun_out/cast_ab
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fit_gpu.py tests/test_comm_capture_gpu.py tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
TDL_CAST_ACCUMULATE=0 timeout -k 10 400 python scripts/bench_resnet50.py > $OUT/bench_off.log 2>&1 || { echo "BENCH OFF FAILED"; tail -30 $OUT/bench_off.log; exit 1; }
tail -1 $OUT/bench_off.log
TDL_CAST_ACCUMULATE=1 timeout -k 10 400 python scripts/bench_resnet50.py > $OUT/bench_on.log 2>&1 || { echo "BENCH ON FAILED"; tail -30 $OUT/bench_on.log; exit 1; }
tail -1 $OUT/bench_on.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python scripts/bench_resnet50.py --steps 5 --warmup 3 > $OUT/prof.log 2>&1 || { echo "PROF FAILED"; tail -20 $OUT/prof.log; exit 1; }
python scripts/prof_summary.py $OUT/prof/run_kernel_stats.csv 30 > $OUT/prof_summary.txt
head -40 $OUT/prof_summary.txt
