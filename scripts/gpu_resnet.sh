#!/bin/bash
# GPU-box: ResNet-50 bench + kernel stats.  Usage: scripts/gpu_resnet.sh TAG [extra bench args]
set -o pipefail
TAG=${1:-rn}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python scripts/bench_resnet50.py "$@" > $OUT/bench.log 2>&1 || { echo "BENCH FAILED"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python scripts/bench_resnet50.py --steps 5 --warmup 3 "$@" > $OUT/prof.log 2>&1 || { echo "PROF FAILED"; tail -20 $OUT/prof.log; exit 1; }
python scripts/prof_summary.py $OUT/prof/run_kernel_stats.csv 30
