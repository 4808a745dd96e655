#!/bin/bash
# GPU-box routine: tests, microbench, kernel-trace profile.  Usage: scripts/gpu_check.sh TAG
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python scripts/microbench_mnist.py > $OUT/mb.log 2>&1 || { echo "MB FAILED"; tail -20 $OUT/mb.log; exit 1; }
grep -E "^b=|stage" $OUT/mb.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python scripts/microbench_mnist.py --iters 20 > $OUT/prof.log 2>&1 || { echo "PROF FAILED"; tail -20 $OUT/prof.log; exit 1; }
python scripts/prof_summary.py $OUT/prof/run_kernel_stats.csv
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
