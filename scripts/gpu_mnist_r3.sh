#!/bin/bash
# Round-3 MNIST iteration: fused-kernel tests, bench (driver K/W and K=1000), kernel-trace stats.
# Usage: scripts/gpu_mnist_r3.sh TAG [extra pytest files...]
set -o pipefail
TAG=${1:-mnist}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_mnist_fused_gpu.py "$@" > $OUT/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench20.log 2>&1 || { echo BENCH FAILED; tail -20 $OUT/bench20.log; exit 1; }
tail -1 $OUT/bench20.log | cut -c1-200
timeout -k 10 200 python bench.py --gpus 1 --steps 1000 --warmup 20 > $OUT/bench1000.log 2>&1 || { echo BENCH FAILED; tail -20 $OUT/bench1000.log; exit 1; }
tail -1 $OUT/bench1000.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 200 --warmup 20 > $OUT/prof.log 2>&1 || { echo "PROF FAILED"; tail -20 $OUT/prof.log; exit 1; }
python scripts/prof_summary.py $(find $OUT/prof -name "*kernel_stats.csv" | head -1)
