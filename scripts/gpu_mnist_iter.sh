#!/bin/bash
# GPU-box routine for MNIST kernel iterations: numerics tests, phase stamps, microbench, bench,
# kernel-trace stats.  Usage: scripts/gpu_mnist_iter.sh TAG
set -o pipefail
TAG=${1:-iter}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_mnist_fused_gpu.py tests/test_fit_gpu.py} -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 \
  || { echo "TESTS FAILED"; tail -60 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 120 python scripts/stamps_mnist.py > $OUT/stamps.log 2>&1 || { echo "STAMPS FAILED"; tail -20 $OUT/stamps.log; exit 1; }
cat $OUT/stamps.log
timeout -k 10 200 python scripts/microbench_mnist.py > $OUT/mb.log 2>&1 || { echo "MB FAILED"; tail -20 $OUT/mb.log; exit 1; }
grep -E "^b=|stage" $OUT/mb.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench_k20.log 2>&1 || { echo "BENCH FAILED"; tail -20 $OUT/bench_k20.log; exit 1; }
tail -1 $OUT/bench_k20.log
timeout -k 10 200 python bench.py > $OUT/bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 200 --warmup 20 > $OUT/prof.log 2>&1 || { echo "PROF FAILED"; tail -20 $OUT/prof.log; exit 1; }
python scripts/prof_summary.py $OUT/prof/run_kernel_stats.csv 8
