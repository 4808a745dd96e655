#!/bin/bash
# MNIST fused-step GPU routine: its tests, bench (driver settings and long), phase stamps, kernel stats.
# Usage: scripts/gpu_mnist_check.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-mnist}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_mnist_fused_gpu.py tests/test_multiproc_gpu.py tests/test_bench_gpu.py tests/test_fit_gpu.py \
  > $OUT/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench20.log 2>&1 || { echo BENCH FAILED; tail -20 $OUT/bench20.log; exit 1; }
tail -1 $OUT/bench20.log
timeout -k 10 200 python bench.py --gpus 1 --steps 1000 --warmup 100 > $OUT/bench1000.log 2>&1 || { echo BENCH FAILED; tail -20 $OUT/bench1000.log; exit 1; }
tail -1 $OUT/bench1000.log | cut -c1-200
timeout -k 10 120 python scripts/stamps_mnist.py > $OUT/stamps.txt 2>&1 || { echo STAMPS FAILED; tail -20 $OUT/stamps.txt; exit 1; }
cat $OUT/stamps.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 200 --warmup 20 > $OUT/prof.log 2>&1 || { echo "PROF FAILED"; tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec head -8 {} \;
if [ -n "$RESNET" ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_slab_grad_gpu.py tests/test_conv_gpu.py tests/test_bn_gpu.py > $OUT/rtests.log 2>&1 || { echo "RTESTS FAILED"; tail -40 $OUT/rtests.log; exit 1; }
  tail -1 $OUT/rtests.log
  timeout -k 10 300 python scripts/bench_resnet50.py > $OUT/resnet.log 2>&1 || { echo RESNET FAILED; tail -20 $OUT/resnet.log; exit 1; }
  tail -1 $OUT/resnet.log | cut -c1-300
fi
