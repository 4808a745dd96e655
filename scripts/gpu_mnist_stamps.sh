#!/bin/bash
# MNIST kernel iteration: fused tests, phase stamps, bench (K=20 / K=1000), kernel stats.  Usage: TAG
set -o pipefail
OUT=gpurun_out/${1:-stamps}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mnist_fused_gpu.py tests/test_mnist_exchange_gpu.py > $OUT/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 120 python scripts/stamps_mnist.py > $OUT/stamps.txt 2>&1 || { echo STAMPS FAILED; tail -20 $OUT/stamps.txt; exit 1; }
grep -v amdgpu.ids $OUT/stamps.txt
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench20.log 2>&1 || { echo BENCH FAILED; tail -20 $OUT/bench20.log; exit 1; }
tail -1 $OUT/bench20.log | cut -c1-190
timeout -k 10 200 python bench.py --gpus 1 --steps 1000 --warmup 20 > $OUT/bench1000.log 2>&1 || { echo BENCH FAILED; tail -20 $OUT/bench1000.log; exit 1; }
tail -1 $OUT/bench1000.log | cut -c1-190
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 200 --warmup 20 > $OUT/prof.log 2>&1 || { echo "PROF FAILED"; tail -20 $OUT/prof.log; exit 1; }
python scripts/prof_summary.py $(find $OUT/prof -name "*kernel_stats.csv" | head -1) 4
