#!/bin/bash
# K=20 / K=1000 bench after the learning-rate fill skip + the trainer GPU tests that read lr_dev
set -o pipefail
O=gpurun_out/lrab
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fit_gpu.py tests/test_mnist_fused_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20_$i.log 2>&1 || { echo BENCH FAILED; tail -20 $O/bench20_$i.log; exit 1; }
  grep -h "timed region" $O/bench20_$i.log; tail -1 $O/bench20_$i.log | cut -c1-200
done
timeout -k 10 200 python bench.py --gpus 1 --steps 1000 --warmup 20 > $O/bench1000.log 2>&1 || { echo BENCH1000 FAILED; exit 1; }
tail -1 $O/bench1000.log | cut -c1-200
