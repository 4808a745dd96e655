#!/bin/bash
# Round 5 MNIST v1: W3 linear prefetch, dC2 scatter, VALU db2, finalize SGD-operand prefetch
set -o pipefail
O=gpurun_out/r5v1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mnist_fused_gpu.py tests/test_head_gpu.py tests/test_eval_gpu.py tests/test_mnist_exchange_gpu.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20_$i.log 2>&1 || { echo BENCH FAILED; tail -20 $O/bench20_$i.log; exit 1; }
tail -1 $O/bench20_$i.log | cut -c1-200
done
timeout -k 10 200 python bench.py --gpus 1 --steps 1000 --warmup 20 > $O/bench1000.log 2>&1 || { echo BENCH1000 FAILED; tail -20 $O/bench1000.log; exit 1; }
tail -1 $O/bench1000.log | cut -c1-200
timeout -k 10 200 python scripts/stamps_step.py > $O/step.log 2>&1 || { echo STEP FAILED; tail -20 $O/step.log; exit 1; }
cat $O/step.log
timeout -k 10 200 python scripts/stamps_mnist.py > $O/phases.log 2>&1 || { echo PH FAILED; tail -20 $O/phases.log; exit 1; }
cat $O/phases.log
echo done
