#!/bin/bash
# no-G-store finalize adopted on the single-replica SGD path: MNIST GPU tests + driver-shaped benches
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5nogadopt
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_mnist_fused_gpu.py tests/test_fit_gpu.py tests/test_eval_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error" $O/tests.log | tail -20; tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for r in 1 2 3; do
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_$r.log 2>&1 || { echo BENCH FAILED; tail -20 $O/b20_$r.log; exit 1; }
grep -o '"value": [0-9.]*.*"ms_per_step": [0-9.]*' $O/b20_$r.log
done
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo BENCH FAILED; tail -20 $O/bench.log; exit 1; }
grep -o '"value": [0-9.]*.*"ms_per_step": [0-9.]*' $O/bench.log
