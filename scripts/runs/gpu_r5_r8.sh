#!/bin/bash
# Round 5: R = 8 on the one-GPU box (xGMI IPC all-reduce, exchange-in-finalize with a capped grid,
# bench --gpus 8 shared) + the graph K sweep of the MNIST step
set -o pipefail
O=gpurun_out/r5r8
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python scripts/mnist_graph_k_sweep.py > $O/ksweep.log 2>&1 || { echo KSWEEP FAILED; tail -20 $O/ksweep.log; exit 1; }
cat $O/ksweep.log | grep -v amdgpu
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_xgmi_gpu.py tests/test_mnist_exchange_gpu.py tests/test_bench_gpu.py > $O/tests.log 2>&1 || { echo TESTS FAILED; grep -E "PASS|FAIL|Error|error" $O/tests.log | tail -30; tail -30 $O/tests.log; exit 1; }
grep -E "PASS|FAIL" $O/tests.log | tail -30
echo done
