#!/bin/bash
# Round 5: R = 8 tests again (finalize range loop now a separate instantiation) + K sweep with lead step
set -o pipefail
O=gpurun_out/r5r8b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python scripts/mnist_graph_k_sweep.py > $O/ksweep.log 2>&1 || { echo KSWEEP FAILED; tail -20 $O/ksweep.log; exit 1; }
grep -v amdgpu $O/ksweep.log
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_mnist_exchange_gpu.py tests/test_bench_gpu.py tests/test_mnist_fused_gpu.py > $O/tests.log 2>&1 || { echo TESTS FAILED; grep -E "PASS|FAIL" $O/tests.log | tail -30; tail -30 $O/tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/tests.log | tail -40
echo done
