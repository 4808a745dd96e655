#!/bin/bash
# exchange-in-finalize without the G stores (trainer path): exchange / bench / fit GPU tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5xnog
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_mnist_exchange_gpu.py tests/test_bench_gpu.py tests/test_mnist_fused_gpu.py tests/test_fit_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error" $O/tests.log | tail -20; tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
