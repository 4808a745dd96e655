#!/bin/bash
# Round 4: the test order that exposed the auto-mode wgrad plan leaking into a forced-hip run
set -o pipefail
O=gpurun_out/r4order
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_bn_gpu.py tests/test_stem_gpu.py tests/test_slab_grad_gpu.py -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
