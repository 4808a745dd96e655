#!/bin/bash
# Round 4: MIOpen find-mode scoped to the trainer and off by default -- trainer tests, BN tests, ResNet bench
set -o pipefail
O=gpurun_out/r4miopen
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_slab_grad_gpu.py tests/test_bn_gpu.py tests/test_fit_gpu.py -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python scripts/bench_resnet50.py > $O/resnet.log 2>&1 || { echo RESNET FAILED; tail -20 $O/resnet.log; exit 1; }
grep metric $O/resnet.log | cut -c1-300
