#!/bin/bash
# Round 4: dma1 default for long reductions -- conv tests, then the ResNet-50 bench + steady-state breakdown.
set -o pipefail
O=gpurun_out/r4dma1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_conv_v2_gpu.py tests/test_slab_grad_gpu.py tests/test_bn_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
bash scripts/gpu_resnet_window.sh rnw_dma1b
