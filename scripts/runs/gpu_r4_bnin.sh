#!/bin/bash
# input-side BN -> ReLU in the 1x1 conv loaders: tests, then the ResNet-50 window
set -o pipefail
O=gpurun_out/bnin
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bn_gpu.py tests/test_conv_gpu.py tests/test_slab_grad_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -2 $O/test.log
./scripts/gpu_resnet_window.sh rnw_bnin
