#!/bin/bash
# Round 4: slab weight gradients on a side stream -- bitwise tests, multi-replica check, ResNet-50 window.
set -o pipefail
O=gpurun_out/r4side
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_slab_grad_gpu.py tests/test_resnet_multireplica_gpu.py tests/test_generic_multiproc_gpu.py -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
bash scripts/gpu_resnet_window.sh rnw_side
