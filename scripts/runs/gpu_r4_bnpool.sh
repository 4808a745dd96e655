#!/bin/bash
# Round 4: BN -> ReLU -> max-pool fusion (the ResNet stem) -- tests, then the ResNet-50 window.
set -o pipefail
O=gpurun_out/r4bnpool
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_bn_gpu.py tests/test_stem_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
bash scripts/gpu_resnet_window.sh rnw_bnpool2
