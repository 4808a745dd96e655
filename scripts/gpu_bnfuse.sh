#!/bin/bash
# GPU box: BN-backward fusion tests (projection shortcut part2, stride-2 epilogue), the conv/BN/slab
# GPU tests, BN pass listing, then ResNet-50 bench + steady-state breakdown.
set -o pipefail
O=gpurun_out/bnfuse
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_slab_grad_gpu.py tests/test_conv_gpu.py tests/test_bn_gpu.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
TDL_BN_DEBUG=1 timeout -k 10 300 python scripts/bench_resnet50.py --steps 2 --warmup 2 > $O/bndebug.log 2>&1 || { echo "BNDEBUG FAILED"; tail -30 $O/bndebug.log; exit 1; }
grep "tdl bn" $O/bndebug.log | sort
scripts/gpu_resnet_window.sh bnfuse_rn
