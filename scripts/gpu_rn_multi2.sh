#!/bin/bash
# GPU box: ResNet-50 with 2 replica processes and the 2x2 config-5 layout on the box's one GPU,
# the generic multi-replica / xGMI tests, then which BN layers still take a separate sum pass.
set -o pipefail
O=gpurun_out/rnmr
mkdir -p $O
export TDL_SHARE_GPU=1
timeout -k 10 400 python scripts/bench_resnet50.py --gpus 2 --batch 32 --steps 10 --warmup 3 > $O/r2.log 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_resnet50.py --strategy mwms --workers 2 --gpus 4 --batch 16 --steps 6 --warmup 3 > $O/c5.log 2>&1 || exit 1
unset TDL_SHARE_GPU
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_generic_multiproc_gpu.py tests/test_xgmi_gpu.py > $O/t2.log 2>&1 || exit 1
TDL_BN_DEBUG=1 timeout -k 10 300 python scripts/bench_resnet50.py --steps 2 --warmup 2 > $O/bndebug.log 2>&1
