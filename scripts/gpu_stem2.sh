#!/bin/bash
set -o pipefail
O=gpurun_out/stem
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_stem_gpu.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
scripts/gpu_resnet_window.sh rn_r3c
