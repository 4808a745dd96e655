#!/bin/bash
set -o pipefail
O=gpurun_out/stem
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_stem_gpu.py tests/test_slab_grad_gpu.py > $O/t.log 2>&1; grep -E "PASS|FAIL|Error|assert" $O/t.log | head -30
timeout -k 10 300 python -u scripts/bench_resnet50.py > $O/rn.log 2>&1; tail -2 $O/rn.log | cut -c1-600
