#!/bin/bash
# conv prologue: direct 1x1 row offsets + reciprocal row split; tests, per-shape microbench, ResNet window
set -o pipefail
O=gpurun_out/prologue
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_conv_v2_gpu.py tests/test_bn_gpu.py tests/test_slab_grad_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 200 python scripts/bench_bn_in.py > $O/micro.jsonl 2>&1 || { tail $O/micro.jsonl; exit 1; }
grep shape $O/micro.jsonl
./scripts/gpu_resnet_window.sh rnw_prologue
