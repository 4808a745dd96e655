#!/bin/bash
# single-stage 2x2 LDS-DMA weight gradient as an autotuner plan kind: tests, per-shape sweep, ResNet-50 bench
set -o pipefail
mkdir -p gpurun_out/wgdma1b
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_conv_v2_gpu.py -k "wgrad" > gpurun_out/wgdma1b/test.log 2>&1 || { tail -30 gpurun_out/wgdma1b/test.log; exit 1; }
tail -2 gpurun_out/wgdma1b/test.log
timeout -k 10 300 python -u scripts/bench_wgrad.py --candidates 6 > gpurun_out/wgdma1b/bench.jsonl 2>&1 || { tail gpurun_out/wgdma1b/bench.jsonl; exit 1; }
tail -1 gpurun_out/wgdma1b/bench.jsonl
timeout -k 10 400 python -u scripts/bench_resnet50.py > gpurun_out/wgdma1b/resnet.log 2>&1 || { tail gpurun_out/wgdma1b/resnet.log; exit 1; }
tail -1 gpurun_out/wgdma1b/resnet.log | cut -c1-600
