#!/bin/bash
# GPU-box: is the ResNet-50 bench divergence batch-size or bench-path specific?
set -o pipefail
OUT=gpurun_out/loss_trace2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python scripts/resnet_loss_trace.py mixed_bfloat16 224 256 16 > $OUT/bf16_b256.log 2>&1 || { echo "b256 FAILED"; tail -20 $OUT/bf16_b256.log; exit 1; }
grep '^{' $OUT/bf16_b256.log
timeout -k 10 300 python scripts/bench_resnet50.py --batch 64 --steps 20 --warmup 5 > $OUT/bench_b64.log 2>&1 || { echo "bench b64 FAILED"; tail -20 $OUT/bench_b64.log; exit 1; }
grep '^{' $OUT/bench_b64.log
