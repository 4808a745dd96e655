#!/bin/bash
# GPU-box: ResNet-50 loss trajectories (bf16 hand-written conv / bf16 MIOpen / fp32).
set -o pipefail
OUT=gpurun_out/loss_trace
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 python scripts/resnet_loss_trace.py mixed_bfloat16 224 64 24 > $OUT/bf16_auto.log 2>&1 || { echo "bf16 auto FAILED"; tail -20 $OUT/bf16_auto.log; exit 1; }
grep '^{' $OUT/bf16_auto.log
TDL_CONV=miopen timeout -k 10 240 python scripts/resnet_loss_trace.py mixed_bfloat16 224 64 24 > $OUT/bf16_miopen.log 2>&1 || { echo "bf16 miopen FAILED"; tail -20 $OUT/bf16_miopen.log; exit 1; }
grep '^{' $OUT/bf16_miopen.log
timeout -k 10 240 python scripts/resnet_loss_trace.py float32 224 64 24 > $OUT/fp32.log 2>&1 || { echo "fp32 FAILED"; tail -20 $OUT/fp32.log; exit 1; }
grep '^{' $OUT/fp32.log
