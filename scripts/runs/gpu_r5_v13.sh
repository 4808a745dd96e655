#!/bin/bash
# v13: write-through P2 / part1 stores (A/B vs ab/v13) + f32 conv kernel bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5v13
OUT=r5v13 AB=r5v13ab REPS=3 ARMS="v13=ab/v13:0 cur=.:0" bash scripts/runs/gpu_r5_v6.sh || exit 1
timeout -k 10 300 python scripts/bench_conv_f32.py > gpurun_out/r5v13/conv_f32.log 2>&1 || { echo CONVF32 FAILED; tail -20 gpurun_out/r5v13/conv_f32.log; exit 1; }
grep "{" gpurun_out/r5v13/conv_f32.log
