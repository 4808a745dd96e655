#!/bin/bash
set -o pipefail
OUT=gpurun_out/loss_trace3
mkdir -p $OUT
export TMPDIR=/tmp
TDL_TRACE_LOSS=1 timeout -k 10 300 python scripts/bench_resnet50.py --batch 64 --steps 10 --warmup 12 > $OUT/bench_b64.log 2>&1 || { echo "bench FAILED"; tail -20 $OUT/bench_b64.log; exit 1; }
grep -E '^warmup|^\{' $OUT/bench_b64.log | cut -c1-120
grep -o '"final_loss": [^}]*' $OUT/bench_b64.log
