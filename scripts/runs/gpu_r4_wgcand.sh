#!/bin/bash
# weight-gradient autotuner breadth: 6 (default) vs 12 timed candidates -- per-shape sweep and the ResNet-50 step
set -o pipefail
O=gpurun_out/wgcand
mkdir -p $O
timeout -k 10 300 python -u scripts/bench_wgrad.py --candidates 12 > $O/sweep12.jsonl 2>&1 || { tail $O/sweep12.jsonl; exit 1; }
tail -1 $O/sweep12.jsonl
for i in 1 2; do
  for N in 6 12; do
    TDL_WGRAD_CANDIDATES=$N timeout -k 10 300 python scripts/bench_resnet50.py > $O/b_${N}_$i.log 2>&1 || { tail $O/b_${N}_$i.log; exit 1; }
    echo "candidates=$N run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/b_${N}_$i.log)"
  done
done
