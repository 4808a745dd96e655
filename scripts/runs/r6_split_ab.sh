#!/bin/bash
# MNIST headline: the execution graph with its first / last kernel launched directly (TDL_SPLIT_GRAPH=1)
# vs the whole-execution graph, interleaved on one box.  Usage: OUTDIR
set -o pipefail
O=${1:-gpurun_out/r6split}
mkdir -p $O
for r in 1 2 3; do
  for v in 0 1; do
    TDL_SPLIT_GRAPH=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/k20_s${v}_$r.log 2>&1 || { tail -5 $O/k20_s${v}_$r.log; exit 1; }
    TDL_SPLIT_GRAPH=$v timeout -k 10 120 python bench.py --steps 1000 --warmup 100 > $O/k1000_s${v}_$r.log 2>&1 || { tail -5 $O/k1000_s${v}_$r.log; exit 1; }
  done
done
for f in $O/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f) $(grep -o 'timed region.*' $f)"; done
