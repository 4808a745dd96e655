#!/bin/bash
# Pooled-gradient loaders (TDL_FUSE_CONV_POOL_BWD=1) vs the max-pool backward pass (=0), generic engine,
# interleaved on one box.  Usage: OUTDIR
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6pbwd}
mkdir -p $O
for r in 1 2 3; do
for f in 1 0; do
  TDL_FUSE_CONV_POOL_BWD=$f timeout -k 10 300 python bench.py --engine generic --steps 200 --warmup 25 > $O/g_f${f}_$r.json 2> $O/g_f${f}_$r.err || { tail -20 $O/g_f${f}_$r.err; exit 1; }
  echo "bwd=$f $r $(grep -o '"ms_per_step": [0-9.]*' $O/g_f${f}_$r.json)"
done
done
