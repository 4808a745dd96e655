#!/bin/bash
# f32 GEMM split-plan cap A/B (TDL_F32_SPLIT=kmin,cap) on the generic engine, interleaved.  Usage: OUTDIR
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6cap}
mkdir -p $O
for r in 1 2 3; do
for c in 64,1024 64,256 64,512 96,1024; do
  TDL_F32_SPLIT=$c timeout -k 10 300 python bench.py --engine generic --steps 200 --warmup 25 > $O/g_${c/,/_}_$r.json 2> $O/g_${c/,/_}_$r.err || { tail -20 $O/g_${c/,/_}_$r.err; exit 1; }
  echo "split=$c $r $(grep -o '"ms_per_step": [0-9.]*' $O/g_${c/,/_}_$r.json)"
done
done
