#!/bin/bash
# Generic engine: f32 GEMM operand loads through buffer resources with 32-bit offsets (TDL_F32_BUF=1, the
# default) vs 64-bit addresses with clamped selects (TDL_F32_BUF=0), interleaved.  Usage: OUTDIR
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6buf}
mkdir -p $O
for r in 1 2 3; do
for c in 1 0; do
  TDL_F32_BUF=$c timeout -k 10 300 python bench.py --engine generic --steps 200 --warmup 25 > $O/g_${c}_$r.json 2> $O/g_${c}_$r.err || { tail -20 $O/g_${c}_$r.err; exit 1; }
  echo "buf=$c $r $(grep -o '"ms_per_step": [0-9.]*' $O/g_${c}_$r.json)"
done
done
