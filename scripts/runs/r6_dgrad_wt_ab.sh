#!/bin/bash
# Generic engine: conv input gradient reading the HWIO kernel transposed in-kernel (default for <= 2^16
# weights) vs a [R][S][K][C] copy + 16-B operand loads (TDL_F32_DGRAD_HWIO_MAX=0), interleaved.  Usage: OUTDIR
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6dwt}
mkdir -p $O
for r in 1 2 3; do
for c in 65536 0; do
  TDL_F32_DGRAD_HWIO_MAX=$c timeout -k 10 300 python bench.py --engine generic --steps 200 --warmup 25 > $O/g_${c}_$r.json 2> $O/g_${c}_$r.err || { tail -20 $O/g_${c}_$r.err; exit 1; }
  echo "hwio_max=$c $r $(grep -o '"ms_per_step": [0-9.]*' $O/g_${c}_$r.json)"
done
done
