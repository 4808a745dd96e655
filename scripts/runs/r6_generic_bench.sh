#!/bin/bash
# Generic-engine cliff: bench.py --engine generic for the reference CNN and two
# model changes the fused path does not take, next to the fused headline.  Usage: OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r6_generic}
mkdir -p $OUT
timeout -k 10 200 python bench.py --steps 200 --warmup 20 > $OUT/fused.json 2> $OUT/fused.err || exit 1
tail -1 $OUT/fused.json
for v in reference same dropout; do
  timeout -k 10 300 python bench.py --engine generic --variant $v --steps 200 --warmup 20 > $OUT/generic_$v.json 2> $OUT/generic_$v.err || { tail -20 $OUT/generic_$v.err; exit 1; }
  tail -1 $OUT/generic_$v.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --engine generic --steps 100 --warmup 10 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python scripts/prof_summary.py $OUT/prof/run_kernel_stats.csv > $OUT/prof_summary.txt 2>&1; head -30 $OUT/prof_summary.txt
