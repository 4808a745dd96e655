#!/bin/bash
# rocprofv3 kernel stats of the generic engine's reference-CNN step (K=100 W=10).  Usage: OUTDIR
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6gprof}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --engine generic --steps 100 --warmup 10 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/prof_summary.py $O/prof/run_kernel_stats.csv > $O/prof_summary.txt 2>&1; head -40 $O/prof_summary.txt
