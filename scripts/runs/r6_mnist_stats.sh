#!/bin/bash
# rocprofv3 kernel stats of the MNIST bench (K=1000) at the end-of-round-6 build
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6stats}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 1000 --warmup 100 > $O/prof.log 2>&1 || { echo PROF FAILED; tail -20 $O/prof.log; exit 1; }
grep "{" $O/prof.log | cut -c1-160
f=$(ls $O/prof/*kernel_stats.csv | head -1); head -5 "$f"
