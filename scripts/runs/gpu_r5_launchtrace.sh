#!/bin/bash
# K=20 bench under rocprofv3 --kernel-trace --hip-trace: hipGraphLaunch call -> first kernel start,
# last kernel end -> synchronize return (same clock domain)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5lt
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d $O/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo PROF FAILED; tail -20 $O/prof.log; exit 1; }
ls $O/prof
python3 scripts/launch_trace.py $O/prof > $O/summary.txt && cat $O/summary.txt
