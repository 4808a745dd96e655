#!/bin/bash
# GPU-box: ResNet-50 bench (b=256 bf16) + steady-state kernel breakdown over the last 3 steps.
# Usage: scripts/gpu_resnet_window.sh TAG [extra bench args]
set -o pipefail
TAG=${1:-rnw}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python scripts/bench_resnet50.py "$@" > $OUT/bench.log 2>&1 || { echo "BENCH FAILED"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- python scripts/bench_resnet50.py --steps 6 --warmup 3 "$@" > $OUT/prof.log 2>&1 || { echo "PROF FAILED"; tail -20 $OUT/prof.log; exit 1; }
python scripts/trace_window.py $OUT/prof/run_kernel_trace.csv --steps 3 --marker k_sgd_momentum > $OUT/window.txt && head -70 $OUT/window.txt
