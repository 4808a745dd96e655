#!/bin/bash
# ResNet-50 b=256 bf16: per-dispatch listing of one steady-state step (which shapes the slow conv / BN calls are)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5rncalls
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python scripts/bench_resnet50.py --steps 6 --warmup 3 > $O/prof.log 2>&1 || { echo "PROF FAILED"; tail -20 $O/prof.log; exit 1; }
tail -2 $O/prof.log
python scripts/trace_calls.py $O/prof/run_kernel_trace.csv --marker k_sgd_momentum > $O/calls.txt && tail -3 $O/calls.txt
python scripts/trace_window.py $O/prof/run_kernel_trace.csv --steps 3 --marker k_sgd_momentum > $O/window.txt && head -12 $O/window.txt
