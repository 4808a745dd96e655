#!/bin/bash
# GPU-box routine: GPU tests, 1-replica bench, 2-replica shared-GPU bench, kernel-trace profile.
# Usage: scripts/gpu_round.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-run}
KEXPR=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$KEXPR" ]; then KARG=(-k "$KEXPR"); else KARG=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "${KARG[@]}" > $OUT/tests.log 2>&1 \
  || { echo "TESTS FAILED"; tail -60 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_k20.log 2>&1 || { echo "BENCH FAILED"; tail -20 $OUT/bench_k20.log; exit 1; }
tail -1 $OUT/bench_k20.log
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
TDL_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --steps 200 --warmup 20 > $OUT/bench_2shared.log 2>&1 || { echo "BENCH2 FAILED"; tail -30 $OUT/bench_2shared.log; exit 1; }
tail -1 $OUT/bench_2shared.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 200 --warmup 20 > $OUT/prof.log 2>&1 || { echo "PROF FAILED"; tail -20 $OUT/prof.log; exit 1; }
python scripts/prof_summary.py $OUT/prof/run_kernel_stats.csv
