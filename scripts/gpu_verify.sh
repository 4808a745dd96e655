#!/bin/bash
# GPU-box check of a tree: GPU tests, smoke, MNIST bench (driver K/W), ResNet-50 bench.
# Usage: scripts/gpu_verify.sh TAG
set -o pipefail
TAG=${1:-verify}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 400 python scripts/bench_resnet50.py > $OUT/rn50.log 2>&1 || { echo "RN50 FAILED"; tail -20 $OUT/rn50.log; exit 1; }
tail -1 $OUT/rn50.log
