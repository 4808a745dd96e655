#!/bin/bash
# Round-3 GPU routine: GPU tests, 1-GPU MNIST bench (driver K/W), ResNet-50 bench.  Usage: scripts/gpu_r3.sh TAG
set -o pipefail
TAG=${1:-r3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench20.log 2>&1 || { echo BENCH FAILED; tail -20 $OUT/bench20.log; exit 1; }
tail -1 $OUT/bench20.log
timeout -k 10 200 python bench.py --gpus 1 --steps 1000 --warmup 20 > $OUT/bench1000.log 2>&1 || { echo BENCH FAILED; tail -20 $OUT/bench1000.log; exit 1; }
tail -1 $OUT/bench1000.log
if [ -n "$RESNET" ]; then
timeout -k 10 300 python scripts/bench_resnet50.py > $OUT/resnet.log 2>&1 || { echo RESNET FAILED; tail -20 $OUT/resnet.log; exit 1; }
tail -1 $OUT/resnet.log
fi
