set -o pipefail
OUT=gpurun_out/r2s4
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench20.log 2>&1 || { echo BENCH FAILED; tail -20 $OUT/bench20.log; exit 1; }
tail -1 $OUT/bench20.log
timeout -k 10 300 python scripts/bench_resnet50.py > $OUT/resnet.log 2>&1 || { echo RESNET FAILED; tail -20 $OUT/resnet.log; exit 1; }
tail -1 $OUT/resnet.log
