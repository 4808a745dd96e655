#!/bin/bash
# Round 4 final: smoke, MNIST bench (driver's K=20 and K=1000), ResNet-50 bench
set -o pipefail
O=gpurun_out/r4final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { echo BENCH FAILED; tail -20 $O/bench20.log; exit 1; }
tail -2 $O/bench20.log
timeout -k 10 200 python bench.py --gpus 1 --steps 1000 --warmup 20 > $O/bench1000.log 2>&1 || { echo BENCH1000 FAILED; tail -20 $O/bench1000.log; exit 1; }
tail -1 $O/bench1000.log
timeout -k 10 400 python scripts/bench_resnet50.py > $O/resnet.log 2>&1 || { echo RESNET FAILED; tail -20 $O/resnet.log; exit 1; }
tail -1 $O/resnet.log | cut -c1-600
echo done
