#!/bin/bash
# End-of-round-3 GPU check: whole GPU suite, smoke, MNIST bench (K=20 as the driver runs it, K=1000),
# ResNet-50 bench, rocprofv3 kernel stats of the MNIST bench. Every GPU step has its own time limit;
# the script stops at the first failing step.
set -o pipefail
O=gpurun_out/r3final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { echo BENCH FAILED; tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log
timeout -k 10 200 python bench.py --gpus 1 --steps 1000 --warmup 20 > $O/bench1000.log 2>&1 || { echo BENCH1000 FAILED; tail -20 $O/bench1000.log; exit 1; }
tail -1 $O/bench1000.log
timeout -k 10 300 python scripts/bench_resnet50.py > $O/resnet.log 2>&1 || { echo RESNET FAILED; tail -20 $O/resnet.log; exit 1; }
tail -1 $O/resnet.log
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o mnist -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 200 --warmup 20 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo PROF FAILED; tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
echo done
