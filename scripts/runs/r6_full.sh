#!/bin/bash
# Round-6 full check: every GPU test, smoke, the driver-shaped MNIST bench (3x), and the ResNet-50 bench
# with its steady-state breakdown.  Usage: OUTDIR
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6full}
mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error|error" $O/tests.log | tail -20; tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2 3; do
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_$r.log 2>&1 || { echo BENCH FAILED; tail -20 $O/b20_$r.log; exit 1; }
grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*' $O/b20_$r.log
done
bash scripts/gpu_resnet_window.sh ${O#gpurun_out/}/rn
