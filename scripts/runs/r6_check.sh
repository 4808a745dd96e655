#!/bin/bash
# Round-6 re-entry check of a fresh-container build: full GPU suite + smoke + driver-shaped benches,
# then the generic-engine cliff bench (scripts/runs/r6_generic_bench.sh).  Usage: OUTDIR
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6check}
mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error|error" $O/tests.log | tail -20; tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2 3; do
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_$r.log 2>&1 || { echo BENCH FAILED; tail -20 $O/b20_$r.log; exit 1; }
grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*' $O/b20_$r.log
done
bash scripts/runs/r6_generic_bench.sh $O/generic
