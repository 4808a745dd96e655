#!/bin/bash
# full GPU suite + smoke + bench (the driver's round-end tiers)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5full
mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error|error" $O/tests.log | tail -20; tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo BENCH FAILED; tail -20 $O/bench.log; exit 1; }
grep "{" $O/bench.log | cut -c1-300
