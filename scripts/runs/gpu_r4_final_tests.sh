#!/bin/bash
# Round 4 final: the whole GPU test suite (one process), durations
set -o pipefail
O=gpurun_out/r4final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=20 > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" $O/tests.log | head -20; tail -40 $O/tests.log; exit 1; }
tail -25 $O/tests.log
