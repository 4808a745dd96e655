#!/bin/bash
set -o pipefail
O=gpurun_out/r4rccl
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_native_rccl_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 $O/tests.log; exit 1; }
tail -6 $O/tests.log
timeout -k 10 300 python scripts/bench_comm_fixed.py > $O/comm_fixed.jsonl 2>$O/comm_fixed.err || { echo COMM FAILED; tail -20 $O/comm_fixed.err; exit 1; }
grep '^{' $O/comm_fixed.jsonl
echo done
