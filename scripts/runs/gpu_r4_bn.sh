#!/bin/bash
# Round 4: blocked BN elementwise kernels -- bitwise vs grid-stride, fp64 checks, bandwidth sweep.
set -o pipefail
O=gpurun_out/r4bn
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_bn_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 500 python -u scripts/bench_bn.py > $O/bench_bn.jsonl 2>&1 || { echo "BENCH FAILED"; tail -30 $O/bench_bn.jsonl; exit 1; }
grep '^{' $O/bench_bn.jsonl
echo done
