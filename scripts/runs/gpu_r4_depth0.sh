#!/bin/bash
# Round 4: native RCCL tests (GIL fix), conv single-stage variant correctness + A/B timing.
set -o pipefail
O=gpurun_out/r4d0
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_native_rccl_gpu.py tests/test_conv_gpu.py tests/test_conv_v2_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python -u scripts/bench_conv.py 256 keras > $O/bench_conv.jsonl 2>&1 || { echo "BENCH FAILED"; tail -30 $O/bench_conv.jsonl; exit 1; }
grep -v amdgpu.ids $O/bench_conv.jsonl
timeout -k 10 300 python scripts/bench_comm_fixed.py > $O/comm_fixed.jsonl 2>$O/comm_fixed.err || { echo COMM FAILED; tail -20 $O/comm_fixed.err; exit 1; }
grep '^{' $O/comm_fixed.jsonl | cut -c1-300
echo done
