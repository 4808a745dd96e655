#!/bin/bash
# Round 4: conv v2 (LDS-DMA ring) correctness vs v1 / fp32, then per-shape timings v1 vs v2 vs MIOpen.
set -o pipefail
O=gpurun_out/r4conv
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv_v2_gpu.py tests/test_conv_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python -u scripts/bench_conv.py 256 keras > $O/bench_conv.jsonl 2>&1 || { echo "BENCH FAILED"; tail -30 $O/bench_conv.jsonl; exit 1; }
cat $O/bench_conv.jsonl | grep -v amdgpu.ids
timeout -k 10 500 python -u scripts/bench_wgrad.py --candidates 8 > $O/bench_wgrad.jsonl 2>&1 || { echo "WGRAD BENCH FAILED"; tail -30 $O/bench_wgrad.jsonl; exit 1; }
grep -v amdgpu.ids $O/bench_wgrad.jsonl | cut -c1-400
echo done
