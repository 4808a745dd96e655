#!/bin/bash
# Round 4: conv main-loop variants (DEPTH 3: single LDS stage + register prefetch, 3 WGs/CU) -- tests + A/B timing.
set -o pipefail
O=gpurun_out/r4d3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_conv_v2_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 500 python -u scripts/bench_conv.py 256 keras > $O/bench_conv.jsonl 2>&1 || { echo "BENCH FAILED"; tail -30 $O/bench_conv.jsonl; exit 1; }
grep -v amdgpu.ids $O/bench_conv.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['dir'], d['shape'][1:], d['hip_us'], d['v1_v2_dma4_dma3_d3_d0_d4_us'], d['miopen_us'], d['calls'])"
echo done
