#!/bin/bash
# Round 4: dmap (half-tile ping-pong LDS-DMA) -- bitwise tests vs v1, then per-shape A/B timings.
set -o pipefail
O=gpurun_out/r4dmap
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_conv_v2_gpu.py -x -v --timeout 200 --timeout-method thread -k dmap > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 500 python -u scripts/bench_conv.py 256 keras > $O/bench_conv.jsonl 2>&1 || { echo "BENCH FAILED"; tail -30 $O/bench_conv.jsonl; exit 1; }
grep -v amdgpu.ids $O/bench_conv.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['dir'], d['shape'][1:], d['hip_us'], d['v1_v2_dma1_dmap_d3_d0_d4_us'], d['miopen_us'], d['calls'])"
echo done
