#!/bin/bash
# Round 4: conv main-loop variants (v1 depths, dma1 single-stage LDS-DMA) and single-stage wgrad:
# bitwise/fp32 tests, then A/B timings.
set -o pipefail
O=gpurun_out/r4ml
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_conv_v2_gpu.py tests/test_bn_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 500 python -u scripts/bench_conv.py 256 keras > $O/bench_conv.jsonl 2>&1 || { echo "BENCH FAILED"; tail -30 $O/bench_conv.jsonl; exit 1; }
grep -v amdgpu.ids $O/bench_conv.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['dir'], d['shape'][1:], d['hip_us'], d['v1_v2_dma4_dma3_d3_d0_d4_us'], d['miopen_us'], d['calls'])"
timeout -k 10 500 python -u scripts/bench_wgrad.py --candidates 8 --single 1 > $O/wg1.jsonl 2>&1 || { echo "WG1 FAILED"; tail -30 $O/wg1.jsonl; exit 1; }
timeout -k 10 500 python -u scripts/bench_wgrad.py --candidates 8 --single 0 > $O/wg0.jsonl 2>&1 || { echo "WG0 FAILED"; tail -30 $O/wg0.jsonl; exit 1; }
python - <<'PY'
import json
def load(f):
    return [json.loads(l) for l in open(f) if l.startswith('{')]
a, b = load('gpurun_out/r4ml/wg1.jsonl'), load('gpurun_out/r4ml/wg0.jsonl')
for x, y in zip(a, b):
    if x.get('dir') == 'wgrad':
        print(x['shape'][1:], 'single', x['hip_us'], x['best_plan'], 'double', y['hip_us'], y['best_plan'], 'miopen', x['miopen_us'])
print(a[-1], b[-1])
PY
echo done
