#!/bin/bash
# Round 5 v5: head operands in LDS, wave 0's W2 prefetch after its head (poll not queued behind it),
# buffer-load W2 prefetch, packed dP2 dot products
set -o pipefail
O=gpurun_out/r5v5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_mnist_fused_gpu.py tests/test_fit_gpu.py tests/test_eval_gpu.py > $O/tests.log 2>&1 || { echo TESTS FAILED; grep -E "PASS|FAIL" $O/tests.log | tail -30; tail -40 $O/tests.log; exit 1; }
grep -E "FAIL|passed|failed" $O/tests.log | tail -5
for i in 1 2 3; do
timeout -k 10 200 python bench.py --gpus 1 --steps 1000 --warmup 20 > $O/b1000_$i.log 2>&1 || { echo BENCH FAILED; tail -20 $O/b1000_$i.log; exit 1; }
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_$i.log 2>&1 || { echo BENCH FAILED; tail -20 $O/b20_$i.log; exit 1; }
python3 -c "
import json
for f in ['$O/b1000_$i.log','$O/b20_$i.log']:
    d=json.loads([l for l in open(f) if l.startswith('{')][-1]); print(f, d['value'], d['ms_per_step'])"
grep -h "timed region" $O/b20_$i.log
done
timeout -k 10 200 python scripts/stamps_mnist.py > $O/phases.log 2>&1 || { echo PH FAILED; tail -20 $O/phases.log; exit 1; }
grep -v amdgpu $O/phases.log
echo done
