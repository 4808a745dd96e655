#!/bin/bash
# Round 5: single-process MirroredStrategy on the GPU, exchange + bench tests incl. R = 8
set -o pipefail
O=gpurun_out/r5local
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_local_replicas_gpu.py tests/test_mnist_exchange_gpu.py tests/test_bench_gpu.py tests/test_fit_gpu.py tests/test_fault_gpu.py > $O/tests.log 2>&1 || { echo TESTS FAILED; grep -E "PASS|FAIL" $O/tests.log | tail -30; tail -40 $O/tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/tests.log | tail -40

for i in 1 2; do
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_$i.log 2>&1 || { echo BENCH FAILED; tail -20 $O/b20_$i.log; exit 1; }
timeout -k 10 200 python bench.py --gpus 1 --steps 1000 --warmup 20 > $O/b1000_$i.log 2>&1 || { echo BENCH FAILED; tail -20 $O/b1000_$i.log; exit 1; }
python3 -c "
import json
for f in ['$O/b20_$i.log','$O/b1000_$i.log']:
    d=json.loads([l for l in open(f) if l.startswith('{')][-1]); print(f, d['value'], d['ms_per_step'])"
done
timeout -k 10 200 python scripts/stamps_mnist.py > $O/phases.log 2>&1 || { echo PH FAILED; tail -20 $O/phases.log; exit 1; }
grep -v amdgpu $O/phases.log
echo done
