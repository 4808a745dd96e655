#!/bin/bash
# Round 5 v4: generic f32 conv/Dense kernels, optimizer kernels, hot-path tests, stagger A/B
set -o pipefail
O=gpurun_out/r5v4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_conv_f32_gpu.py tests/test_fit_gpu.py tests/test_hot_path_kernels_gpu.py > $O/tests.log 2>&1 || { echo TESTS FAILED; grep -E "PASS|FAIL" $O/tests.log | tail -30; tail -40 $O/tests.log; exit 1; }
grep -E "FAIL|passed|failed" $O/tests.log | tail -5
for i in 1 2 3; do
for v in 0 2; do
TDL_MNIST_VARIANT=$v timeout -k 10 200 python bench.py --gpus 1 --steps 1000 --warmup 20 > $O/b1000_v${v}_$i.log 2>&1 || { echo BENCH FAILED; tail -20 $O/b1000_v${v}_$i.log; exit 1; }
TDL_MNIST_VARIANT=$v timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_v${v}_$i.log 2>&1 || { echo BENCH FAILED; tail -20 $O/b20_v${v}_$i.log; exit 1; }
python3 -c "
import json
for f in ['$O/b1000_v${v}_$i.log','$O/b20_v${v}_$i.log']:
    d=json.loads([l for l in open(f) if l.startswith('{')][-1]); print(f, d['value'], d['ms_per_step'])"
done
done
for v in 0 2; do
TDL_MNIST_VARIANT=$v timeout -k 10 200 python scripts/stamps_mnist.py > $O/phases_v$v.log 2>&1 || { echo PH FAILED; tail -20 $O/phases_v$v.log; exit 1; }
echo "== v$v"; grep -v amdgpu $O/phases_v$v.log
done
echo done
