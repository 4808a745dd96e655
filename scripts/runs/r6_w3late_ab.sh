#!/bin/bash
# W3 prefetch moved from conv1 into conv2 (TDL_MNIST_VARIANT bit 16) on top of the XCD map (8):
# numerics, phase stamps of both arms, same-box interleaved A/B.
set -o pipefail
O=gpurun_out/${1:-r6w3}
mkdir -p $O
export TMPDIR=/tmp
TDL_MNIST_VARIANT=24 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mnist_fused_gpu.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 8 24; do
TDL_MNIST_VARIANT=$v timeout -k 10 200 python scripts/stamps_mnist.py > $O/phases_$v.log 2>&1 || { echo PH FAILED; tail -20 $O/phases_$v.log; exit 1; }
echo "== variant $v"; grep -v amdgpu $O/phases_$v.log | head -22
done
bash scripts/runs/ab_arms.sh ${1:-r6w3}/ab ${REPS:-3} xcd=.:8 late=.:24
