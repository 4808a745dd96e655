#!/bin/bash
# Round 5 MNIST v2: A/B of TDL_MNIST_VARIANT (1 = s_setprio 1 for waves 4-7), interleaved
set -o pipefail
O=gpurun_out/r5v2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mnist_fused_gpu.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
for v in 0 1; do
TDL_MNIST_VARIANT=$v timeout -k 10 200 python bench.py --gpus 1 --steps 1000 --warmup 20 > $O/b1000_v${v}_$i.log 2>&1 || { echo BENCH FAILED; tail -20 $O/b1000_v${v}_$i.log; exit 1; }
echo "v$v K=1000: $(tail -1 $O/b1000_v${v}_$i.log | cut -c100-160)"
TDL_MNIST_VARIANT=$v timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_v${v}_$i.log 2>&1 || { echo BENCH FAILED; tail -20 $O/b20_v${v}_$i.log; exit 1; }
echo "v$v K=20: $(tail -1 $O/b20_v${v}_$i.log | cut -c100-160)"
done
done
TDL_MNIST_VARIANT=1 timeout -k 10 200 python scripts/stamps_mnist.py > $O/phases_v1.log 2>&1 || { echo PH FAILED; tail -20 $O/phases_v1.log; exit 1; }
cat $O/phases_v1.log
echo done
