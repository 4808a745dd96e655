#!/bin/bash
# conv kernel change: correctness tests, per-shape forward timings, ResNet-50 step.
set -o pipefail
O=gpurun_out/convab
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_gpu.py tests/test_slab_grad_gpu.py tests/test_bn_gpu.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for S in "14 14 256 256 3 1 1" "28 28 128 128 3 1 1" "7 7 512 512 3 1 1" "56 56 64 64 3 1 1" "14 14 1024 256 1 1 0" "28 28 512 128 1 1 0" "7 7 2048 512 1 1 0" "56 56 64 256 1 1 0"; do
  timeout -k 10 120 python scripts/conv_one.py $S 2>/dev/null | grep conv >> $O/time.txt || exit 1
done
cat $O/time.txt
timeout -k 10 400 python scripts/bench_resnet50.py --steps 20 --warmup 5 > $O/rn.log 2>&1 || { tail -20 $O/rn.log; exit 1; }
grep '"metric"' $O/rn.log | cut -c1-200
