#!/bin/bash
# hardware bf16 packing in the conv epilogues + input-side BN: tests, ResNet A/B, per-shape microbench
set -o pipefail
O=gpurun_out/epi
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_conv_v2_gpu.py tests/test_bn_gpu.py tests/test_slab_grad_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for i in 1 2; do
  for F in 0 1; do
    TDL_FUSE_BN_INPUT=$F timeout -k 10 300 python scripts/bench_resnet50.py > $O/b_${F}_$i.log 2>&1 || { tail $O/b_${F}_$i.log; exit 1; }
    echo "fuse=$F run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/b_${F}_$i.log)"
  done
done
timeout -k 10 200 python scripts/bench_bn_in.py > $O/micro.jsonl 2>&1 || { tail $O/micro.jsonl; exit 1; }
grep shape $O/micro.jsonl
