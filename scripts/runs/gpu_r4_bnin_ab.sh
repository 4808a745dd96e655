#!/bin/bash
# same-box A/B of the deferred BN apply (TDL_FUSE_BN_INPUT) on the ResNet-50 step, interleaved runs
set -o pipefail
O=gpurun_out/bnin_ab
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_gpu.py -k "input_side or deferred" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for i in 1 2; do
  for F in 0 1; do
    TDL_FUSE_BN_INPUT=$F timeout -k 10 300 python scripts/bench_resnet50.py > $O/b_${F}_$i.log 2>&1 || { tail $O/b_${F}_$i.log; exit 1; }
    echo "fuse=$F run $i: $(tail -1 $O/b_${F}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
