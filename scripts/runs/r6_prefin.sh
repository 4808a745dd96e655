#!/bin/bash
# BN prereduce + finalize in one launch: BN GPU tests, then the ResNet-50 window with it on (default) and off.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6prefin}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_bn_gpu.py tests/test_slab_grad_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 1 0; do
    TDL_BN_PREFIN=$v timeout -k 10 400 python scripts/bench_resnet50.py > $O/rn_${v}_$r.log 2>&1 || { tail -20 $O/rn_${v}_$r.log; exit 1; }
    echo "prefin=$v rep$r $(grep -o '"value": [0-9.]*, "unit": "images/sec", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*' $O/rn_${v}_$r.log)"
  done
done
