#!/bin/bash
# GPU box: MNIST exchange-in-finalize tests (one-/two-shot), communicator tests + ResNet-50 with 2 replica processes and the config-5 layout
# (2 TF_CONFIG workers x 2 replicas) on the box's one GPU (gloo control plane, xGMI data plane).
set -o pipefail
O=gpurun_out/rnmr
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mnist_exchange_gpu.py > $O/tx.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_xgmi_gpu.py \
  tests/test_generic_multiproc_gpu.py tests/test_comm_capture_gpu.py tests/test_bucket_wire_gpu.py > $O/t.log 2>&1 || exit 1
export TDL_SHARE_GPU=1
timeout -k 10 400 python scripts/bench_resnet50.py --gpus 2 --batch 32 --steps 10 --warmup 3 > $O/r2.log 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_resnet50.py --strategy mwms --workers 2 --gpus 4 --batch 16 --steps 6 --warmup 3 > $O/c5.log 2>&1
