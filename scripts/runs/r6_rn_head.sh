#!/bin/bash
# Fused loss head for bf16 / large logits (ResNet-50's 256 x 1000 head) + the multi-replica generic-engine
# device-graph test, then the ResNet-50 bench + steady-state window.  Usage: OUTDIR
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6rnhead}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_conv_f32_gpu.py tests/test_generic_device_gpu.py tests/test_generic_multiproc_gpu.py -x -v --timeout 450 --timeout-method thread -k "xent or device or bucketed_xgmi_replicas and 2" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
bash scripts/gpu_resnet_window.sh ${O#gpurun_out/}/rn
