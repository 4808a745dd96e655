#!/bin/bash
# DIAG variants of the finalize: 16 skip conv2 pieces, 32 skip dW3, 64 dW4 without dL loads, 128 dW4 without H loads
# (the DIAG bits were a temporary build of mnist_cnn.hip: finalize_x_body returned early for those ranges / skipped those loads; not in the tree)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5diag
for v in ${VARS:-0 16 32 48}; do
TDL_MNIST_VARIANT=$v timeout -k 10 200 python scripts/stamps_step.py > gpurun_out/r5diag/step_$v.log 2>&1 || { echo FAILED; tail gpurun_out/r5diag/step_$v.log; exit 1; }
echo "== $v"; grep -E "KF-X span|latest" gpurun_out/r5diag/step_$v.log
done
