#!/bin/bash
# DIAG (temporary build): fused-kernel staging without the dependent index load (variant 16: image = workgroup's batch slot)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5idxdiag
mkdir -p $O
for v in 0 16 0 16; do
TDL_MNIST_VARIANT=$v timeout -k 10 200 python scripts/stamps_mnist.py > $O/phases_$v.log 2>&1 || { echo FAILED; tail $O/phases_$v.log; exit 1; }
TDL_MNIST_VARIANT=$v timeout -k 10 200 python scripts/stamps_step.py > $O/step_$v.log 2>&1 || { echo FAILED; tail $O/step_$v.log; exit 1; }
echo "== $v"; grep -E "fused span|step span" $O/step_$v.log; grep -E "kernel span|stage-issued|stage-barrier|conv1-done|dense1-partial|bwd reduced" $O/phases_$v.log
done
