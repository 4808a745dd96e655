#!/bin/bash
# current fused MNIST step: per-wave phase stamps + whole-step stamps (baseline for round-5 re-entry work)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5stamps
mkdir -p $O
timeout -k 10 200 python scripts/stamps_mnist.py > $O/phases.log 2>&1 || { echo FAILED; tail $O/phases.log; exit 1; }
timeout -k 10 200 python scripts/stamps_step.py > $O/step.log 2>&1 || { echo FAILED; tail $O/step.log; exit 1; }
cat $O/step.log | head -30; cat $O/phases.log | head -40
