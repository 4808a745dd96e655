#!/bin/bash
# the pre-change tree (df563a5): unfused model, async vs launch-blocking
set -o pipefail
O=gpurun_out/bnfuse
mkdir -p $O
cd oldtree
timeout -k 10 120 python -u scripts/diag_bnfuse2.py F ../$O/w_old_base.npz > ../$O/d_old_base.log 2>&1 || { tail -5 ../$O/d_old_base.log; exit 1; }
HIP_LAUNCH_BLOCKING=1 timeout -k 10 120 python -u scripts/diag_bnfuse2.py F ../$O/w_old_lb.npz > ../$O/d_old_lb.log 2>&1 || { tail -5 ../$O/d_old_lb.log; exit 1; }
echo done
