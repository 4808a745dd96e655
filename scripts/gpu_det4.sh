#!/bin/bash
set -o pipefail
O=gpurun_out/bnfuse
mkdir -p $O
run() { env $2 timeout -k 10 120 python -u scripts/diag_bnfuse2.py F $O/w_$1.npz > $O/d_$1.log 2>&1 || { tail -5 $O/d_$1.log; exit 1; }; }
run base ""
run ser "AMD_SERIALIZE_KERNEL=3"
run ca0 "TDL_CAST_ACCUMULATE=0"
run ca0ser "TDL_CAST_ACCUMULATE=0 AMD_SERIALIZE_KERNEL=3"
run fuse0 "TDL_FUSE=0"
run fuse0ser "TDL_FUSE=0 AMD_SERIALIZE_KERNEL=3"
run lb "HIP_LAUNCH_BLOCKING=1"
echo done
