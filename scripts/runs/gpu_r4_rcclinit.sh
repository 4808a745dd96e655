#!/bin/bash
set -o pipefail
O=gpurun_out/r4rcclinit; mkdir -p $O
export NCCL_DEBUG=INFO
PYTHONPATH=. timeout -k 10 120 python -u scripts/diag_rccl_init.py direct > $O/direct.log 2>&1; echo "direct rc=$?"
tail -40 $O/direct.log
