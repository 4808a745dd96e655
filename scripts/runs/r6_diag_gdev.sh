#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6diag
timeout -k 10 300 python scripts/diag_generic_device.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r6diag/diag.log
