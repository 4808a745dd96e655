#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6gmulti
timeout -k 10 900 python -u -m pytest tests/test_generic_multiproc_gpu.py -x -v --timeout 450 --timeout-method thread -k "device_execution or bucketed_xgmi_replicas and 2" > gpurun_out/r6gmulti/tests.log 2>&1 || { tail -60 gpurun_out/r6gmulti/tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r6gmulti/tests.log | tail -6
