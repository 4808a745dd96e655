#!/bin/bash
set -o pipefail
O=gpurun_out/stem
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_stem_gpu.py > $O/t.log 2>&1; grep -E "PASS|FAIL|Error|assert" $O/t.log | head -30
scripts/diag_det.sh
