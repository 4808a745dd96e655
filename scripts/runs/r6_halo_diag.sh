#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/halodiag
mkdir -p $O
timeout -k 10 200 python -u scripts/bench_conv_halo.py 256 > $O/d0.log 2>&1 && \
TDL_CONV_HALO_DIAG=1 timeout -k 10 200 python -u scripts/bench_conv_halo.py 256 > $O/d1.log 2>&1 && \
TDL_CONV_HALO_DIAG=2 timeout -k 10 200 python -u scripts/bench_conv_halo.py 256 > $O/d2.log 2>&1
for f in d0 d1 d2; do echo == $f; grep -o '"dir": "[a-z]*", "shape": \[[0-9, ]*\], "default_us": [0-9.]*, "halo_us": [0-9.]*' $O/$f.log; done
