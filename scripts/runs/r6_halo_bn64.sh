#!/bin/bash
# Halo conv with 64-column tiles on every shape (conv_force_halo(3)) vs the default kernels.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6halo64}
mkdir -p $O
timeout -k 10 300 python -u scripts/bench_conv_halo.py 256 3 > $O/bench.log 2>&1 || { echo BENCH FAILED; tail -20 $O/bench.log; exit 1; }
grep -o '"dir": "[a-z]*", "shape": \[[0-9, ]*\], "default_us": [0-9.]*, "halo_us": [0-9.]*' $O/bench.log
