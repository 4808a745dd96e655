#!/bin/bash
# Timed-region breakdown of bench.py at several K (host launch vs device drain), plus the
# synchronous-index variant at K=1000.  Usage: scripts/diag_bench_overhead.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-diag}
mkdir -p $OUT
for k in 20 200 1000; do
  TDL_HOST_TIMING=1 timeout -k 10 120 python bench.py --steps $k --warmup 5 > $OUT/k$k.log 2>&1 || exit 1
  grep -E "timed region|host us" $OUT/k$k.log; tail -1 $OUT/k$k.log | cut -c1-200
done
TDL_ASYNC_INDICES=0 TDL_HOST_TIMING=1 timeout -k 10 120 python bench.py --steps 1000 --warmup 5 > $OUT/k1000_sync.log 2>&1 || exit 1
grep -E "timed region|host us" $OUT/k1000_sync.log; tail -1 $OUT/k1000_sync.log | cut -c1-200
