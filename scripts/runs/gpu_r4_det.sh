#!/bin/bash
# Round 4: generic-engine nondeterminism bisection.  (1) bitwise determinism of every hand-written
# ResNet-path kernel, (2) per-op checksums of the BN-heavy diag model's 2-step run: async twice,
# HIP_LAUNCH_BLOCKING=1, and async with torch deterministic algorithms (warn-only), then diffs,
# (3) MNIST bench at the driver's K=20 as a box calibration.
set -o pipefail
O=gpurun_out/r4det
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/diag_kernel_determinism.py > $O/kdet.log 2>&1 || { echo "KDET FAILED rc=$?"; tail -30 $O/kdet.log; exit 1; }
grep -E "NONDET|SUMMARY" $O/kdet.log || true
for run in a1 a2; do
  timeout -k 10 200 python -u scripts/diag_checksums.py run F $O/F_$run.json 2 > $O/F_$run.log 2>&1 || { echo "RUN $run FAILED"; tail -30 $O/F_$run.log; exit 1; }
done
HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 python -u scripts/diag_checksums.py run F $O/F_b1.json 2 > $O/F_b1.log 2>&1 || { echo "RUN b1 FAILED"; tail -30 $O/F_b1.log; exit 1; }
TDL_DETERMINISTIC=1 timeout -k 10 200 python -u scripts/diag_checksums.py run F $O/F_d1.json 2 > $O/F_d1.log 2>&1 || { echo "RUN d1 FAILED"; tail -30 $O/F_d1.log; exit 1; }
for p in "a1 a2" "a1 b1" "a2 b1" "a1 d1"; do
  set -- $p
  echo "== F $1 vs $2"
  python scripts/diag_checksums.py compare $O/F_$1.json $O/F_$2.json | head -20 || true
done
grep -i "warn\|nondetermin" $O/F_d1.log | sort | uniq -c | head -20 || true
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { echo BENCH FAILED; tail -20 $O/bench20.log; exit 1; }
tail -3 $O/bench20.log
echo done
