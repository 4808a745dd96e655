#!/bin/bash
# Round 4: confirm the determinism fix (first conv cast to bf16 under mixed precision): per-op
# checksums async x2 vs launch-blocking, the pinned GPU tests, the kernel sweep (data rows only).
set -o pipefail
O=gpurun_out/r4det2
mkdir -p $O
export TMPDIR=/tmp
for run in a1 a2; do
  timeout -k 10 200 python -u scripts/diag_checksums.py run T $O/T_$run.json 2 > $O/T_$run.log 2>&1 || { echo "RUN $run FAILED"; tail -30 $O/T_$run.log; exit 1; }
done
HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 python -u scripts/diag_checksums.py run T $O/T_b1.json 2 > $O/T_b1.log 2>&1 || { echo "RUN b1 FAILED"; tail -30 $O/T_b1.log; exit 1; }
for p in "a1 a2" "a1 b1"; do
  set -- $p
  echo "== T $1 vs $2"
  python scripts/diag_checksums.py compare $O/T_$1.json $O/T_$2.json > $O/cmp_$1_$2.txt 2>&1; head -8 $O/cmp_$1_$2.txt
done
timeout -k 10 400 python -u -m pytest tests/test_slab_grad_gpu.py -x -v --timeout 300 --timeout-method thread > $O/slab_tests.log 2>&1 || { echo "SLAB TESTS FAILED"; tail -40 $O/slab_tests.log; exit 1; }
tail -3 $O/slab_tests.log
timeout -k 10 400 python -u scripts/diag_kernel_determinism.py > $O/kdet.log 2>&1 || { echo "KDET FAILED"; tail -30 $O/kdet.log; exit 1; }
grep -E "NONDET|SUMMARY" $O/kdet.log || true
timeout -k 10 600 python -u -m pytest tests/test_generic_multiproc_gpu.py -x -v --timeout 500 --timeout-method thread -k "autotune or R-2" > $O/multiproc.log 2>&1 || { echo "MULTIPROC FAILED"; tail -40 $O/multiproc.log; exit 1; }
tail -4 $O/multiproc.log
echo done
