#!/bin/bash
# K=20 (the driver's bench setting): steps per execution sweep, 3 runs each
set -o pipefail
OUT=gpurun_out/${1:-spe20}; mkdir -p $OUT; export TMPDIR=/tmp
for spe in 20 10 5 4; do
  for i in 1 2 3; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --steps-per-execution $spe > $OUT/one.log 2>&1 || { echo FAILED; tail -20 $OUT/one.log; exit 1; }
    echo "spe=$spe $(grep '^timed region' $OUT/one.log | tail -1) $(tail -1 $OUT/one.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $OUT/spe.txt
  done
done
cat $OUT/spe.txt
