#!/bin/bash
# steps per execution at K=1000: 50 / 25 / 20, interleaved, 3 reps
set -o pipefail
O=gpurun_out/r5spe2
mkdir -p $O
export TMPDIR=/tmp
res() { python3 -c "
import json,sys
d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$1'.split('/')[-1], d['value'], round(d['ms_per_step']*1e3,3))"; }
for i in 1 2 3; do
for s in 50 25 20; do
timeout -k 10 200 python bench.py --gpus 1 --steps 1000 --warmup 20 --steps-per-execution $s > $O/b1000_s${s}_$i.log 2>&1 || { echo FAILED; tail $O/b1000_s${s}_$i.log; exit 1; }
res $O/b1000_s${s}_$i.log
done
done
echo done
