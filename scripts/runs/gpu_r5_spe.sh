#!/bin/bash
# steps per execution (graph size) at the driver's K=20 and at K=1000, interleaved, 3 reps
set -o pipefail
O=gpurun_out/r5spe
mkdir -p $O
export TMPDIR=/tmp
res() { python3 -c "
import json,sys
d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$1'.split('/')[-1], d['value'], round(d['ms_per_step']*1e3,3))"; }
for i in 1 2 3; do
for s in 20 10 5 4; do
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --steps-per-execution $s > $O/b20_s${s}_$i.log 2>&1 || { echo FAILED; tail $O/b20_s${s}_$i.log; exit 1; }
res $O/b20_s${s}_$i.log
done
done
for s in 50 20 10; do
timeout -k 10 200 python bench.py --gpus 1 --steps 1000 --warmup 20 --steps-per-execution $s > $O/b1000_s${s}.log 2>&1 || { echo FAILED; tail $O/b1000_s${s}.log; exit 1; }
res $O/b1000_s${s}.log
done
echo done
