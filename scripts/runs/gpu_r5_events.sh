#!/bin/bash
# K=20 bench with and without the device events inside the timed region (interleaved, 5 reps)
set -o pipefail
O=gpurun_out/r5ev
mkdir -p $O
export TMPDIR=/tmp
res() { python3 -c "
import json,sys
d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$1'.split('/')[-1], d['value'], round(d['ms_per_step']*1e3,3))"; grep -h "timed region" $1; }
for i in 1 2 3 4 5; do
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_noev_$i.log 2>&1 || { echo FAILED; tail $O/b20_noev_$i.log; exit 1; }
res $O/b20_noev_$i.log
TDL_BENCH_EVENTS=1 timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_ev_$i.log 2>&1 || { echo FAILED; tail $O/b20_ev_$i.log; exit 1; }
res $O/b20_ev_$i.log
done
echo done
