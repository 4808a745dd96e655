#!/bin/bash
# K=20 bench: default vs HSA_ENABLE_INTERRUPT=0 (signal waits poll) vs that + TDL_HIP_SCHEDULE=spin,
# interleaved, 4 reps; then the launch trace with HSA_ENABLE_INTERRUPT=0
set -o pipefail
O=gpurun_out/r5intr
mkdir -p $O
export TMPDIR=/tmp
res() { python3 -c "
import json,sys
d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$1'.split('/')[-1], d['value'], round(d['ms_per_step']*1e3,3))"; }
for i in 1 2 3 4; do
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_def_$i.log 2>&1 || { echo FAILED; tail $O/b20_def_$i.log; exit 1; }
res $O/b20_def_$i.log
HSA_ENABLE_INTERRUPT=0 timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_poll_$i.log 2>&1 || { echo FAILED; tail $O/b20_poll_$i.log; exit 1; }
res $O/b20_poll_$i.log
HSA_ENABLE_INTERRUPT=0 TDL_HIP_SCHEDULE=spin timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_pollspin_$i.log 2>&1 || { echo FAILED; tail $O/b20_pollspin_$i.log; exit 1; }
res $O/b20_pollspin_$i.log
done
HSA_ENABLE_INTERRUPT=0 timeout -k 10 200 python bench.py --gpus 1 --steps 1000 --warmup 20 > $O/b1000_poll.log 2>&1 && res $O/b1000_poll.log
HSA_ENABLE_INTERRUPT=0 timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d $O/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo PROF FAILED; tail -20 $O/prof.log; exit 1; }
python3 scripts/launch_trace.py $O/prof
echo done
