#!/bin/bash
# Same-box A/B of the MNIST bench: ab/base (snapshot, scripts/ab_snapshot.sh) vs the current build,
# interleaved, K=1000 and K=20, then the step stamps of each.  Usage: bash scripts/runs/ab_mnist.sh <out> [reps]
set -o pipefail
O=gpurun_out/${1:?out}
R=${2:-3}
mkdir -p $O
export TMPDIR=/tmp
res() { python3 -c "
import json,sys
d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$1'.split('/')[-1], d['value'], round(d['ms_per_step']*1e3,3))"; }
for i in $(seq 1 $R); do
for v in base cur; do
B=bench.py; [ $v = base ] && B=ab/base/bench.py
timeout -k 10 200 python $B --gpus 1 --steps 1000 --warmup 20 > $O/b1000_${v}_$i.log 2>&1 || { echo BENCH FAILED; tail -20 $O/b1000_${v}_$i.log; exit 1; }
timeout -k 10 200 python $B --gpus 1 --steps 20 --warmup 5 > $O/b20_${v}_$i.log 2>&1 || { echo BENCH FAILED; tail -20 $O/b20_${v}_$i.log; exit 1; }
res $O/b1000_${v}_$i.log; res $O/b20_${v}_$i.log
done
done
for v in base cur; do
S=scripts; [ $v = base ] && S=ab/base/scripts
timeout -k 10 200 python $S/stamps_step.py > $O/step_$v.log 2>&1 || { echo STEP FAILED; tail -20 $O/step_$v.log; exit 1; }
timeout -k 10 200 python $S/stamps_mnist.py > $O/phases_$v.log 2>&1 || { echo PH FAILED; tail -20 $O/phases_$v.log; exit 1; }
echo "== $v"; grep -v amdgpu $O/step_$v.log | head -12; grep -v amdgpu $O/phases_$v.log | head -8
done
echo done
