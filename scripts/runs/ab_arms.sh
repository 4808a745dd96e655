#!/bin/bash
# Same-box interleaved A/B of MNIST bench arms.  Usage: bash scripts/runs/ab_arms.sh <out> <reps> arm...
# arm = name=<snapshot dir or .>:<TDL_MNIST_VARIANT>   e.g. base=ab/base:0 cur=.:0 cur4=.:4
set -o pipefail
O=gpurun_out/${1:?out}; R=${2:?reps}; shift 2
mkdir -p $O
export TMPDIR=/tmp
res() { python3 -c "
import json,sys
d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$1'.split('/')[-1], d['value'], round(d['ms_per_step']*1e3,3))"; }
for i in $(seq 1 $R); do
for arm in "$@"; do
n=${arm%%=*}; rest=${arm#*=}; d=${rest%%:*}; v=${rest#*:}
TDL_MNIST_VARIANT=$v timeout -k 10 200 python $d/bench.py --gpus 1 --steps 1000 --warmup 20 > $O/b1000_${n}_$i.log 2>&1 || { echo BENCH FAILED; tail -20 $O/b1000_${n}_$i.log; exit 1; }
TDL_MNIST_VARIANT=$v timeout -k 10 200 python $d/bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_${n}_$i.log 2>&1 || { echo BENCH FAILED; tail -20 $O/b20_${n}_$i.log; exit 1; }
res $O/b1000_${n}_$i.log; res $O/b20_${n}_$i.log
done
done
for arm in "$@"; do
n=${arm%%=*}; rest=${arm#*=}; d=${rest%%:*}; v=${rest#*:}
TDL_MNIST_VARIANT=$v timeout -k 10 200 python $d/scripts/stamps_step.py > $O/step_$n.log 2>&1 || { echo STEP FAILED; tail -20 $O/step_$n.log; exit 1; }
echo "== $n"; grep -v amdgpu $O/step_$n.log | head -6
done
echo done
