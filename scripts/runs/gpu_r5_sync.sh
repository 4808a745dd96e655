#!/bin/bash
# Host wait mode A/B at the driver's K=20: runtime default vs TDL_HIP_SCHEDULE=spin vs
# ROC_ACTIVE_WAIT_TIMEOUT=2000 (interleaved, 4 reps, plus one K=1000 each)
set -o pipefail
O=gpurun_out/r5sync
mkdir -p $O
export TMPDIR=/tmp
res() { python3 -c "
import json,sys
d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$1'.split('/')[-1], d['value'], round(d['ms_per_step']*1e3,3))"; grep -h "timed region" $1; }
for i in 1 2 3 4; do
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_def_$i.log 2>&1 || { echo FAILED; tail $O/b20_def_$i.log; exit 1; }
res $O/b20_def_$i.log
TDL_HIP_SCHEDULE=spin timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_spin_$i.log 2>&1 || { echo FAILED; tail $O/b20_spin_$i.log; exit 1; }
res $O/b20_spin_$i.log
ROC_ACTIVE_WAIT_TIMEOUT=2000 timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_awt_$i.log 2>&1 || { echo FAILED; tail $O/b20_awt_$i.log; exit 1; }
res $O/b20_awt_$i.log
done
TDL_HIP_SCHEDULE=spin timeout -k 10 200 python bench.py --gpus 1 --steps 1000 --warmup 20 > $O/b1000_spin.log 2>&1 && res $O/b1000_spin.log
timeout -k 10 200 python bench.py --gpus 1 --steps 1000 --warmup 20 > $O/b1000_def.log 2>&1 && res $O/b1000_def.log
python -c "import tensorflow_distributed_learning_amd as t; print('applied', t._hipsync.applied)"
TDL_HIP_SCHEDULE=spin python -c "import tensorflow_distributed_learning_amd as t; print('applied', t._hipsync.applied)"
echo done
