#!/bin/bash
# stamps + one bench pair of the current build
set -o pipefail
O=gpurun_out/${1:-r5st}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python scripts/stamps_mnist.py > $O/phases.log 2>&1 || { echo PH FAILED; tail -20 $O/phases.log; exit 1; }
grep -v amdgpu $O/phases.log
timeout -k 10 200 python scripts/stamps_step.py > $O/step.log 2>&1 || { echo STEP FAILED; tail -20 $O/step.log; exit 1; }
grep -v amdgpu $O/step.log | head -8
for K in 1000 20; do
timeout -k 10 200 python bench.py --gpus 1 --steps $K --warmup 20 > $O/b$K.log 2>&1 || { echo BENCH FAILED; tail -20 $O/b$K.log; exit 1; }
python3 -c "
import json
d=json.loads([l for l in open('$O/b$K.log') if l.startswith('{')][-1]); print('K=$K', d['value'], round(d['ms_per_step']*1e3,3))"
done
