#!/bin/bash
# Round 5 baseline: MNIST bench K=20/K=1000 + whole-step and fused-kernel phase stamps
set -o pipefail
O=gpurun_out/r5base
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { echo BENCH FAILED; tail -20 $O/bench20.log; exit 1; }
tail -2 $O/bench20.log
timeout -k 10 200 python bench.py --gpus 1 --steps 1000 --warmup 20 > $O/bench1000.log 2>&1 || { echo BENCH1000 FAILED; tail -20 $O/bench1000.log; exit 1; }
tail -1 $O/bench1000.log | cut -c1-300
timeout -k 10 200 python scripts/stamps_step.py > $O/step.log 2>&1 || { echo STEP FAILED; tail -20 $O/step.log; exit 1; }
cat $O/step.log
timeout -k 10 200 python scripts/stamps_mnist.py > $O/phases.log 2>&1 || { echo PH FAILED; tail -20 $O/phases.log; exit 1; }
cat $O/phases.log

# eager (no hipGraph) vs graph at the driver's K=20, interleaved
for i in 1 2; do
timeout -k 10 200 env TDL_GRAPH=0 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20_eager$i.log 2>&1 || { echo EAGER FAILED; tail -20 $O/bench20_eager$i.log; exit 1; }
echo "eager $i: $(tail -1 $O/bench20_eager$i.log | cut -c1-200)"; grep "timed region" $O/bench20_eager$i.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20_graph$i.log 2>&1 || { echo GRAPH FAILED; tail -20 $O/bench20_graph$i.log; exit 1; }
echo "graph $i: $(tail -1 $O/bench20_graph$i.log | cut -c1-200)"; grep "timed region" $O/bench20_graph$i.log
done
echo done
