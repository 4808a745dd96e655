#!/bin/bash
set -o pipefail
# A/B of the fused MNIST engine's graph variants: at R=2 (two replica processes sharing the GPU)
# the serial vs side-stream-overlapped gradient all-reduce; R=4; forced in-forward dP2 at R=2
OUT=gpurun_out/${1:-mnist_ab}; mkdir -p $OUT; export TMPDIR=/tmp
for cfg in "python bench.py --steps 1000 --warmup 100" "TDL_SHARE_GPU=1 TDL_OVERLAP_ALLREDUCE=1 python bench.py --gpus 2 --steps 500 --warmup 50" "TDL_SHARE_GPU=1 TDL_OVERLAP_ALLREDUCE=0 python bench.py --gpus 2 --steps 500 --warmup 50" "TDL_SHARE_GPU=1 python bench.py --gpus 4 --steps 300 --warmup 30" "TDL_SHARE_GPU=1 TDL_MNIST_DP2_FWD=1 python bench.py --gpus 2 --per-replica-batch 16 --steps 200 --warmup 20"; do
  echo "== $cfg" >> $OUT/ab.txt
  timeout -k 10 300 env $cfg > $OUT/one.log 2>&1 || { echo FAILED $cfg; tail -20 $OUT/one.log; exit 1; }
  tail -1 $OUT/one.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config'].get('allreduce'), d['config'].get('replicas_identical'))" >> $OUT/ab.txt
done
cat $OUT/ab.txt
