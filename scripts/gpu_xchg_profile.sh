#!/bin/bash
# R=2 replicas (per-replica batch 16, so both replicas' 4b workgroups are resident) on the box's one GPU: kernel trace of the bench with the gradient exchange inside the
# finalize launch (default) and with the serial standalone xGMI all-reduce (TDL_MNIST_FINALIZE_XCHG=0).
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export TDL_SHARE_GPU=1 TDL_MNIST_DP2_FWD=1
O=gpurun_out/xchg
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/fin -o run --output-format csv -- python3 bench.py --gpus 2 --per-replica-batch 16 --steps 20 --warmup 5 > $O/fin.log 2>&1
TDL_MNIST_FINALIZE_XCHG=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/ser -o run --output-format csv -- python3 bench.py --gpus 2 --per-replica-batch 16 --steps 20 --warmup 5 > $O/ser.log 2>&1
