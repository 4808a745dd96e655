#!/bin/bash
# Single-process (one host thread, G device graphs) vs one-process-per-replica bench at N=2 on the
# shared GPU; interleaved repeats.  Usage: scripts/runs/r6_single_vs_process.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r6_svp}
mkdir -p $OUT
export TDL_SHARE_GPU=1 TDL_XGMI_TIMEOUT=30
for rep in 1 2 3; do
  for cfg in "16 1" "64 0"; do
    set -- $cfg
    for mode in process single; do
      timeout -k 10 240 env TDL_MNIST_DP2_FWD=$2 python bench.py --gpus 2 --mode $mode --per-replica-batch $1 \
        --steps 200 --warmup 20 > $OUT/b${1}_dp$2_${mode}_$rep.json 2> $OUT/b${1}_dp$2_${mode}_$rep.err || exit 1
      python - "$OUT/b${1}_dp$2_${mode}_$rep.json" "$1 dp2=$2 $mode rep$rep" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
c = d["config"]
print(f"{sys.argv[2]:28s} {d['value']:12.1f} img/s {d['ms_per_step']:.4f} ms/step allreduce={c['allreduce']} identical={c['replicas_identical']}")
PY
    done
  done
done
