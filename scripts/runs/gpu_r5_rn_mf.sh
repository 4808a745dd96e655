#!/bin/bash
# ResNet-50 step A/B of the dma1 MFMA form (interleaved): 32x32x16 default, 16x16x32 (TDL_CONV_MFMA=16),
# 32x32x16 dma1 for every conv (TDL_CONV_IMPL=6)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5rnmf
mkdir -p $O
for i in 1 2; do
for arm in mf32 mf16 all32; do
  case $arm in mf32) E="";; mf16) E="TDL_CONV_MFMA=16";; all32) E="TDL_CONV_IMPL=6";; esac
  env $E timeout -k 10 400 python scripts/bench_resnet50.py --steps 20 --warmup 5 > $O/${arm}_$i.log 2>&1 || { echo "BENCH $arm FAILED"; tail -20 $O/${arm}_$i.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$O/${arm}_$i.log') if l.startswith('{')][-1]); print('$arm', $i, d['value'], d['ms_per_step'])"
done
done
