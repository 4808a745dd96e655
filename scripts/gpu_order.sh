#!/bin/bash
O=gpurun_out/bnfuse
mkdir -p $O
for s in F,O F,T O,F T,F; do
  timeout -k 10 200 python -u scripts/diag_order.py $s > $O/o_$s.log 2>&1; grep -v Warning $O/o_$s.log | grep -v amdgpu.ids
done
