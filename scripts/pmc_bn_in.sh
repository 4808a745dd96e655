#!/bin/bash
# PMC passes (counter collection only, no trace domains) over the plain vs input-side-BN 1x1 forward
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_bn_in
mkdir -p $OUT
i=0
for SET in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $SET -d $OUT/p$i -o run --output-format csv -- python scripts/microbench_bn_in.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail $OUT/p$i.log; exit 1; }
done
python scripts/pmc_summary.py $OUT
