#!/bin/bash
# PMC counter passes over the generic-engine reference-CNN step (bench.py --engine generic) (kernel-trace + --pmc only; no sys/runtime trace).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_generic}
mkdir -p $OUT
i=0
for SET in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $SET -d $OUT/p$i -o run --output-format csv -- python bench.py --engine generic --steps 50 --warmup 10 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail $OUT/p$i.log; exit 1; }
done
python scripts/pmc_summary.py $OUT
