#!/bin/bash
# PMC passes (one counter group per run) over the hand-written conv forward of one compute-bound shape.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/convpmc
mkdir -p $O
SHAPE="14 14 256 256 3 1 1"
timeout -k 10 120 python scripts/conv_one.py $SHAPE > $O/time.txt 2>&1 || exit 1
timeout -k 10 120 python scripts/conv_one.py 28 28 128 128 3 1 1 >> $O/time.txt 2>&1 || exit 1
timeout -k 10 120 python scripts/conv_one.py 7 7 512 512 3 1 1 >> $O/time.txt 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES -d $O/p1 -o run --output-format csv -- python3 scripts/conv_one.py $SHAPE 256 10 > $O/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/p2 -o run --output-format csv -- python3 scripts/conv_one.py $SHAPE 256 10 > $O/p2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_LDS_DATA_FIFO_FULL SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d $O/p3 -o run --output-format csv -- python3 scripts/conv_one.py $SHAPE 256 10 > $O/p3.log 2>&1
