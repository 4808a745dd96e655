set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
timeout -k 10 200 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc/p1 -o run --output-format csv -- python scripts/microbench_mnist.py --iters 5 > gpurun_out/pmc/p1.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr SQ_INSTS_VMEM SQ_INSTS_VALU_MFMA_F32 -d gpurun_out/pmc/p2 -o run --output-format csv -- python scripts/microbench_mnist.py --iters 5 > gpurun_out/pmc/p2.log 2>&1
echo rc=$?
ls gpurun_out/pmc/p1 gpurun_out/pmc/p2
