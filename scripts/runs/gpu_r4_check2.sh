#!/bin/bash
# continuation of gpu_r4_check.sh after the first failure: remaining GPU tests, smoke, benches
set -o pipefail
O=gpurun_out/r4check
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_resnet_multireplica_gpu.py tests/test_slab_grad_gpu.py tests/test_stem_gpu.py tests/test_xgmi_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests2.log 2>&1 || { echo "TESTS FAILED"; tail -60 $O/tests2.log; exit 1; }
tail -3 $O/tests2.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { echo BENCH FAILED; tail -20 $O/bench20.log; exit 1; }
tail -2 $O/bench20.log
timeout -k 10 200 python bench.py --gpus 1 --steps 1000 --warmup 20 > $O/bench1000.log 2>&1 || { echo BENCH1000 FAILED; tail -20 $O/bench1000.log; exit 1; }
tail -1 $O/bench1000.log
timeout -k 10 400 python scripts/bench_resnet50.py > $O/resnet.log 2>&1 || { echo RESNET FAILED; tail -20 $O/resnet.log; exit 1; }
tail -2 $O/resnet.log
timeout -k 10 300 python scripts/bench_comm_fixed.py > $O/comm_fixed.jsonl 2>$O/comm_fixed.err || { echo COMM FAILED; tail -20 $O/comm_fixed.err; exit 1; }
cat $O/comm_fixed.jsonl
echo done
