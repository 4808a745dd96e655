#!/bin/bash
# SGD kernels zero the gradient slab after reading it (the generic trainer then skips its per-step fill):
# generic-engine / fit / multi-replica GPU tests, then the generic bench.  Usage: OUTDIR
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6zg}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fit_gpu.py tests/test_generic_device_gpu.py tests/test_conv_pool_f32_gpu.py tests/test_local_replicas_gpu.py tests/test_generic_multiproc_gpu.py tests/test_resnet_multireplica_gpu.py tests/test_slab_grad_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
for r in 1 2; do
for v in reference same dropout; do
  timeout -k 10 300 python bench.py --engine generic --variant $v --steps 200 --warmup 25 > $O/g_${v}_$r.json 2> $O/g_${v}_$r.err || { tail -20 $O/g_${v}_$r.err; exit 1; }
  echo "$v $r $(grep -o '"ms_per_step": [0-9.]*' $O/g_${v}_$r.json)"
done
done
