#!/bin/bash
set -o pipefail
O=gpurun_out/r3b_end
timeout -k 10 300 python -u -m pytest -v --timeout 280 --timeout-method thread tests/test_slab_grad_gpu.py -k projection > $O/t1.log 2>&1; tail -3 $O/t1.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread --deselect tests/test_slab_grad_gpu.py::test_fused_bn_backward_projection_shortcut_and_stride2 -p no:cacheprovider > $O/tests_rest.log 2>&1; tail -2 $O/tests_rest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1; tail -1 $O/bench.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_k20.log 2>&1; tail -1 $O/bench_k20.log
