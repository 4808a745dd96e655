set -o pipefail
mkdir -p gpurun_out/c2
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > gpurun_out/c2/test.log 2>&1 &&
timeout -k 10 200 python -u scripts/bench_conv.py 256 > gpurun_out/c2/conv_bench.jsonl 2>&1 &&
TDL_CONV=miopen timeout -k 10 300 python -u scripts/bench_resnet50.py --steps 20 --warmup 5 > gpurun_out/c2/rn_miopen.log 2>&1 &&
timeout -k 10 300 python -u scripts/bench_resnet50.py --steps 20 --warmup 5 > gpurun_out/c2/rn_auto.log 2>&1
