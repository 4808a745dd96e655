set -o pipefail
mkdir -p gpurun_out/c9
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py > gpurun_out/c9/test.log 2>&1
timeout -k 10 200 python -u scripts/bench_conv.py 256 > gpurun_out/c9/conv_bench.jsonl 2>&1
bash scripts/pmc_conv.sh pmc_conv2 > gpurun_out/c9/pmc.txt 2>&1
