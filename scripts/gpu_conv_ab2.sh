set -o pipefail
mkdir -p gpurun_out/c5
TDL_CONV=hip TDL_GRAPH_STEP=0 timeout -k 10 200 python -u scripts/bench_resnet50.py --steps 10 --warmup 3 > gpurun_out/c5/hip_eager.log 2>&1 &&
TDL_CONV=hip timeout -k 10 200 python -u scripts/bench_resnet50.py --steps 10 --warmup 3 > gpurun_out/c5/hip_graph.log 2>&1 &&
TDL_CONV=miopen timeout -k 10 200 python -u scripts/bench_resnet50.py --steps 10 --warmup 3 > gpurun_out/c5/miopen_graph.log 2>&1
