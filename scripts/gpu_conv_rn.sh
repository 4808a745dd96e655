set -o pipefail
OUT=gpurun_out/c7
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > $OUT/test.log 2>&1 &&
timeout -k 10 300 python -u scripts/bench_resnet50.py --steps 20 --warmup 5 > $OUT/rn_auto.log 2>&1 &&
TDL_CONV=miopen timeout -k 10 300 python -u scripts/bench_resnet50.py --steps 20 --warmup 5 > $OUT/rn_miopen.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python scripts/bench_resnet50.py --steps 5 --warmup 3 > $OUT/prof.log 2>&1 &&
python scripts/prof_summary.py $OUT/prof/run_kernel_stats.csv 40 > $OUT/kernel_stats.txt
