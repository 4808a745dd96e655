set -o pipefail
mkdir -p gpurun_out/diag1
for k in 20 200 1000; do
  TDL_HOST_TIMING=1 timeout -k 10 120 python bench.py --steps $k --warmup 5 > gpurun_out/diag1/k$k.log 2>&1 || exit 1
  grep -E "timed region|host us" gpurun_out/diag1/k$k.log; tail -1 gpurun_out/diag1/k$k.log | cut -c1-200
done
