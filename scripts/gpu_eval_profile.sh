set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/evprof
timeout -k 10 200 python scripts/eval_profile.py > gpurun_out/evprof/run.log 2>&1 || { tail -20 gpurun_out/evprof/run.log; exit 1; }
tail -1 gpurun_out/evprof/run.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/evprof/prof -o run --output-format csv -- python scripts/eval_profile.py > gpurun_out/evprof/prof.log 2>&1 || { tail -20 gpurun_out/evprof/prof.log; exit 1; }
python scripts/prof_summary.py gpurun_out/evprof/prof/run_kernel_stats.csv 20
