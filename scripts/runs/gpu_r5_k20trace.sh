#!/bin/bash
# kernel trace of the driver's K=20 bench: per-kernel start/end of the timed region's 40 dispatches
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5k20
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo PROF FAILED; tail -20 $O/prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r5k20/prof/*kernel_trace.csv")[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ks = [r for r in rows if "k_fwd_conv" in r["Kernel_Name"] or "finalize" in r["Kernel_Name"]]
last = ks[-40:]
t0 = int(last[0]["Start_Timestamp"])
prev = None
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev else 0.0
    print(f'{r["Kernel_Name"][:28]:28s} start {(s - t0) / 1000:8.2f} us  dur {(e - s) / 1000:6.2f}  gap {gap:5.2f}')
    prev = e
print("region (first start -> last end):", (int(last[-1]["End_Timestamp"]) - t0) / 1000, "us")
PY
