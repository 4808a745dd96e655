"""Per-dispatch listing of one steady-state step from a rocprofv3 kernel_trace.csv: every kernel
between the last two occurrences of a step-marker kernel, in order, with its grid (workgroups),
workgroup size and duration -- the per-call view behind trace_window.py's per-name totals (the
grid of a conv dispatch identifies its shape: M/BM x K/BN tiles).

    python scripts/trace_calls.py run_kernel_trace.csv --marker k_sgd_momentum [--min-us 20]
"""
import argparse
import csv
import re


def short(name: str) -> str:
    n = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))
    return re.sub(r"^void ", "", n)[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="k_sgd_momentum")
    ap.add_argument("--min-us", type=float, default=0.0)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(idx) < 2:
        raise SystemExit("fewer than two markers in the trace")
    step = rows[idx[-2]:idx[-1]]
    tot = 0.0
    for k, r in enumerate(step):
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += d
        wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) // max(wg, 1)
        if d >= a.min_us:
            print(f"{k:4d} {short(r['Kernel_Name']):60s} wgs {grid:7d} x {wg:4d}  {d:8.1f} us")
    print(f"step: {len(step)} dispatches, {tot:.1f} us kernel time")


if __name__ == "__main__":
    main()
