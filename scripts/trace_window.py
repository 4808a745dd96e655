"""Steady-state kernel breakdown from a rocprofv3 kernel_trace.csv.

Takes the last ``--steps`` occurrences of a step-marker kernel (the first kernel of every step, a
name substring) and aggregates every dispatch between the first of those markers and the end of the
trace by kernel name.  Warm-up and solver-search dispatches (MIOpen find mode) fall outside the
window, which kernel_stats.csv cannot exclude.

    python scripts/trace_window.py run_kernel_trace.csv --marker distribution_elementwise --steps 3
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"^void ", "", n)
    return n[:90]


def category(name: str) -> str:
    n = name.lower()
    # the framework's own kernels first: their names contain "conv" / "gemm" as well
    if "tdl::" in n:
        if "conv" in n or "gemm" in n:
            return "tdl conv/gemm (hand-written)"
        return "tdl HIP kernels (bn/pool/other)"
    if "igemm" in n or "conv" in n or "gemm" in n or "cijk" in n:
        return "conv/gemm (library)"
    if "subtensor" in n or "fillbuffer" in n or "copybuffer" in n:
        return "MIOpen/runtime fill+cast"
    if "at::native" in n:
        return "torch elementwise/reduce"
    if "nccl" in n or "rccl" in n:
        return "rccl"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", required=True, help="substring of the first kernel of each step")
    ap.add_argument("--marker-grid-min", type=int, default=0, help="only marker dispatches with a grid >= this")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows)
             if a.marker in r["Kernel_Name"] and int(r.get("Grid_Size_X") or 0) >= a.marker_grid_min]
    # the window spans the last `steps` complete steps: marker[-steps-1] .. marker[-1]
    if len(marks) < a.steps + 1:
        raise SystemExit(f"only {len(marks)} marker dispatches")
    win = rows[marks[-a.steps - 1]:marks[-1]]
    t0 = int(win[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in win)
    busy = defaultdict(float)
    calls = defaultdict(int)
    cat = defaultdict(float)
    for r in win:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        k = short(r["Kernel_Name"])
        busy[k] += d
        calls[k] += 1
        cat[category(r["Kernel_Name"])] += d
    wall = (t1 - t0) / 1e3
    tot = sum(busy.values())
    print(f"window: {a.steps} steps, wall {wall / a.steps:.1f} us/step, kernel busy {tot / a.steps:.1f} us/step, "
          f"{len(win) // a.steps} dispatches/step, idle {100 * (1 - tot / wall):.1f}%")
    for c, v in sorted(cat.items(), key=lambda x: -x[1]):
        print(f"  {c:28s} {v / a.steps:10.1f} us/step {100 * v / tot:6.1f}%")
    print(f"{'kernel':90s} {'calls/step':>10s} {'us/step':>10s} {'pct':>6s}")
    for k, v in sorted(busy.items(), key=lambda x: -x[1])[: a.top]:
        print(f"{k:90s} {calls[k] / a.steps:10.1f} {v / a.steps:10.1f} {100 * v / tot:6.1f}")


if __name__ == "__main__":
    main()
