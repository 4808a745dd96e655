"""Per-kernel duration and idle gap before it, from a rocprofv3 kernel_trace.csv (tdl kernels only
unless --all).  The gap column shows launch/dependency bubbles between consecutive kernels."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
keep_all = "--all" in sys.argv
ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
if not keep_all:
    ev = [e for e in ev if "tdl::" in e[2]]
ev = ev[len(ev) // 10:]  # skip warm-up
dur, gap = defaultdict(list), defaultdict(list)
for (s0, e0, _), (s1, e1, n1) in zip(ev, ev[1:]):
    gap[n1].append(max(0, s1 - e0) / 1e3)
for s, e, n in ev:
    dur[n].append((e - s) / 1e3)
span = (ev[-1][1] - ev[0][0]) / 1e3
print(f"{'kernel':48s} {'n':>6s} {'dur_us':>8s} {'gap_us':>8s} {'gap_med':>8s}")
tot_d = tot_g = 0.0
for n in sorted(dur, key=lambda k: -sum(dur[k])):
    d, g = dur[n], sorted(gap.get(n, [0.0]))
    tot_d += sum(d)
    tot_g += sum(g)
    short = n.replace("tdl::", "").split("(")[0][:48]
    print(f"{short:48s} {len(d):6d} {sum(d)/len(d):8.2f} {sum(g)/len(g):8.2f} {g[len(g)//2]:8.2f}")
print(f"span {span:.0f} us: busy {tot_d:.0f} us ({100*tot_d/span:.1f}%), gaps {tot_g:.0f} us")
