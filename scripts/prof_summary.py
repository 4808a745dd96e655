"""Summarise a rocprofv3 kernel_stats.csv: name, calls, avg/min us, share."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
print(f"{'kernel':70s} {'calls':>7s} {'avg_us':>8s} {'min_us':>8s} {'pct':>6s}")
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 15]:
    print(f"{r['Name'][:70]:70s} {r['Calls']:>7s} {float(r['AverageNs'])/1e3:8.2f} {float(r['MinNs'])/1e3:8.2f} {float(r['Percentage']):6.2f}")
