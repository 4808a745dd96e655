"""Average PMC counters per tdl kernel over all passes under a directory."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "tdl::" not in n:
            continue
        n = n.replace("(anonymous namespace)::", "").replace("void ", "", 1)
        agg[n.split("(")[0].replace("tdl::", "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    d = {c: sum(x) / len(x) for c, x in v.items()}
    w = d.get("SQ_WAVES", 1)
    print(k)
    print("   " + "  ".join(f"{c.replace('SQ_', '')}={val:,.0f}" for c, val in sorted(d.items())))
    if "SQ_WAVE_CYCLES" in d:
        wc = d["SQ_WAVE_CYCLES"]
        print(f"   per-wave: cycles={4 * wc / max(w, 1):,.0f}  wait_any={d['SQ_WAIT_ANY'] / wc:.0%}  "
              f"wait_inst={d['SQ_WAIT_INST_ANY'] / wc:.0%}  active={d['SQ_ACTIVE_INST_ANY'] / wc:.0%}  "
              f"wait_lds={d['SQ_WAIT_INST_LDS'] / wc:.0%}")
