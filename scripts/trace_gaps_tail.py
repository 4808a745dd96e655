import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
ev = [e for e in ev if "tdl::" in e[2]]
N = int(sys.argv[2])  # number of trailing kernels (timed region)
ev = ev[-N:]
gaps = [(max(0, s1 - e0) / 1e3, i) for i, ((s0, e0, _), (s1, e1, n1)) in enumerate(zip(ev, ev[1:]))]
span = (ev[-1][1] - ev[0][0]) / 1e3
busy = sum((e - s) for s, e, _ in ev) / 1e3
big = sorted(gaps, reverse=True)[:10]
print(f"span {span:.1f} us busy {busy:.1f} us gaps {sum(g for g,_ in gaps):.1f} us; largest gaps (us, index): {[(round(g,1), i) for g, i in big]}")
