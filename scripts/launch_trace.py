"""Host-API vs kernel timeline of the last hipGraphLaunch in a rocprofv3 --kernel-trace --hip-trace
run: graph-launch call -> first kernel start, kernel span, last kernel end -> the next synchronize's
return.  Usage: python scripts/launch_trace.py <rocprofv3 output dir>"""
import csv
import glob
import sys


def rows(pattern):
    fs = glob.glob(pattern, recursive=True)
    return list(csv.DictReader(open(fs[0]))) if fs else []


def main(d):
    ks = rows(f"{d}/**/*kernel_trace.csv")
    api = rows(f"{d}/**/*hip_api_trace.csv")
    ks.sort(key=lambda r: int(r["Start_Timestamp"]))
    api.sort(key=lambda r: int(r["Start_Timestamp"]))
    launches = [r for r in api if r["Function"].startswith("hipGraphLaunch")]
    if not launches:
        print("no hipGraphLaunch in the trace")
        return
    gl = launches[-1]
    g0, g1 = int(gl["Start_Timestamp"]), int(gl["End_Timestamp"])
    after = [r for r in ks if int(r["Start_Timestamp"]) >= g0]
    mine = [r for r in after if "k_fwd_conv" in r["Kernel_Name"] or "finalize" in r["Kernel_Name"]]
    k0, k1 = int(mine[0]["Start_Timestamp"]), int(mine[-1]["End_Timestamp"])
    syncs = [r for r in api if "ynchronize" in r["Function"] and int(r["Start_Timestamp"]) >= g0]
    print(f"hipGraphLaunch call: {(g1 - g0) / 1e3:.1f} us; its kernels: {len(mine)}")
    print(f"launch call start -> first kernel start: {(k0 - g0) / 1e3:.1f} us")
    print(f"launch call end   -> first kernel start: {(k0 - g1) / 1e3:.1f} us")
    print(f"kernel span (first start -> last end): {(k1 - k0) / 1e3:.1f} us")
    for s in syncs[:3]:
        s0, s1 = int(s["Start_Timestamp"]), int(s["End_Timestamp"])
        print(f"{s['Function']}: called {(s0 - k1) / 1e3:+.1f} us vs last kernel end, returned {(s1 - k1) / 1e3:+.1f} us")
    prev = [r for r in api if int(r["End_Timestamp"]) <= g0][-6:]
    for r in prev:
        print(f"  before launch: {r['Function']} ends {(int(r['End_Timestamp']) - g0) / 1e3:+.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
