"""Timeline of the last N kernel dispatches of a rocprofv3 --kernel-trace run: each kernel's
duration and the idle gap before it (host-side stalls show as gaps).
  python tools/trace_gaps.py <dir> [N]"""
import csv, glob, os, sys

d = sys.argv[1]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 60
rows = []
for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    with open(fn) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70]))
rows.sort()
rows = rows[-N:]
prev = None
t0 = rows[0][0]
for s, e, k in rows:
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    print(f"{(s - t0) / 1e3:9.1f} us  gap {gap:8.1f}  dur {(e - s) / 1e3:8.1f}  {k}")
    prev = e
