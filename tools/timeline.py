"""Timeline of one planner step 1 call from a rocprofv3 --kernel-trace --memory-copy-trace CSV run
(tools/gpu_r04l.sh): every kernel and copy of the LAST eik_rover_path_f64 call (from its DEM upload
to the last path kernel), start offsets and durations in microseconds, and the gaps between them."""
import csv, glob, sys

d = sys.argv[1]
ev = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"][:70]))
for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C " + r.get("Direction", "?") + " " + r.get("Bytes", r.get("Size", "?"))))
ev.sort()
# the last call: the last cm_min_kernel (first costmap kernel) ... the last gdm2d_kernel end
mins = [i for i, e in enumerate(ev) if "cm_min_kernel" in e[2]]
gdm = [i for i, e in enumerate(ev) if "gdm2d_kernel" in e[2]]
i0 = mins[-1]
while i0 > 0 and ("copyBuffer" in ev[i0 - 1][2] or ev[i0 - 1][2].startswith("C ")) and ev[i0][0] - ev[i0 - 1][1] < 2_000_000:
    i0 -= 1
i1 = gdm[-1]
t0 = ev[i0][0]
prev_end = t0
for s, e, n in ev[i0:i1 + 1]:
    gap = (s - prev_end) / 1e3
    print(f"{(s - t0) / 1e3:9.1f} +{(e - s) / 1e3:8.1f}  gap {gap:7.1f}  {n}")
    prev_end = max(prev_end, e)
print(f"total {(ev[i1][1] - t0) / 1e3:.1f} us")
