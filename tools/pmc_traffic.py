"""Per-launch HBM-side traffic of the solver kernel from two rocprofv3 --pmc passes.

  rocprofv3 --pmc FETCH_SIZE --kernel-trace -d <dir_f> -- python bench.py ...
  rocprofv3 --pmc WRITE_SIZE --kernel-trace -d <dir_w> -- python bench.py ...
  python tools/pmc_traffic.py <dir_f> <dir_w> [kernel substring] [dtype] > profiles/pmc_traffic_<dtype>.json

FETCH_SIZE / WRITE_SIZE are kilobytes at the L2's memory side (TCC_EA0_RDREQ / _WRREQ;
Infinity-Cache hits included).  gfx950 correction (MI355X_MICROARCH.md, HBM section):
FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced reads -> x2; WRITE_SIZE is exact
for 16 B/lane stores.  The solver's T/cost traffic is 16 B/lane, so both corrections apply as is.
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter, kernel):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
                if kernel not in name or row.get("Counter_Name") != counter:
                    continue
                key = (fn, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for kernel '{kernel}' under {d}")
    return vals


def main():
    dir_f, dir_w = sys.argv[1], sys.argv[2]
    kernel = sys.argv[3] if len(sys.argv) > 3 else "fim2d_persist_kernel"
    dtype = sys.argv[4] if len(sys.argv) > 4 else ("f64" if "double" in kernel else "f32")
    f = per_dispatch(dir_f, "FETCH_SIZE", kernel)
    w = per_dispatch(dir_w, "WRITE_SIZE", kernel)
    fetch_kb = sum(f.values()) / len(f)
    write_kb = sum(w.values()) / len(w)
    out = {
        "kernel": kernel,
        "dtype": dtype,
        "dispatches": {"fetch_pass": len(f), "write_pass": len(w)},
        "fetch_size_kb_raw": round(fetch_kb, 1),
        "write_size_kb_raw": round(write_kb, 1),
        "fetch_bytes": round(fetch_kb * 1024 * 2),  # gfx950: x2 for 16 B/lane reads
        "write_bytes": round(write_kb * 1024),
        "bytes_per_launch": round(fetch_kb * 1024 * 2 + write_kb * 1024),
        "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); WRITE_SIZE as is",
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
