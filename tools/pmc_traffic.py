"""Per-launch memory-side traffic of a kernel from rocprofv3 --pmc passes (separate runs).

  rocprofv3 --pmc TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B --kernel-trace -d <dir_r> -- python ...
  rocprofv3 --pmc TCC_EA0_WRREQ TCC_EA0_WRREQ_64B --kernel-trace -d <dir_w> -- python ...
  python tools/pmc_traffic.py <dir_r> <dir_w> [kernel substring] [dtype] > profiles/pmc_traffic_<cfg>.json

Bytes from the L2's memory-side request counters by request size (round 6): reads = 32 x RDREQ_32B +
64 x RDREQ_64B + 128 x RDREQ_128B, writes = 64 x WRREQ_64B + 32 x (WRREQ - WRREQ_64B).  (Rounds 1-5
used FETCH_SIZE x 2 + WRITE_SIZE: FETCH_SIZE tallies every non-32-B request at 64 B, so doubling it is
right only when all reads are 128-B requests -- MI355X_MICROARCH.md, HBM section.)  Directories of
FETCH_SIZE / WRITE_SIZE passes are still accepted and reduced the old way.
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counters, kernel):
    """{counter: {dispatch: value}} for the kernel's dispatches under d (rows of one counter summed)."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = {c: {} for c in counters}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
                c = row.get("Counter_Name")
                if kernel not in name or c not in vals:
                    continue
                key = (fn, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                vals[c][key] = vals[c].get(key, 0.0) + float(row["Counter_Value"])
    return {c: v for c, v in vals.items() if v}


def avg(v):
    return sum(v.values()) / len(v)


def main():
    dir_r, dir_w = sys.argv[1], sys.argv[2]
    kernel = sys.argv[3] if len(sys.argv) > 3 else "fim2d_persist_kernel"
    dtype = sys.argv[4] if len(sys.argv) > 4 else ("f64" if "double" in kernel else "f32")
    r = per_dispatch(dir_r, ["TCC_EA0_RDREQ_32B", "TCC_EA0_RDREQ_64B", "TCC_EA0_RDREQ_128B", "FETCH_SIZE"], kernel)
    w = per_dispatch(dir_w, ["TCC_EA0_WRREQ", "TCC_EA0_WRREQ_64B", "WRITE_SIZE"], kernel)
    out = {"kernel": kernel, "dtype": dtype}
    if "TCC_EA0_RDREQ_128B" in r and "TCC_EA0_WRREQ" in w:
        n32, n64, n128 = (avg(r.get(k, {0: 0.0})) for k in ("TCC_EA0_RDREQ_32B", "TCC_EA0_RDREQ_64B", "TCC_EA0_RDREQ_128B"))
        wr, wr64 = avg(w["TCC_EA0_WRREQ"]), avg(w.get("TCC_EA0_WRREQ_64B", {0: 0.0}))
        fb, wb = 32 * n32 + 64 * n64 + 128 * n128, 64 * wr64 + 32 * (wr - wr64)
        out.update({"dispatches": {"read_pass": len(r["TCC_EA0_RDREQ_128B"]), "write_pass": len(w["TCC_EA0_WRREQ"])},
                    "read_requests": {"32B": round(n32), "64B": round(n64), "128B": round(n128)},
                    "write_requests": {"all": round(wr), "64B": round(wr64)},
                    "fetch_bytes": round(fb), "write_bytes": round(wb), "bytes_per_launch": round(fb + wb),
                    "method": "TCC_EA0 request counters by size (exact bytes at the L2's memory side)"})
    else:
        fetch_kb, write_kb = avg(r["FETCH_SIZE"]), avg(w["WRITE_SIZE"])
        out.update({"dispatches": {"fetch_pass": len(r["FETCH_SIZE"]), "write_pass": len(w["WRITE_SIZE"])},
                    "fetch_size_kb_raw": round(fetch_kb, 1), "write_size_kb_raw": round(write_kb, 1),
                    "fetch_bytes": round(fetch_kb * 1024 * 2), "write_bytes": round(write_kb * 1024),
                    "bytes_per_launch": round(fetch_kb * 1024 * 2 + write_kb * 1024),
                    "method": "FETCH_SIZE x 2 + WRITE_SIZE (assumes 128-B read requests)"})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
