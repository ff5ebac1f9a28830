"""Raw TCC counters of the solver kernel, per dispatch (rocprofv3 --pmc <counters> passes), and the
memory-side bytes they imply without FETCH_SIZE's width assumption:
  read bytes  = 32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B
  write bytes = 64 x WRREQ_64B + 32 x (WRREQ - WRREQ_64B)
  python tools/pmc_raw.py "<kernel substring>" <dir> [<dir> ...] > summary.json
"""
import csv
import glob
import json
import os
import sys


def main():
    kernel, dirs = sys.argv[1], sys.argv[2:]
    per = {}  # counter -> {dispatch: value}
    for d in dirs:
        for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(fn) as f:
                for row in csv.DictReader(f):
                    name = row.get("Kernel_Name") or ""
                    if kernel not in name:
                        continue
                    c = row.get("Counter_Name", "")
                    key = (fn, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                    per.setdefault(c, {})
                    per[c][key] = per[c].get(key, 0.0) + float(row["Counter_Value"])
    avg = {c: sum(v.values()) / len(v) for c, v in per.items() if v}
    out = {"kernel": kernel, "dispatches": {c: len(v) for c, v in per.items()}, "per_launch": avg}
    g = avg.get
    if all(k in avg for k in ("TCC_EA0_RDREQ_32B", "TCC_EA0_RDREQ_64B", "TCC_EA0_RDREQ_128B")):
        out["read_bytes"] = 32 * g("TCC_EA0_RDREQ_32B") + 64 * g("TCC_EA0_RDREQ_64B") + 128 * g("TCC_EA0_RDREQ_128B")
    if "TCC_EA0_WRREQ" in avg and "TCC_EA0_WRREQ_64B" in avg:
        out["write_bytes"] = 64 * g("TCC_EA0_WRREQ_64B") + 32 * (g("TCC_EA0_WRREQ") - g("TCC_EA0_WRREQ_64B"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
