"""Per-dispatch SQ counters of one kernel from rocprofv3 --pmc counter_collection.csv files.

  python tools/sq_summary.py <csv> [<csv> ...] [--kernel fim2d_persist_kernel<double] [--label X]

Values are averaged over the kernel's dispatches (each counter summed over its dimensions within a
dispatch).  Derived: LDS bank-conflict share of LDS-array cycles, VALU / LDS busy per SIMD / CU
(256 CUs, 4 SIMDs each; GRBM_GUI_ACTIVE is summed over the 8 XCDs).
"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--kernel", default="fim2d_persist_kernel")
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    per = {}
    for fn in a.csv:
        with open(fn) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name") or ""
                if a.kernel not in name:
                    continue
                key = (fn, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                c = row["Counter_Name"]
                per.setdefault(c, {}).setdefault(key, 0.0)
                per[c][key] += float(row["Counter_Value"])
    out = {"label": a.label, "kernel": a.kernel}
    for c, d in sorted(per.items()):
        out[c] = sum(d.values()) / len(d)
        out.setdefault("dispatches", len(d))
    der = {}
    if "SQ_LDS_BANK_CONFLICT" in out and out.get("SQ_LDS_IDX_ACTIVE"):
        der["lds_bank_conflict_share"] = out["SQ_LDS_BANK_CONFLICT"] / out["SQ_LDS_IDX_ACTIVE"]
    if "GRBM_GUI_ACTIVE" in out:
        cyc = out["GRBM_GUI_ACTIVE"] / 8
        der["cycles_per_dispatch"] = cyc
        if "SQ_ACTIVE_INST_VALU" in out:
            der["valu_busy_per_simd"] = out["SQ_ACTIVE_INST_VALU"] / (cyc * 256)  # as profiles/r02_sq_counters.json
        if "SQ_LDS_IDX_ACTIVE" in out:
            der["lds_array_busy_per_cu"] = out["SQ_LDS_IDX_ACTIVE"] / (cyc * 256)
    out["derived"] = der
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
