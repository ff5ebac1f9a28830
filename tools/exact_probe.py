"""Probe of the exact band replay on one fixture (EIK_OPT_EXACT_BAND, csrc/bidir_exact.hip): runs
FastMarching3D's early exit (3D fixtures) or biComputeTmap (2D) with EIK_EXACT_DEBUG's per-pass trace
and reports the result against the reference's output.
  EIK_EXACT_DEBUG=1 python tools/exact_probe.py fm3d_early c3_
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "planning-motion_planning_amd"))
import eikonal  # noqa: E402
from eikonal import _lib as L  # noqa: E402


def main():
    name, p = sys.argv[1], sys.argv[2]
    d = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"), allow_pickle=False)
    c = eikonal.Context(0)
    c.set_option(L.OPT_EXACT_BAND, 1)
    cost = d[p + "cost"].astype(np.float64)
    try:
        if name == "fmm2d_bidir":
            TG, TS, j = c.tmap2d_bidir(cost, d[p + "goal"], d[p + "start"])
            out = {"join": j.tolist(), "ref_join": d[p + "join"].tolist()}
            pairs = ((TG, d[p + "TG"]), (TS, d[p + "TS"]))
        else:
            T = c.tmap3d(cost, d[p + "goal"], start=d[p + "start"])
            out = {}
            pairs = ((T, d[p + "T_early"]),)
        for k, (A, B) in enumerate(pairs):
            fa, fb = np.isfinite(A), np.isfinite(B)
            both = fa & fb
            out[f"field{k}"] = {"mask_diff": int((fa != fb).sum()), "value_diff": int((A[both] != B[both]).sum()),
                                "max_abs": float(np.abs(A[both] - B[both]).max()) if both.any() else 0.0}
        out["info"] = c.exact_info()
        # a second identical call: the steady-state cost (the first pays the kernels' first launches)
        if name == "fmm2d_bidir":
            c.tmap2d_bidir(cost, d[p + "goal"], d[p + "start"])
        else:
            c.tmap3d(cost, d[p + "goal"], start=d[p + "start"])
        out["ms_second_call"] = c.exact_info()["ms"]
    except eikonal.EikError as e:
        out = {"error": str(e)}
    print(name, p, out, flush=True)
    c.close()


if __name__ == "__main__":
    main()
