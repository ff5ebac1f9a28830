"""Row-pitch probe of the C2 hop chain (a visit's write-back drain of 64 rows
x 512 B took ~9 us, and tile rows sit W x sizeof(R) = 32 KiB apart in the 4096-wide raster).

Solves bench.py's C2 raster (terrain seed 42, 4096^2, goal at the centre) as is and widened with
+inf columns on the east (inert tiles: never activated), so every tile row's address stride changes
while the front's work stays the same.  If the drain is slow because of the power-of-two stride
(rows of a tile falling on few HBM channels), the widened rasters solve faster per tile visit.

  python tools/pitch_probe.py [--dtype f64|f32] [--reps 7] [--pads 0,16,64,128]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "planning-motion_planning_amd"))
import eikonal  # noqa: E402
from eikonal import _lib as L  # noqa: E402
from eikonal import terrain  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--pads", default="0,16,64,128,192")
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    f64 = args.dtype == "f64"
    tdt = torch.float64 if f64 else torch.float32
    edt = L.EIK_F64 if f64 else L.EIK_F32
    N = 4096
    base = terrain.cost_block(0, 0, N, N, N, N, seed=42, device=dev).to(tdt)
    goal = (N // 2, N // 2)
    ctx = eikonal.Context(0)
    st = torch.cuda.current_stream(dev)
    pads = [int(p) for p in args.pads.split(",")]
    sol = {}
    for p in pads:
        c = torch.full((N, N + p), float("inf"), dtype=tdt, device=dev)
        c[:, :N] = base
        T = torch.empty_like(c)
        sol[p] = (c, T, eikonal.Fim2d(ctx, 1, N, N + p, edt))
    ref = None
    res = {p: [] for p in pads}
    vis = {}
    for _ in range(args.rounds):  # alternate the widths (drift on the box hits all alike)
        for p in pads:
            c, T, f = sol[p]
            f.solve(c.data_ptr(), T.data_ptr(), [goal], st.cuda_stream)
            torch.cuda.synchronize()
            for _ in range(args.reps):
                t0 = time.perf_counter()
                f.solve(c.data_ptr(), T.data_ptr(), [goal], st.cuda_stream)
                res[p].append((time.perf_counter() - t0) * 1e3)
            s = f.stats()
            vis[p] = (s["tile_visits"], s["inplace_passes"])
            Tn = T[:, :N]
            if ref is None:
                ref = Tn.clone()
            else:
                fin = torch.isfinite(ref)
                assert torch.equal(fin, torch.isfinite(Tn)), p
                err = float(((Tn[fin] - ref[fin]).abs() / ref[fin].clamp(min=1e-30)).max())
                assert err <= (1e-11 if f64 else 1e-5), (p, err)
    out = {"dtype": args.dtype, "rows": {}}
    for p in pads:
        v, ps = vis[p]
        med = float(np.median(res[p]))
        out["rows"][p] = {"W": N + p, "pitch_bytes": (N + p) * (8 if f64 else 4), "ms_median": round(med, 4),
                          "ms_min": round(float(np.min(res[p])), 4), "tile_visits": v, "inplace_passes": ps,
                          "us_per_pass": round(med * 1e3 / max(v + ps, 1) * 1.0, 4)}
        print(f"pad {p:4d} W {N + p} pitch {(N + p) * (8 if f64 else 4):6d} B: {med:.4f} ms (min {np.min(res[p]):.4f}), "
              f"visits {v} passes {ps}", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
