"""Golden fixtures for the planner's end-effector volume:
GetObstMap (Coupled_motion_planner.py:319-358) and TunnelCost (:505-725).

Run ONCE in the build container, where the reference sources are readable:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_arm.py

The reference module cannot be imported here (its top-level `import cv2` fails: OpenCV is not
installed), so this script reads /root/reference/src/Coupled_motion_planner.py as text, compiles
ONLY the two function definitions (found with `ast`, unmodified) and runs them in a namespace
holding what they use (numpy as np, math, numpy.dot as dot -- the module's own imports, :1-16).
Nothing else of the planner runs.  Inputs are shaped as main() builds them (:1462-1575): a square
area of 2h x 2h DEM cells with resX = res (2h - 1) / (2h), resZ = 0.02, sZ = round(aZ / 0.02), the
arm base path and heading inside it, waypoints rounded to uint32 nodes.  Outputs are stored next to
this script as arm.npz; nothing under tests/ reads /root/reference at test time.
"""
import ast
import math
import os
import sys

import numpy as np

REF = "/root/reference/src/Coupled_motion_planner.py"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True


def load_reference_functions(names):
    src = open(REF).read()
    tree = ast.parse(src)
    defs = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in names]
    assert sorted(d.name for d in defs) == sorted(names)
    ns = {"np": np, "math": math, "dot": np.dot}
    exec(compile(ast.Module(body=defs, type_ignores=[]), REF, "exec"), ns)
    return [ns[n] for n in names]


GetObstMap, TunnelCost = load_reference_functions(["GetObstMap", "TunnelCost"])

Rm, rm = 0.4241, 0.1105          # :1121-1122
rO = (Rm + rm) / 2               # :1123
Rlim = 0.527                     # :1124


def case(seed, half, res=0.05, m=12, sample_on_grid=False):
    rng = np.random.default_rng(seed)
    n = 2 * half
    ixmin, ixmax = 100, 100 + n  # :1487-1509 (an interior area)
    aX = res * (ixmax - 1) - res * ixmin  # :1523
    # smooth heights >= 0 (ZsMap - Zmin, :1537-1545)
    yy, xx = np.mgrid[0:n, 0:n] * res
    Z = 0.08 * np.sin(1.7 * xx + seed) * np.cos(1.3 * yy) + 0.05 * np.sin(3.1 * yy + 0.4 * xx)
    Z = Z + 0.02 * rng.standard_normal((n, n))
    Z = Z - Z.min()
    aZ = Z.max() - Z.min() + 0.5  # :1525
    sX, sY = Z.shape  # :1528
    sZ = int(round(aZ / 0.02))  # :1529
    resX, resY, resZ = aX / sX, aX / sY, 0.02  # :1532-1534
    obst = (rng.random((n, n)) < 0.08).astype(np.float64)
    # arm base path towards the sample, heading (roll, pitch, yaw) along it
    p0 = np.array([0.25 * n * resX, 0.3 * n * resY])
    p1 = np.array([0.55 * n * resX, 0.6 * n * resY])
    t = np.linspace(0, 1, m)[:, None]
    xy = p0 + t * (p1 - p0) + 0.02 * rng.standard_normal((m, 2))
    base = np.zeros((m, 3))
    base[:, :2] = xy
    base[:, 2] = 0.23 + 0.1 * rng.random(m)
    yaw = math.atan2(p1[1] - p0[1], p1[0] - p0[0]) + 0.1 * rng.standard_normal(m)
    heading = np.stack([0.05 * rng.standard_normal(m), 0.05 * rng.standard_normal(m), yaw], 1)
    xmNew, ymNew, zmNew = p1[0] + 0.25, p1[1] + 0.2, Z.max() * 0.5 + 0.1
    finalWP = np.uint32(np.round([xmNew / resX, ymNew / resY, zmNew / resZ]))  # :1574
    initWP = np.uint32(np.round([(p0[0] + 0.2) / resX, (p0[1] + 0.1) / resY, 0.4 / resZ]))  # :1573
    # GetObstMap's sample test compares resX * i with the GLOBAL xm (:329); one case puts the
    # sample exactly on a grid column/row to exercise the skip
    xm, ym = (resX * 7, resY * 9) if sample_on_grid else (12.3456, 7.891)
    fm, om, gm = GetObstMap(Z, resX, resY, resZ, sX, sY, sZ, obst, xm, ym)
    cm = TunnelCost(Rlim, rO, rm, base, sX, sY, sZ, resX, resY, resZ, heading, finalWP, initWP)
    return dict(Z=Z, obst=obst, res=np.array([resX, resY, resZ]), shape=np.array([sX, sY, sZ]),
                xy_m=np.array([xm, ym]), base=base, heading=heading, finalWP=finalWP, initWP=initWP,
                finalMap=fm, obstMap=om, groundMap=gm, tunnel=cm, radii=np.array([Rlim, rO, rm]))


if __name__ == "__main__":
    out = {}
    for i, (seed, half, grid) in enumerate([(1, 16, False), (2, 20, True), (3, 24, False)]):
        c = case(seed, half, sample_on_grid=grid)
        for k, v in c.items():
            out[f"a{i}_{k}"] = v
        print(i, c["shape"], "tunnel finite/inf/10:", int(np.isfinite(c["tunnel"]).sum()),
              int(np.isinf(c["tunnel"]).sum()), int((c["tunnel"] == 10).sum()), flush=True)
    np.savez_compressed(os.path.join(OUT, "arm.npz"), **out)
