"""Golden fixtures for the planner's cost raster and step-1 tail, made
by running the REFERENCE's own statements in this container.

Run ONCE in the build container, where the reference sources are readable:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_costmap.py

The planner module cannot be imported here (its top-level `import cv2` fails: OpenCV is not
installed), so, as make_golden_arm.py does, this script reads
/root/reference/src/Coupled_motion_planner.py as text and compiles, unmodified:
  * the function definitions `surface_normal` (:37-80) and `structural_disk` (:96-105);
  * statement slices of `main()` (found with `ast` by line number, executed in order in one
    namespace holding the module's own imports :3-16 -- numpy as np, array, dot, math, scipy's
    signal / ndimage, epsilon):
      head   :1101, :1104, :1145-1163  DEM shift, normals, slope obstacles, cleared border, uint8;
      tail   :1180-1216                border, float64, obstacle cost, EDT ramp, 50 x 50 blur with
                                       fill 300, +inf border -- EXCEPT :1192 (cv2.dilate);
      step1  :1101, :1113, :1131, :1232-1255   path stitching, metres, pruning near the rover /
                                       sample, z lookup, heading.
Only the cv2 calls stay outside: image_filling (:82-94, cv2.floodFill / bitwise_not) and the
erode / dilate pairs of :1164-1177 and :1192.  Their outputs are produced by the oracle's
restatement (oracle/costmap_oracle.py, itself checked against brute-force definitions) and fed to
the next reference statement as INPUTS, so every array recorded here as an output is the
reference's own arithmetic on recorded inputs.  Nothing under tests/ reads /root/reference at test
time; the fixture is pure data (costmap.npz).
"""
import ast
import math
import os
import sys

import numpy as np
from scipy import ndimage, signal

REF = "/root/reference/src/Coupled_motion_planner.py"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import costmap_oracle as CO  # noqa: E402  (the cv2 restatements only)
import oracle as O  # noqa: E402  (biComputeTmap / getPathGDM, pinned by fmm2d_bidir.npz)
import terrain_np  # noqa: E402

SRC = open(REF).read()
TREE = ast.parse(SRC)


def module_namespace():
    ns = {"np": np, "array": np.array, "dot": np.dot, "math": math, "signal": signal, "ndimage": ndimage,
          "epsilon": sys.float_info.epsilon}
    defs = [n for n in TREE.body if isinstance(n, ast.FunctionDef) and n.name in ("surface_normal", "structural_disk")]
    assert len(defs) == 2
    exec(compile(ast.Module(body=defs, type_ignores=[]), REF, "exec"), ns)
    return ns


MAIN = [n for n in TREE.body if isinstance(n, ast.FunctionDef) and n.name == "main"][0]


def stmts(*ranges):
    """main()'s top-level statements whose first line lies in one of the (lo, hi) ranges."""
    out = [s for s in MAIN.body if any(lo <= s.lineno <= hi for lo, hi in ranges)]
    for s in out:
        assert "cv2" not in ast.get_source_segment(SRC, s), ast.get_source_segment(SRC, s)
    return out


def run(ns, body):
    exec(compile(ast.Module(body=body, type_ignores=[]), REF, "exec"), ns)


HEAD = stmts((1101, 1101), (1104, 1104), (1145, 1163))
TAIL_A = stmts((1180, 1191))  # ... up to the cv2.dilate of :1192
TAIL_B = stmts((1194, 1216))
STEP1 = stmts((1101, 1101), (1113, 1113), (1131, 1131), (1232, 1255))
assert [s.lineno for s in TAIL_A][-1] == 1191 and TAIL_B[0].lineno == 1194


def cost_case(Z, res):
    """Reference head -> oracle cv2 middle -> reference tail on the DEM Z (square, size = n res)."""
    n = Z.shape[0]
    ns = module_namespace()
    ns.update(Zs=Z.copy(), resolution=res, size=n * res)
    run(ns, HEAD)
    out = {"Z": Z, "res": np.float64(res), "Nx": ns["Nx"], "Ny": ns["Ny"], "Nz": ns["Nz"],
           "obst_head": ns["obstMap"].copy()}
    # :1164-1177 (cv2), restated
    ob = CO.image_filling(ns["obstMap"])
    se = CO.structural_disk(10)
    ob = CO.dilate(CO.erode(ob, se), se)
    se = CO.structural_disk(int(round((0.9 / 2) / res)))
    ob = CO.erode(CO.image_filling(CO.dilate(ob, se)), se)
    out.update(tail_in(ob, res))
    return out


def tail_in(ob, res):
    """Reference tail :1180-1216 on the uint8 obstacle map `ob` (the state after :1177), with
    :1192's cv2.dilate restated (recorded as the input `dilated`)."""
    ns = module_namespace()
    ns.update(obstMap=ob.copy(), resolution=res)
    run(ns, TAIL_A)
    dil = CO.dilate(ns["obstMap"], ns["se"])
    ns["dilatedObstMap"] = dil
    run(ns, TAIL_B)
    return {"obst_mid": ob, "dilated": dil, "obst_final": ns["obstMap"], "cmap": ns["cMap"]}


def step1_case(pathS, pathG, Z, xm, ym, xr, yr, h0, res):
    ns = module_namespace()
    ns.update(Zs=Z.copy(), pathS=pathS.copy(), pathG=pathG.copy(), xm=xm, ym=ym, xr=xr, yr=yr, initialHeading=h0,
              resolution=res)
    run(ns, STEP1)
    return {"pathS": pathS, "pathG": pathG, "Z": Z, "q": np.array([xm, ym, xr, yr, h0, res]),
            "roverPath": ns["roverPath"], "heading": ns["heading"]}


def walk(rng, start, n, W):
    p = np.cumsum(rng.normal(0, 0.45, (n, 2)), 0) + start
    return np.clip(p, 1, W - 3)


def main():
    d = {}
    # structural_disk (:96-105) at the radii the planner uses (10, 0.45 / res, 1 / res) and others
    radii = [0, 1, 2, 5, 9, 10, 20]
    ns = module_namespace()
    for r in radii:
        d[f"disk{r}"] = ns["structural_disk"](r)
    d["disk_radii"] = np.array(radii)
    # cost raster cases: two fractal DEMs (steep: slope obstacles + morphology), one gentle
    cases = [(96, 5, 0.25), (128, 6, 0.30), (112, 7, 0.12)]
    for k, (n, seed, slope) in enumerate(cases):
        Z = terrain_np.dem(n, n, seed=seed, rms_slope=slope) + 3.0
        for key, v in cost_case(Z, 0.05).items():
            d[f"c{k}_{key}"] = v
    d["n_cost"] = np.array(len(cases))
    # the tail alone on synthetic obstacle maps (blobs, a map with no interior obstacle)
    rng = np.random.default_rng(11)
    ob = np.zeros((90, 100), np.uint8)
    for _ in range(6):
        cy, cx, r = rng.integers(5, 85), rng.integers(5, 95), rng.integers(2, 9)
        yy, xx = np.mgrid[0:90, 0:100]
        ob[(yy - cy) ** 2 + (xx - cx) ** 2 <= r * r] = 1
    for key, v in tail_in(ob, 0.05).items():
        d[f"t0_{key}"] = v
    for key, v in tail_in(np.zeros((70, 70), np.uint8), 0.1).items():
        d[f"t1_{key}"] = v
    d["t_res"] = np.array([0.05, 0.1])
    # step-1 tail: random walks (as test_rover_assemble), exact binary spacings (np.round ties),
    # and the real chain on cost case 0 (oracle biComputeTmap + getPathGDM on the reference cMap)
    s1 = []
    for seed, res in [(0, 0.05), (2, 0.25), (3, 0.5)]:
        rng = np.random.default_rng(seed)
        W = 64
        Z = rng.normal(0, 1, (W, W)) + 7.5
        join = rng.uniform(20, 40, 2)
        pS, pG = walk(rng, join, 40, W), walk(rng, join, 50, W)
        pS[0] = pG[0] = join
        if res >= 0.25:
            pS[5] = [10.5, 11.5]
            pG[7] = [12.5, 3.5]
        xr, yr = res * (pS[-1] + 1)
        xm, ym = res * (pG[-1] + 1)
        s1.append(step1_case(pS, pG, Z, xm, ym, xr, yr, 0.3, res))
    Z0, cm0 = d["c0_Z"], d["c0_cmap"]
    res = 0.05
    goal, start = [70, 60], [12, 15]  # sampleNode, roverNode (:1107-1117) of xm, ym, xr, yr below
    xm, ym = res * (goal[0] + 1), res * (goal[1] + 1)
    xr, yr = res * (start[0] + 1), res * (start[1] + 1)
    O.set_strict(False)
    TG, TS, join = O.fmm2d_bidir(cm0.T, goal, start)
    pG, _ = O.gdm2d(TG, join, goal, 0.5)
    pS, _ = O.gdm2d(TS, join, start, 0.5)
    s1.append(step1_case(pS, pG, Z0, xm, ym, xr, yr, -0.7, res))
    for k, c in enumerate(s1):
        for key, v in c.items():
            d[f"s{k}_{key}"] = v
    d["n_step1"] = np.array(len(s1))
    np.savez_compressed(os.path.join(HERE, "costmap.npz"), **d)
    print("wrote costmap.npz:", len(d), "arrays")


if __name__ == "__main__":
    main()
