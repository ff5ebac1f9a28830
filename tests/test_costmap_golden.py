"""The cost-raster and step-1-tail oracles against the REFERENCE's own functions and statements run
in the build container (tests/golden/make_golden_costmap.py -> costmap.npz; SURVEY.md §8(f) ranks
1-2).  Pinned bit for bit: surface_normal (Coupled_motion_planner.py:37-80), structural_disk
(:96-105), main()'s head (:1101-1163: shift, normals, slope obstacles, cleared border) and tail
(:1180-1216: border, obstacle cost, EDT ramp, 50 x 50 blur, +inf border) given the recorded state
after the cv2 block, and the step-1 tail (:1232-1255: stitching, metres, pruning, z, heading).
The cv2 calls themselves (:82-94, :1164-1177, :1192) stay "parity unpinned" (no OpenCV here) and
are pinned to brute-force definitions in test_costmap_oracle.py.  No GPU."""
import numpy as np
import pytest

import costmap_oracle as CO
import planner_oracle as PO


@pytest.fixture(scope="module")
def g(golden):
    return golden("costmap")


def test_structural_disk(g):
    for r in g["disk_radii"]:
        assert np.array_equal(CO.structural_disk(int(r)), g[f"disk{r}"]), r


@pytest.mark.parametrize("k", range(3))
def test_surface_normal_and_head(g, k):
    Z, res = g[f"c{k}_Z"], float(g[f"c{k}_res"])
    n = Z.shape[0]
    nx, ny, nz = CO.surface_normal(res, n * res, Z - Z.min())
    assert np.array_equal(nx, g[f"c{k}_Nx"]) and np.array_equal(ny, g[f"c{k}_Ny"]) and np.array_equal(nz, g[f"c{k}_Nz"])
    head = CO.obstacle_head(Z, res, n * res)
    assert head.dtype == np.uint8 and np.array_equal(head, g[f"c{k}_obst_head"])


@pytest.mark.parametrize("p", ["c0", "c1", "c2", "t0", "t1"])
def test_cost_tail(g, p):
    res = float(g[f"{p}_res"]) if f"{p}_res" in g else float(g["t_res"][int(p[1])])
    cm, ob = CO.cost_tail(g[f"{p}_obst_mid"], res, dilated=g[f"{p}_dilated"])
    assert np.array_equal(ob, g[f"{p}_obst_final"])
    assert np.array_equal(cm, g[f"{p}_cmap"])  # +inf border and every finite value, bit for bit
    # and the restated dilation of :1192 reproduces the recorded input
    cm2, _ = CO.cost_tail(g[f"{p}_obst_mid"], res)
    assert np.array_equal(cm2, cm)


@pytest.mark.parametrize("k", range(3))
def test_cost_map_end_to_end(g, k):
    """The whole builder: reference head -> (restated cv2 middle) -> reference tail."""
    Z, res = g[f"c{k}_Z"], float(g[f"c{k}_res"])
    n = Z.shape[0]
    assert np.array_equal(CO.obstacle_morphology(g[f"c{k}_obst_head"], res), g[f"c{k}_obst_mid"])
    cm, ob = CO.cost_map(Z, res, n * res)
    assert np.array_equal(cm, g[f"c{k}_cmap"]) and np.array_equal(ob, g[f"c{k}_obst_final"])


@pytest.mark.parametrize("k", range(4))
def test_step1_tail(g, k):
    xm, ym, xr, yr, h0, res = (float(v) for v in g[f"s{k}_q"])
    p, h = PO.assemble(g[f"s{k}_pathS"], g[f"s{k}_pathG"], g[f"s{k}_Z"], xm, ym, xr, yr, h0, res)
    assert np.array_equal(p, g[f"s{k}_roverPath"]) and np.array_equal(h, g[f"s{k}_heading"])


@pytest.mark.parametrize("k", range(4))
def test_step1_tail_native(g, k):
    """The product's host tail (eik_rover_assemble, csrc/rover.cpp; no device work) against the
    reference's statements: path bit-exact, heading within 1e-15 rad (glibc atan2 vs numpy's)."""
    import planner

    xm, ym, xr, yr, h0, res = (float(v) for v in g[f"s{k}_q"])
    p, h = planner.assemble(g[f"s{k}_pathS"], g[f"s{k}_pathG"], g[f"s{k}_Z"], xm, ym, xr, yr, h0, res)
    ref_p, ref_h = g[f"s{k}_roverPath"], g[f"s{k}_heading"]
    assert np.array_equal(p, ref_p)
    if len(ref_p):
        assert h[0] == ref_h[0] and np.abs(h - ref_h).max() <= 1e-15
