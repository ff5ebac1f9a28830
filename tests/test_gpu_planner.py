"""Planner step 1 on the GPU (planner.rover_path / eik_rover_path_f64: cost raster -> both fronts
-> device join -> two path kernels -> host assembly) against the oracle chain
(oracle/planner_oracle.py: cost_map restatement -> C FMM bidirectional (bit-identical to the
reference's biComputeTmap) -> C GDM -> numpy assembly of Coupled_motion_planner.py:1228-1252).

Tolerances: the cost raster within 1e-12 relative (blur summation order, tests/test_gpu_costmap.py);
the join equal (no exact ties of T on terrain costs); the rover path of the same length within 0.01
cells Hausdorff (both chains descend the fronts' partial fields, whose band values differ,
tests/test_gpu_path.py::test_bidirectional); z and heading exactly as the assembly defines them
on the GPU path."""
import math

import numpy as np
import pytest

import planner
import planner_oracle as PO
import terrain_np

pytestmark = pytest.mark.gpu
RES = 0.05


def hausdorff(a, b):
    d = np.sqrt(((a[:, None, :] - b[None, :, :]) ** 2).sum(-1))
    return max(d.min(1).max(), d.min(0).max())


def free_cell(cT, x, y):
    """nearest cell to (x, y) with a low finite cost ([y][x] raster)"""
    ys, xs = np.nonzero(np.isfinite(cT) & (cT < 5))
    k = np.argmin((xs - x) ** 2 + (ys - y) ** 2)
    return int(xs[k]), int(ys[k])


@pytest.mark.parametrize("n,seed", [(160, 5), (224, 11)])
def test_rover_path_matches_oracle_chain(n, seed):
    Z = terrain_np.dem(n, n, seed=seed) + 3.0
    size = RES * n
    cref, _ = PO.CO.cost_map(Z, RES, size)
    cT = cref.T
    sx, sy = free_cell(cT, int(0.78 * n), int(0.72 * n))
    rx, ry = free_cell(cT, int(0.2 * n), int(0.25 * n))
    # main() receives metres; the nodes are int(round(v / res - 1))
    xm, ym, xr, yr = RES * (sx + 1), RES * (sy + 1), RES * (rx + 1), RES * (ry + 1)
    ref_p, ref_h, ref_j, _ = PO.rover_path(Z, xm, ym, xr, yr, 0.4, RES, size)
    q = planner.query(xm, ym, xr, yr, 0.4, RES, size)
    got_p, got_h, got_j, cost = planner._ctx().rover_path(Z, q, want_cost=True)
    fin = np.isfinite(cT)
    assert np.array_equal(np.isfinite(cost), fin)
    assert np.abs(cost[fin] - cT[fin]).max() <= 1e-12 * np.abs(cT[fin]).max()
    assert got_j.dtype == np.uint32 and np.array_equal(got_j, ref_j)
    assert len(got_p) > 10 and got_p.shape[1] == 3
    # both descend the fronts' partial fields (FastMarching.py:141-162) from the same join
    h = hausdorff(got_p[:, :2] / RES, ref_p[:, :2] / RES)
    assert got_p.shape == ref_p.shape and h <= 0.01, (got_p.shape, ref_p.shape, h)
    # z and heading of the GPU path follow :1246-1252 on its own waypoints
    Zs = Z - Z.min()
    iy = np.round(got_p[:, 1] / RES).astype(np.int64)
    ix = np.round(got_p[:, 0] / RES).astype(np.int64)
    assert np.array_equal(got_p[:, 2], 0.07 + Zs[iy, ix])
    assert got_h[0] == 0.4
    assert np.abs(got_h[1:] - np.arctan2(np.diff(got_p[:, 1]), np.diff(got_p[:, 0]))).max() <= 1e-15
    # no waypoint left within 0.1 m of the rover or the sample (:1232-1243)
    assert np.hypot(got_p[:, 0] - xr, got_p[:, 1] - yr).min() >= 0.1
    assert np.hypot(got_p[:, 0] - xm, got_p[:, 1] - ym).min() >= 0.1


@pytest.mark.parametrize("n,seed", [(160, 5), (224, 11)])
def test_rover_path_exact_band_matches_oracle_chain(n, seed):
    """The same chain with EIK_OPT_EXACT_BAND: the fronts' partial fields are the reference's own
    (band values and LIFO ties replayed, csrc/bidir_exact.hip), so the rover path follows the oracle
    chain's to the path kernel's tolerance on fields whose costs agree to 1e-12 -- not 0.01 cells."""
    import eikonal
    from eikonal import _lib as L

    Z = terrain_np.dem(n, n, seed=seed) + 3.0
    size = RES * n
    cref, _ = PO.CO.cost_map(Z, RES, size)
    cT = cref.T
    sx, sy = free_cell(cT, int(0.78 * n), int(0.72 * n))
    rx, ry = free_cell(cT, int(0.2 * n), int(0.25 * n))
    xm, ym, xr, yr = RES * (sx + 1), RES * (sy + 1), RES * (rx + 1), RES * (ry + 1)
    ref_p, ref_h, ref_j, _ = PO.rover_path(Z, xm, ym, xr, yr, 0.4, RES, size)
    c = eikonal.Context(0)
    try:
        c.set_option(L.OPT_EXACT_BAND, 1)
        got_p, got_h, got_j = c.rover_path(Z, planner.query(xm, ym, xr, yr, 0.4, RES, size))
        assert c.exact_info()["passes"] >= 1
    finally:
        c.close()
    assert np.array_equal(got_j, ref_j)
    assert got_p.shape == ref_p.shape
    assert np.abs(got_p[:, :2] - ref_p[:, :2]).max() / RES <= 1e-6


def test_rover_path_exact_switch(monkeypatch):
    """planner.rover_path reads EIKONAL_EXACT_BAND per call, like the FastMarching drop-ins."""
    n, seed = 160, 5
    Z = terrain_np.dem(n, n, seed=seed) + 3.0
    size = RES * n
    cref, _ = PO.CO.cost_map(Z, RES, size)
    cT = cref.T
    sx, sy = free_cell(cT, int(0.78 * n), int(0.72 * n))
    rx, ry = free_cell(cT, int(0.2 * n), int(0.25 * n))
    xm, ym, xr, yr = RES * (sx + 1), RES * (sy + 1), RES * (rx + 1), RES * (ry + 1)
    ref_p, _, ref_j, _ = PO.rover_path(Z, xm, ym, xr, yr, 0.4, RES, size)
    monkeypatch.setenv("EIKONAL_EXACT_BAND", "1")
    got_p, _, got_j = planner.rover_path(Z, xm, ym, xr, yr, 0.4, RES, size)
    assert planner._ctx().exact_info()["passes"] >= 1
    assert np.array_equal(got_j, ref_j) and got_p.shape == ref_p.shape
    assert np.abs(got_p[:, :2] - ref_p[:, :2]).max() / RES <= 1e-6
    monkeypatch.setenv("EIKONAL_EXACT_BAND", "0")
    planner.rover_path(Z, xm, ym, xr, yr, 0.4, RES, size)
    assert planner._ctx().exact_info()["passes"] == 0


def test_rover_path_unreachable():
    """Rover on the corner node (0, 0): both its neighbours are +inf border cells.  The reference's
    fronts still "meet" there by popping +inf band entries and return a degenerate path; the GPU
    pipeline reports EIK_ERR_UNREACHABLE instead (documented deviation)."""
    import eikonal

    n = 96
    Z = np.zeros((n, n))
    q = planner.query(RES * 40, RES * 40, RES * 1, RES * 1, 0.0, RES, RES * n)
    with pytest.raises(eikonal.EikError) as e:
        planner._ctx().rover_path(Z, q)
    assert e.value.code == eikonal._lib.EIK_ERR_UNREACHABLE


def test_rover_path_node_outside():
    import eikonal

    Z = np.zeros((64, 64))
    q = planner.query(RES * 100, RES * 10, RES * 10, RES * 10, 0.0, RES, RES * 64)
    with pytest.raises(eikonal.EikError) as e:
        planner._ctx().rover_path(Z, q)
    assert e.value.code == eikonal._lib.EIK_ERR_ARG
