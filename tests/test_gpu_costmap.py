"""GPU cost-raster builder (csrc/costmap.hip, eik_costmap_*) against the oracle restatement of
Coupled_motion_planner.py:37-105, :1101-1216 (oracle/costmap_oracle.py; cv2 semantics pinned by
tests/test_costmap_oracle.py).  Masks (obstacles, hole filling) bit-exact; normals and costs
within 1e-12 relative (the 50 x 50 blur sums in another order than scipy's convolve2d)."""
import numpy as np
import pytest

import costmap_oracle as CO
import terrain_np

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import eikonal

    c = eikonal.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("n,seed", [(40, 1), (97, 2), (160, 3)])
def test_surface_normal(ctx, n, seed):
    Z = terrain_np.dem(n, n, seed=seed)
    size = 0.05 * n
    ref = CO.surface_normal(0.05, size, Z - Z.min())
    got = ctx.surface_normal(Z - Z.min(), size)
    for g, r in zip(got, ref):
        assert np.abs(g - r).max() <= 1e-12


@pytest.mark.parametrize("shape,seed,p", [((64, 64), 0, 0.4), ((129, 77), 1, 0.5), ((300, 311), 2, 0.45),
                                          ((50, 60), 3, 0.6)])
def test_image_filling(ctx, shape, seed, p):
    rng = np.random.default_rng(seed)
    im = (rng.random(shape) < p).astype(np.uint8)
    for s in (0, 1):  # seed pixel free / obstacle (the reference fills everything then)
        im[0, 0] = s
        assert np.array_equal(ctx.image_fill(im), CO.image_filling(im))


@pytest.mark.parametrize("n,seed,rms", [(120, 5, 0.25), (200, 6, 0.2), (257, 7, 0.3)])
def test_costmap_vs_oracle(ctx, n, seed, rms):
    Z = terrain_np.dem(n, n, seed=seed, rms_slope=rms) + 3.0
    size = 0.05 * n
    cref, oref = CO.cost_map(Z, 0.05, size)
    cost, obst = ctx.costmap(Z, 0.05, size)
    assert np.array_equal(obst.astype(np.float64), oref)
    R = cref.T  # the GPU returns [y][x] = the array the planner hands to the solver
    fin = np.isfinite(R)
    assert np.array_equal(np.isfinite(cost), fin)
    assert (np.abs(cost[fin] - R[fin]) / R[fin]).max() <= 1e-12


def test_costmap_dropin_and_solver(ctx):
    """costmap.cost_map mirrors main()'s orientation; its output feeds the solver directly."""
    import costmap
    import FastMarching.FastMarching as FM

    n = 140
    Z = terrain_np.dem(n, n, seed=9, rms_slope=0.22)
    cmap, obst = costmap.cost_map(Z, 0.05, 0.05 * n)
    cref, oref = CO.cost_map(Z, 0.05, 0.05 * n)
    assert np.array_equal(obst, oref)
    fin = np.isfinite(cref)
    assert (np.abs(cmap[fin] - cref[fin]) / cref[fin]).max() <= 1e-12
    free = np.argwhere(np.isfinite(cmap.T) & (cmap.T < 50))
    gy, gx = free[len(free) // 2]
    T = FM.computeTmap(cmap.T, [int(gx), int(gy)], [-1, -1])
    assert T[gy, gx] == 0 and np.isfinite(T).sum() > n * n // 4
