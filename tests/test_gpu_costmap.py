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


def _spiral(n, w=2):
    """A one-corridor spiral of free pixels from (0, 0) inwards: one component that winds through
    every 32 x 32 tile of the union-find many times, plus closed pockets (holes) beside it."""
    im = np.ones((n, n), np.uint8)
    y0, x0, y1, x1 = 0, 0, n - 1, n - 1
    while y1 - y0 > 2 * w and x1 - x0 > 2 * w:
        im[y0:y0 + w, x0:x1 + 1] = 0
        im[y0:y1 + 1, x1 - w + 1:x1 + 1] = 0
        im[y1 - w + 1:y1 + 1, x0 + w + 1:x1 + 1] = 0
        im[y0 + 2 * w:y1 + 1, x0 + w + 1:x0 + 2 * w + 1] = 0
        y0, x0, y1, x1 = y0 + 2 * w, x0 + 2 * w + 1, y1 - 2 * w, x1 - 2 * w
    return im


@pytest.mark.parametrize("n", [97, 300, 1025])
def test_image_filling_spiral(ctx, n):
    """image_filling (:82-94) on a maze: a corridor spiralling through many union-find tiles, and
    pockets of free pixels it does not reach (the holes filled), against the oracle's flood fill."""
    im = _spiral(n)
    rng = np.random.default_rng(n)
    pockets = (rng.random(im.shape) < 0.002) & (im == 1)
    im[pockets] = 0  # isolated free pixels inside the walls: holes to fill
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


@pytest.mark.parametrize("k", range(3))
def test_costmap_vs_reference_fixture(ctx, golden, k):
    """The GPU builder against the reference's own statements (tests/golden/costmap.npz: the
    reference's head :1101-1163 and tail :1180-1216 run in the build container, the cv2 middle
    restated): normals <= 1e-12, obstacle masks bit-exact, costs <= 1e-12 relative."""
    g = golden("costmap")
    Z, res = g[f"c{k}_Z"], float(g[f"c{k}_res"])
    n = Z.shape[0]
    got = ctx.surface_normal(Z - Z.min(), n * res)
    for a, key in zip(got, ("Nx", "Ny", "Nz")):
        assert np.abs(a - g[f"c{k}_{key}"]).max() <= 1e-12
    cost, obst = ctx.costmap(Z, res, n * res)
    assert np.array_equal(obst.astype(np.float64), g[f"c{k}_obst_final"])
    R = g[f"c{k}_cmap"].T
    fin = np.isfinite(R)
    assert np.array_equal(np.isfinite(cost), fin)
    assert (np.abs(cost[fin] - R[fin]) / R[fin]).max() <= 1e-12


MORPH_CASES = [((300, 257), 1), ((300, 257), 9), ((300, 257), 10), ((300, 257), 20), ((130, 200), 63),
               ((130, 200), 64), ((131, 66), 65), ((70, 300), 3)]


@pytest.mark.parametrize("shape,r", MORPH_CASES, ids=[f"{s[0]}x{s[1]}-r{r}" for s, r in MORPH_CASES])
@pytest.mark.parametrize("erode", [False, True])
def test_disk_morphology_vs_oracle(ctx, shape, r, erode):
    """cv2.erode / cv2.dilate with structural_disk (Coupled_motion_planner.py:96-105, :1168-1177) on
    random masks, bit-exact against the oracle's restatement: the segment scans of the bounded
    transform (csrc/costmap.hip cm_bnd_*) at radii around the 64-pixel segment length, ragged shapes."""
    rng = np.random.default_rng(r * 7 + erode)
    p = 0.92 if erode else 0.02  # erosion of a mostly-set mask, dilation of a sparse one
    im = (rng.random(shape) < p).astype(np.uint8)
    se = CO.structural_disk(r)
    ref = CO.erode(im, se) if erode else CO.dilate(im, se)
    got = ctx.disk_morph(im, r, erode)
    assert np.array_equal(got, ref), (shape, r, erode, int((got != ref).sum()))
