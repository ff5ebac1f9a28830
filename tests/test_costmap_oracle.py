"""CPU checks of the cost-builder oracle (oracle/costmap_oracle.py): the restated cv2 semantics
against brute-force definitions, and the builder end to end on small DEMs.  The reference
builder itself needs OpenCV, absent here: its parity is pinned to these restatements."""
import collections

import numpy as np
import pytest

import costmap_oracle as CO


def brute_morph(im, r, erode):
    """per pixel: min / max over in-image pixels q with |p - q|^2 <= r^2 (cv2 border rule)"""
    H, W = im.shape
    out = np.empty_like(im)
    for y in range(H):
        for x in range(W):
            vals = [im[y + dy, x + dx] for dy in range(-r, r + 1) for dx in range(-r, r + 1)
                    if dy * dy + dx * dx <= r * r and 0 <= y + dy < H and 0 <= x + dx < W]
            out[y, x] = min(vals) if erode else max(vals)
    return out


def brute_fill(im):
    """cv2.floodFill(im, mask, (0, 0), 1) (4-connected, pixels equal to the seed), then the
    reference's `im | (bitwise_not(filled) - 254)` in uint8"""
    H, W = im.shape
    seed = im[0, 0]
    filled = im.copy()
    seen = np.zeros_like(im, dtype=bool)
    dq = collections.deque([(0, 0)])
    seen[0, 0] = True
    while dq:
        y, x = dq.popleft()
        filled[y, x] = 1
        for dy, dx in ((1, 0), (-1, 0), (0, 1), (0, -1)):
            yy, xx = y + dy, x + dx
            if 0 <= yy < H and 0 <= xx < W and not seen[yy, xx] and im[yy, xx] == seed:
                seen[yy, xx] = True
                dq.append((yy, xx))
    inv = ((255 - filled.astype(np.int32)) - 254) % 256
    return im | inv.astype(np.uint8)


@pytest.mark.parametrize("r,seed", [(1, 0), (2, 1), (3, 2), (5, 3)])
def test_morph_vs_brute(r, seed):
    rng = np.random.default_rng(seed)
    im = (rng.random((23, 31)) < 0.3).astype(np.uint8)
    se = CO.structural_disk(r)
    assert np.array_equal(CO.erode(im, se), brute_morph(im, r, True))
    assert np.array_equal(CO.dilate(im, se), brute_morph(im, r, False))


@pytest.mark.parametrize("seed", range(4))
def test_fill_vs_brute(seed):
    rng = np.random.default_rng(seed)
    im = (rng.random((29, 27)) < 0.45).astype(np.uint8)
    im[0, 0] = seed % 2  # both seed values (1: the reference turns the whole image to 1)
    assert np.array_equal(CO.image_filling(im), brute_fill(im))


def test_disk():
    d = CO.structural_disk(3)
    yy, xx = np.mgrid[-3:4, -3:4]
    assert np.array_equal(d, (yy * yy + xx * xx <= 9).astype(np.uint8))


def test_normals_plane():
    """z = a x + b y on the reference grid: Nz = 1 / sqrt(1 + a^2 + b^2) everywhere (the quadratic
    edge extrapolation is exact for a plane)."""
    n, size = 40, 2.0
    g = np.linspace(0, size, n)
    x, y = np.meshgrid(g, g)
    a, b = 0.3, -0.2
    nx, ny, nz = CO.surface_normal(size / n, size, a * x + b * y)
    assert np.allclose(nz, 1 / np.sqrt(1 + a * a + b * b), atol=1e-12)
    assert np.allclose(nx, -a / np.sqrt(1 + a * a + b * b), atol=1e-12)


def test_costmap_runs():
    import terrain_np

    Z = terrain_np.dem(120, 120, seed=5)
    cmap, obst = CO.cost_map(Z, 0.05, 6.0)
    assert cmap.shape == (120, 120) and np.isinf(cmap[0]).all() and np.isfinite(cmap[1:-1, 1:-1]).all()
    assert set(np.unique(obst)) <= {0.0, 1.0} and obst[0].all()
