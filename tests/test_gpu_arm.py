"""End-effector cost volume and its FM3D solve on the GPU.

* GetObstMap / TunnelCost (arm.hip, eik_arm_*): bit-exact against the reference's own outputs
  (tests/golden/arm.npz) and against the pinned restatement (oracle/arm_oracle.py) on further
  random areas;
* eik_arm_path_f64 (Cmap = GetObstMap * TunnelCost -> FM3D early-exit field -> 3D path): the
  volume bit-exact, the field against the oracle's exact early-exit FMM (closed cells <= 1e-9, band
  within the bracket of tests/test_gpu_fm3d_early.py), the path within 1e-9 of the oracle's walk on
  the oracle's own field; the reference's own paths: tests/test_gpu_fm3d_early.py;
* eik_tmap3d_batch_f64: B volumes in one solve equal the oracle field of each volume (<= 1e-9)."""
import math

import numpy as np
import pytest

import arm_oracle as AO
import oracle as O
from band import BAND_BRACKET, band_ratio
import planner

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import eikonal

    c = eikonal.Context(0)
    yield c
    c.close()


def _case(golden, i):
    d = golden("arm")
    return {k[len(f"a{i}_"):]: d[k] for k in d.files if k.startswith(f"a{i}_")}


@pytest.mark.parametrize("i", range(3))
def test_golden_obst_map(golden, i):
    c = _case(golden, i)
    sX, sY, sZ = (int(v) for v in c["shape"])
    f, o, g = planner.GetObstMap(c["Z"], *c["res"], sX, sY, sZ, c["obst"], *c["xy_m"])
    assert np.array_equal(f, c["finalMap"]) and np.array_equal(o, c["obstMap"]) and np.array_equal(g, c["groundMap"])


@pytest.mark.parametrize("i", range(3))
def test_golden_tunnel_cost(golden, i):
    c = _case(golden, i)
    sX, sY, sZ = (int(v) for v in c["shape"])
    Rlim, rO, rm = c["radii"]
    got = planner.TunnelCost(Rlim, rO, rm, c["base"], sX, sY, sZ, *c["res"], c["heading"], c["finalWP"], c["initWP"])
    assert np.array_equal(got, c["tunnel"]), int((got != c["tunnel"]).sum())


def random_area(seed, half, m, res=0.05):
    rng = np.random.default_rng(seed)
    n = 2 * half
    yy, xx = np.mgrid[0:n, 0:n] * res
    Z = 0.1 * np.sin(2.1 * xx + seed) * np.cos(0.9 * yy + 0.3) + 0.03 * rng.standard_normal((n, n))
    Z -= Z.min()
    resX = resY = res * (2 * n - 1) / (2 * n)
    sZ = int(round((Z.max() + 0.5) / 0.02))
    obst = (rng.random((n, n)) < 0.1).astype(np.float64)
    p0, p1 = np.array([0.2, 0.35]) * n * resX, np.array([0.6, 0.5]) * n * resX
    t = np.linspace(0, 1, m)[:, None]
    base = np.zeros((m, 3))
    base[:, :2] = p0 + t * (p1 - p0) + 0.03 * rng.standard_normal((m, 2))
    base[:, 2] = 0.25 + 0.05 * rng.random(m)
    yaw = math.atan2(*(p1 - p0)[::-1]) + 0.2 * rng.standard_normal(m)
    heading = np.stack([0.08 * rng.standard_normal(m), 0.08 * rng.standard_normal(m), yaw], 1)
    fw = np.uint32(np.round([(p1[0] + 0.2) / resX, (p1[1] + 0.15) / resY, (Z.max() * 0.6 + 0.1) / 0.02]))
    iw = np.uint32(np.round([(p0[0] + 0.15) / resX, (p0[1] + 0.1) / resY, 0.45 / 0.02]))
    return Z, obst, (resX, resY, 0.02), (n, n, sZ), base, heading, fw, iw


@pytest.mark.parametrize("seed,half,m", [(10, 14, 5), (11, 22, 30), (12, 30, 64)])
def test_random_areas_vs_oracle(seed, half, m):
    Z, obst, res, shape, base, heading, fw, iw = random_area(seed, half, m)
    f, o, g = planner.GetObstMap(Z, *res, *shape, obst, 1.0, 2.0)
    rf, ro, rg = AO.get_obst_map(Z, *res, *shape, obst, 1.0, 2.0)
    assert np.array_equal(f, rf) and np.array_equal(o, ro) and np.array_equal(g, rg)
    got = planner.TunnelCost(0.527, 0.2673, 0.1105, base, *shape, *res, heading, fw, iw)
    ref = AO.tunnel_cost(0.527, 0.2673, 0.1105, base, *shape, *res, heading, fw, iw)
    assert np.array_equal(got, ref), int((got != ref).sum())


@pytest.mark.parametrize("seed,half,m", [(20, 16, 10), (21, 24, 25)])
def test_arm_path_vs_oracle(ctx, seed, half, m):
    Z, obst, res, shape, base, heading, fw, iw = random_area(seed, half, m)
    vol = planner.volume(*shape, *res, 1.0, 2.0, 0.527, 0.2673, 0.1105, fw, iw)
    path, st, cost, T = ctx.arm_path(Z, obst, base, heading, vol, 0.5, want_fields=True)
    rf, _, _ = AO.get_obst_map(Z, *res, *shape, obst, 1.0, 2.0)
    ref_cost = rf * AO.tunnel_cost(0.527, 0.2673, 0.1105, base, *shape, *res, heading, fw, iw)  # :1580
    assert np.array_equal(cost, ref_cost)
    # the oracle's exact early-exit run (FastMarching3D.py:141, pinned bit-exact to the reference
    # by tests/test_oracle_golden.py) and ITS walk -- not the GPU's own field
    R = O.fmm3d(ref_cost, [int(v) for v in fw], [int(v) for v in iw])
    fin = np.isfinite(R)
    assert np.array_equal(np.isfinite(T), fin)
    ts = R[iw[1], iw[0], iw[2]]
    closed = fin & (R < ts)
    assert np.abs(T[closed] - R[closed]).max() <= 1e-9
    band = fin & ~closed
    assert np.all(T[band] <= R[band] + 1e-9)
    r = band_ratio(T, R, band)
    assert r <= BAND_BRACKET, f"band: reference / GPU up to {r:.4f} (bracket {BAND_BRACKET})"
    ref_path, ref_st = O.gdm3d(R, [float(v) for v in iw], [float(v) for v in fw], 0.5)
    assert st == ref_st and path.shape == ref_path.shape and np.abs(path - ref_path).max() <= 1e-9
    assert len(path) >= 2 and np.array_equal(path[-1], fw.astype(float))


def test_tmap3d_batch(ctx):
    rng = np.random.default_rng(3)
    B, H, W, Lz = 4, 24, 20, 9
    cost = rng.uniform(1, 5, (B, H, W, Lz))
    cost[:, 8:16, 5:7, :6] = np.inf
    goals = np.stack([rng.integers(0, W, B), rng.integers(0, H, B), rng.integers(0, Lz, B)], 1)
    for b in range(B):
        cost[b, goals[b, 1], goals[b, 0], goals[b, 2]] = 1.0
    T = ctx.tmap3d_batch(cost, goals)
    for b in range(B):
        R = O.fmm3d(cost[b], [int(v) for v in goals[b]])
        fin = np.isfinite(R)
        assert np.array_equal(np.isfinite(T[b]), fin) and np.abs(T[b][fin] - R[fin]).max() <= 1e-9
