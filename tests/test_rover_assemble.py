"""Host tail of the planner's step 1 (eik_rover_assemble, Coupled_motion_planner.py:1228-1252)
against the oracle's statement-by-statement numpy restatement (oracle/planner_oracle.py): path
stitching, metres, pruning near the rover / sample, z lookup with half-to-even rounding, heading.
Bit-exact except the heading's arctan2: numpy's vectorised arctan2 and glibc's atan2 may differ
in the last ulp (|diff| <= 1e-15 rad).  No GPU."""
import numpy as np
import pytest

import planner
import planner_oracle as PO


def walk(rng, start, n, W):
    steps = rng.normal(0, 0.45, (n, 2))
    p = np.cumsum(steps, 0) + start
    return np.clip(p, 1, W - 3)


@pytest.mark.parametrize("seed,res", [(0, 0.05), (1, 0.05), (2, 0.25), (3, 0.5), (4, 0.1)])
def test_assemble_matches_oracle(seed, res):
    rng = np.random.default_rng(seed)
    W = 64
    Z = rng.normal(0, 1, (W, W)) + 7.5
    join = rng.uniform(20, 40, 2)
    pathS = walk(rng, join, 40, W)
    pathG = walk(rng, join, 50, W)
    pathS[0] = pathG[0] = join
    if res >= 0.25:  # exact binary spacing: hit the half-to-even ties of np.round
        pathS[5] = [10.5, 11.5]
        pathG[7] = [12.5, 3.5]
    # rover at the end of pathS, sample at the end of pathG (in metres, as main() receives them)
    xr, yr = res * (pathS[-1] + 1)
    xm, ym = res * (pathG[-1] + 1)
    ref_p, ref_h = PO.assemble(pathS, pathG, Z, xm, ym, xr, yr, 0.3, res)
    got_p, got_h = planner.assemble(pathS, pathG, Z, xm, ym, xr, yr, 0.3, res)
    assert got_p.shape == ref_p.shape and len(ref_p) < len(pathS) + len(pathG) - 1  # something was pruned
    assert np.array_equal(got_p, ref_p)
    assert got_h[0] == ref_h[0] and np.abs(got_h - ref_h).max() <= 1e-15


def test_assemble_prunes_everything():
    Z = np.zeros((8, 8))
    p = np.array([[1.0, 1.0], [1.02, 1.0]])
    got_p, got_h = planner.assemble(p, p, Z, 0.1, 0.1, 0.1, 0.1, 0.0, 0.05)
    ref_p, ref_h = PO.assemble(p, p, Z, 0.1, 0.1, 0.1, 0.1, 0.0, 0.05)
    assert got_p.shape == ref_p.shape == (0, 3)
    # the reference's hstack keeps initialHeading alone for an empty path; the ABI returns n rows
    assert got_h.shape == (0,) and ref_h.tolist() == [0.0]


def test_assemble_outside_dem_raises():
    Z = np.zeros((8, 8))
    pS = np.array([[3.0, 3.0], [2.0, 2.0]])
    pG = np.array([[3.0, 3.0], [20.0, 3.0]])  # x index 21 > 7: the reference raises IndexError
    with pytest.raises(IndexError):
        PO.assemble(pS, pG, Z, 9.0, 9.0, 9.0, 9.0, 0.0, 1.0)
    with pytest.raises(IndexError):
        planner.assemble(pS, pG, Z, 9.0, 9.0, 9.0, 9.0, 0.0, 1.0)
