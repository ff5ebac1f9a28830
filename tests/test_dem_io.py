"""DEM ingest: eik_load_dem_txt / costmap.load_dem against the
reference's own parsing expression (Coupled_motion_planner.py:1098-1099), bit-exact.  Host only
(runs without a GPU)."""
import time

import numpy as np
import pytest

from eikonal import _lib as L


def reference_parse(path):
    # Coupled_motion_planner.py:1098-1099
    with open(path, "r") as file:
        return np.array([[float(num) for num in line.split(",")] for line in file])


@pytest.mark.parametrize("fmt", ["repr", "%.6f", "%.3e", "mixed"])
def test_matches_reference_parse(tmp_path, fmt):
    rng = np.random.default_rng(3)
    Z = rng.normal(0, 50, (37, 53))
    Z[0, 0] = 0.0
    Z[1, 2] = -1234.5
    p = tmp_path / "PRL_DEM.txt"
    with open(p, "w") as f:
        for r, row in enumerate(Z):
            if fmt == "repr":
                f.write(",".join(repr(float(v)) for v in row) + "\n")
            elif fmt == "mixed":  # ints, exponents, blanks around values, CRLF
                items = [str(int(v)) if i % 5 == 0 else (f" {v:.9g} " if i % 3 else f"{v:.4E}") for i, v in enumerate(row)]
                f.write(",".join(items) + ("\r\n" if r % 2 else "\n"))
            else:
                f.write(",".join(fmt % v for v in row) + "\n")
    got = L.load_dem_txt(str(p), nthreads=4)
    ref = reference_parse(p)
    assert got.shape == ref.shape and np.array_equal(got, ref)


def test_dropin_and_errors(tmp_path):
    import costmap

    p = tmp_path / "PRL_DEM.txt"
    p.write_text("1,2,3\n4,5,6\n")
    assert np.array_equal(costmap.load_dem(str(tmp_path) + "/"), [[1, 2, 3], [4, 5, 6]])
    p.write_text("1,2,3\n4,5\n")
    with pytest.raises(ValueError):
        L.load_dem_txt(str(p))
    p.write_text("1,2,x\n")
    with pytest.raises(ValueError):
        L.load_dem_txt(str(p))
    with pytest.raises(ValueError):
        L.load_dem_txt(str(tmp_path / "missing.txt"))


def test_speed_vs_reference(tmp_path):
    Z = np.random.default_rng(1).uniform(0, 10, (600, 600))
    p = tmp_path / "PRL_DEM.txt"
    np.savetxt(p, Z, delimiter=",", fmt="%.8f")
    t0 = time.perf_counter()
    ref = reference_parse(p)
    t1 = time.perf_counter()
    got = L.load_dem_txt(str(p))
    t2 = time.perf_counter()
    assert np.array_equal(got, ref)
    assert (t2 - t1) < (t1 - t0)  # parallel from_chars beats a Python float() per value
