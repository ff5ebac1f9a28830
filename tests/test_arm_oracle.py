"""The end-effector volume restatement (oracle/arm_oracle.py) against the reference's own
GetObstMap / TunnelCost outputs (tests/golden/arm.npz, tests/golden/make_golden_arm.py).
Bit-exact; no GPU."""
import numpy as np
import pytest

import arm_oracle as AO


def _case(golden, i):
    d = golden("arm")
    return {k[len(f"a{i}_"):]: d[k] for k in d.files if k.startswith(f"a{i}_")}


@pytest.mark.parametrize("i", range(3))
def test_get_obst_map_golden(golden, i):
    c = _case(golden, i)
    sX, sY, sZ = (int(v) for v in c["shape"])
    resX, resY, resZ = c["res"]
    fm, om, gm = AO.get_obst_map(c["Z"], resX, resY, resZ, sX, sY, sZ, c["obst"], *c["xy_m"])
    assert np.array_equal(fm, c["finalMap"]) and np.array_equal(om, c["obstMap"]) and np.array_equal(gm, c["groundMap"])


@pytest.mark.parametrize("i", range(3))
def test_tunnel_cost_golden(golden, i):
    c = _case(golden, i)
    sX, sY, sZ = (int(v) for v in c["shape"])
    resX, resY, resZ = c["res"]
    Rlim, rO, rm = c["radii"]
    got = AO.tunnel_cost(Rlim, rO, rm, c["base"], sX, sY, sZ, resX, resY, resZ, c["heading"], c["finalWP"], c["initWP"])
    ref = c["tunnel"]
    assert got.shape == ref.shape
    assert np.array_equal(got, ref), int((got != ref).sum())
