"""The exact band replay's formulation on the CPU (tests/replay_np.py, the prototype of
csrc/bidir_exact.hip) against the reference's own outputs: update events as a DAG in pop order,
relaxed by Jacobi sweeps from a field, pops ordered by (value, -insertion time).

* full fields (FastMarching.py:92-112 driven to the end, tests/golden/fmm2d_fields.npz): from the
  oracle's field, the replay's popped values are the reference's bits on every map, ties included;
* biComputeTmap (:114-162, fmm2d_bidir.npz): from fields a few ulps off (as the GPU's are), nodeJoin
  and both partial fields -- tentative band values included -- are the reference's bits."""
import numpy as np
import pytest

import oracle as O
import replay_np as R


@pytest.mark.parametrize("i", range(12))
def test_replay_full_field_is_the_reference(golden, i):
    d = golden("fmm2d_fields")
    p = f"c{i}_"
    if d[p + "T"].size == 0:
        pytest.skip("the reference raised on this map")
    cost = d[p + "cost"].astype(np.float64)
    goal = tuple(int(v) for v in d[p + "goal"])
    T, *_ = R.replay(cost, goal, O.fmm2d(cost, goal))
    ref = d[p + "T"]
    assert np.array_equal(np.isfinite(T), np.isfinite(ref))
    f = np.isfinite(ref)
    assert np.array_equal(T[f], ref[f])


@pytest.mark.parametrize("i", [0, 2, 4])
def test_replay_bidirectional_is_the_reference(golden, i):
    d = golden("fmm2d_bidir")
    p = f"b{i}_"
    cost = d[p + "cost"].astype(np.float64)
    goal = tuple(int(v) for v in d[p + "goal"])
    start = tuple(int(v) for v in d[p + "start"])
    rng = np.random.default_rng(i)
    fields = []
    for s in (goal, start):
        F = O.fmm2d(cost, s)
        fields.append(F * (1 + rng.integers(-4, 5, F.shape) * 2.0 ** -52))  # a few ulps off
    TG, TS, join = R.bidir(cost, goal, start, *fields)
    assert np.array_equal(join, d[p + "join"])
    for A, B in ((TG, d[p + "TG"]), (TS, d[p + "TS"])):
        assert np.array_equal(A.view(np.uint64), B.view(np.uint64))
