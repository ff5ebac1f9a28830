"""Edge cases of the host-only C/C++ sources for the sanitizer run (tools/san.sh): the
DEM parser's chunking across threads (more threads than lines, empty and blank lines, a last line
without a newline, ragged rows, malformed numbers), the rover tail's smallest inputs and its
buffer-capacity check, and the shared-memory vote across processes.  They also run in the normal
CPU suite against the regular library; under tools/san.sh ASan / UBSan watch every access.
Reference behaviour: Coupled_motion_planner.py:1098-1099 (DEM parse), :1228-1252 (rover tail)."""
import multiprocessing as mp
import os

import numpy as np
import pytest

from eikonal import _lib as L


def reference_parse(path):
    with open(path, "r") as file:  # Coupled_motion_planner.py:1098-1099
        return np.array([[float(num) for num in line.split(",")] for line in file])


@pytest.mark.parametrize("rows,cols", [(1, 1), (1, 9), (3, 2), (17, 1), (64, 31)])
@pytest.mark.parametrize("nthreads", [1, 2, 7, 64])
def test_dem_chunking(tmp_path, rows, cols, nthreads):
    rng = np.random.default_rng(rows * 100 + cols)
    Z = rng.normal(0, 1e3, (rows, cols))
    p = tmp_path / "dem.txt"
    text = "\n".join(",".join(repr(float(v)) for v in r) for r in Z)
    for trailing in ("", "\n"):  # with and without the final newline
        p.write_text(text + trailing)
        got = L.load_dem_txt(str(p), nthreads=nthreads)
        assert got.shape == (rows, cols) and np.array_equal(got, reference_parse(p))


@pytest.mark.parametrize("body", ["", "\n", "1,2\n3\n", "1,,2\n", "1,2,\n", "nan_x,1\n", "1e999999,1\n", "-1e999,2e-999\n", "inf,-Infinity\n",
                                  "1,2\n\n3,4\n",
                                  ",\n", "-\n", "1 2\n"])
def test_dem_malformed(tmp_path, body):
    p = tmp_path / "dem.txt"
    p.write_text(body)
    try:
        ref = reference_parse(p)
        ok = ref.ndim == 2 and ref.size > 0
    except (ValueError, OverflowError):
        ok = False
    if ok:
        got = L.load_dem_txt(str(p), nthreads=3)
        assert np.array_equal(got, ref, equal_nan=True)
    elif body == "1,2\n\n3,4\n":  # documented leniency: blank lines are skipped (the reference raises)
        assert np.array_equal(L.load_dem_txt(str(p), nthreads=3), [[1, 2], [3, 4]])
    else:
        with pytest.raises((ValueError, L.EikError)):
            L.load_dem_txt(str(p), nthreads=3)


def test_dem_large_many_threads(tmp_path):
    Z = np.random.default_rng(5).uniform(-50, 50, (300, 257))
    p = tmp_path / "dem.txt"
    np.savetxt(p, Z, delimiter=",", fmt="%.17g")
    for t in (3, 16, 300):
        assert np.array_equal(L.load_dem_txt(str(p), nthreads=t), reference_parse(p))


def test_rover_small_inputs_and_capacity():
    import planner

    Z = np.arange(16, dtype=np.float64).reshape(4, 4)
    one = np.array([[1.0, 1.0]])
    p, h = planner.assemble(one, one, Z, 0.1, 0.1, 0.1, 0.1, 0.0, 0.05)
    assert p.shape[1] == 3 and len(p) == len(h)
    pS = np.array([[1.0, 1.0], [2.0, 2.0], [2.5, 1.5]])
    pG = np.array([[1.0, 1.0], [0.0, 0.0], [3.0, 3.0]])
    q = L.RoverQuery()
    q.xm, q.ym, q.xr, q.yr, q.dist, q.resolution = 0.2, 0.2, 0.175, 0.125, 0.0, 0.05
    full, _ = L.rover_assemble(pS, pG, Z, q)
    if len(full) > 1:
        with pytest.raises(IndexError):  # the ABI reports a too-small output buffer, never overruns it
            L.rover_assemble(pS, pG, Z, q, cap=len(full) - 1)


def _vote(name, rank, world, rounds, q):
    try:
        addr = L.node_shm_open(name, 64 * world, False)
        tot = 0
        for r in range(1, rounds + 1):  # rounds count from 1 (0 is the zeroed segment's)
            tot += L.node_allreduce(addr, rank, world, r, rank + r, timeout_s=30.0)
        L.node_shm_close(addr, 64 * world)
        q.put((rank, tot))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))


@pytest.mark.parametrize("world", [2, 3])
def test_node_vote_processes(world):
    name = f"/eik_san_{os.getpid()}_{world}"
    rounds = 200
    addr = L.node_shm_open(name, 64 * world, True)
    try:
        ctx = mp.get_context("fork")
        q = ctx.Queue()
        ps = [ctx.Process(target=_vote, args=(name, r, world, rounds, q)) for r in range(world)]
        for p in ps:
            p.start()
        got = dict(q.get(timeout=120) for _ in ps)
        for p in ps:
            p.join(30)
        want = sum(sum(k + r for k in range(world)) for r in range(1, rounds + 1))
        assert all(v == want for v in got.values()), got
    finally:
        L.node_shm_close(addr, 64 * world)
        L.node_shm_unlink(name)
