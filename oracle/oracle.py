"""ctypes front-end of the CPU oracle (oracle/eikonal_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker and the timed CPU baseline.  The product never imports it.
Each function cites the reference line it restates (see the C file header for the full map).
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# ORACLE_LIB: tools/san.sh points it at the ASan/UBSan build (`make -C oracle san`)
LIB_PATH = os.environ.get("ORACLE_LIB", os.path.join(HERE, "liboracle.so"))

OK, ERR_ARG, ERR_NOMEM = 0, -1, -2
REF_STOPITERATION, REF_UNBOUND, REF_VALUEERROR, REF_INDEXERROR = 2, 3, 4, 5
GDM_DONE, GDM_FALLBACK, GDM_ERROR = 0, 1, 2
REF_ERR_NAMES = {REF_STOPITERATION: "StopIteration", REF_UNBOUND: "UnboundLocalError",
                 REF_VALUEERROR: "ValueError", REF_INDEXERROR: "IndexError"}

_lib = None
_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_ip = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_up = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
i64 = C.c_int64


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.orc_eikonal.restype = C.c_double
        L.orc_eikonal.argtypes = [C.c_double] * 3
        L.orc_fmm2d.argtypes = [_dp, i64, i64, i64, i64, i64, i64, _dp, C.POINTER(i64)]
        L.orc_fmm2d_bidir.argtypes = [_dp, i64, i64, i64, i64, i64, i64, _dp, _dp, _up]
        L.orc_gradient2d.argtypes = [_dp, i64, i64, C.c_int, C.c_double, C.c_double, _dp, _dp]
        L.orc_interp2.restype = C.c_double
        L.orc_interp2.argtypes = [C.c_double, C.c_double, _dp, i64, i64, C.POINTER(C.c_int)]
        L.orc_interp3.restype = C.c_double
        L.orc_interp3.argtypes = [C.c_double] * 3 + [_dp, i64, i64, i64, C.POINTER(C.c_int)]
        L.orc_gdm2d.argtypes = [_dp, i64, i64] + [C.c_double] * 5 + [_dp, i64, C.POINTER(i64), C.POINTER(C.c_int)]
        L.orc_fmm3d.argtypes = [_dp, i64, i64, i64, _ip, C.c_void_p, _dp]
        L.orc_fmm3d_trace.argtypes = [_dp, i64, i64, i64, _ip, C.c_void_p, _dp, _ip]
        L.orc_gdm3d.argtypes = [_dp, i64, i64, i64, _dp, _dp, C.c_double, _dp, i64, C.POINTER(i64),
                                C.POINTER(C.c_int)]
        L.orc_set_strict.argtypes = [C.c_int]
        L.orc_fmm2d_batch.argtypes = [_dp, i64, i64, i64, _ip, _dp, C.c_int]
        _lib = L
    return _lib


def set_strict(strict):
    """strict (default) reproduces the reference's StopIteration on tied decrease-keys."""
    lib().orc_set_strict(1 if strict else 0)


class RefError(RuntimeError):
    """The reference would raise here; .name is the Python exception it raises."""

    def __init__(self, code):
        self.code = code
        self.name = REF_ERR_NAMES.get(code, f"code{code}")
        super().__init__(self.name)


def _chk(rc):
    if rc in REF_ERR_NAMES:
        raise RefError(rc)
    if rc != OK:
        raise ValueError(f"oracle error {rc}")


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def eikonal(thor, tver, c):
    """getEikonal FastMarching.py:17-29"""
    return lib().orc_eikonal(float(thor), float(tver), float(c))


def fmm2d(cost, goal, start=None):
    """computeTmap FastMarching.py:92-112 (intended semantics; full field if start is None)."""
    cost = _f64(cost)
    H, W = cost.shape
    T = np.empty_like(cost)
    pops = i64(0)
    sx, sy = (-1, -1) if start is None else (int(start[0]), int(start[1]))
    _chk(lib().orc_fmm2d(cost, H, W, int(goal[0]), int(goal[1]), sx, sy, T, C.byref(pops)))
    return T


def fmm2d_bidir(cost, goal, start):
    """biComputeTmap FastMarching.py:114-162 -> (TG, TS, nodeJoin uint32[2])."""
    cost = _f64(cost)
    H, W = cost.shape
    TG, TS = np.empty_like(cost), np.empty_like(cost)
    join = np.zeros(2, np.uint32)
    _chk(lib().orc_fmm2d_bidir(cost, H, W, int(goal[0]), int(goal[1]), int(start[0]), int(start[1]), TG, TS, join))
    return TG, TS, join


def gradient2d(T, point=None):
    """computeGradient FastMarching.py:242-300 -> (Gnx, Gny)."""
    T = _f64(T)
    H, W = T.shape
    gx, gy = np.empty_like(T), np.empty_like(T)
    px, py = (0.0, 0.0) if point is None or len(point) == 0 else (float(point[0]), float(point[1]))
    _chk(lib().orc_gradient2d(T, H, W, 0 if point is None or len(point) == 0 else 1, px, py, gx, gy))
    return gx, gy


def interp2(point, M):
    """interpolatePoint FastMarching.py:305-338"""
    M = _f64(M)
    e = C.c_int(0)
    v = lib().orc_interp2(float(point[0]), float(point[1]), M, M.shape[0], M.shape[1], C.byref(e))
    _chk(e.value)
    return v


def interp3(point, M):
    """FastMarching3D.interpolatePoint :275-314"""
    M = _f64(M)
    e = C.c_int(0)
    v = lib().orc_interp3(float(point[0]), float(point[1]), float(point[2]), M, *M.shape, C.byref(e))
    _chk(e.value)
    return v


def gdm2d(T, init, end, tau=0.5, max_out=None):
    """getPathGDM FastMarching.py:164-236 -> (path (K,2), status)."""
    T = _f64(T)
    H, W = T.shape
    steps = int(round(15000 / tau))
    max_out = max_out or steps + 4
    out = np.empty((max_out, 2))
    n, st = i64(0), C.c_int(0)
    rc = lib().orc_gdm2d(T, H, W, float(init[0]), float(init[1]), float(end[0]), float(end[1]), float(tau),
                         out, max_out, C.byref(n), C.byref(st))
    if rc not in (OK,) and st.value != GDM_ERROR:
        _chk(rc)
    return out[: n.value].copy(), st.value


def fmm3d(cost, goal, start=None):
    """FastMarching3D.computeTmap :126-145"""
    cost = _f64(cost)
    H, W, L = cost.shape
    T = np.empty_like(cost)
    g = np.ascontiguousarray(goal, dtype=np.int64)
    s = None if start is None else np.ascontiguousarray(start, dtype=np.int64)
    _chk(lib().orc_fmm3d(cost, H, W, L, g, None if s is None else s.ctypes.data, T))
    return T


def fmm3d_trace(cost, goal, start=None):
    """fmm3d plus the pop order: (T, popidx) with popidx = 0 at the goal, k for the k-th pop of
    getMinNB (FastMarching3D.py:138), -1 for cells never popped."""
    cost = _f64(cost)
    H, W, L = cost.shape
    T = np.empty_like(cost)
    pop = np.empty(cost.shape, np.int64)
    g = np.ascontiguousarray(goal, dtype=np.int64)
    s = None if start is None else np.ascontiguousarray(start, dtype=np.int64)
    _chk(lib().orc_fmm3d_trace(cost, H, W, L, g, None if s is None else s.ctypes.data, T, pop))
    return T, pop


def fm3d_early_from_full(cost, Tf, goal, start):
    """The GPU's restatement of FastMarching3D.computeTmap's early exit (:141) on a converged full
    field Tf (eikonal_api.cpp eik_fim3d_early_exit): closed = {Tf < Tf[start]} + start (exact ties
    with start count as not yet popped) and the narrow band (finite cost, a closed 6-neighbour)
    keep Tf; +inf elsewhere.  start == goal / outside the volume -> Tf itself."""
    cost = _f64(cost)
    Tf = _f64(Tf)
    H, W, L = Tf.shape
    sx, sy, sz = (int(v) for v in start)
    if not (0 <= sx < W and 0 <= sy < H and 0 <= sz < L) or [sx, sy, sz] == [int(v) for v in goal]:
        return Tf.copy()
    ts = Tf[sy, sx, sz]
    closed = Tf < ts
    closed[sy, sx, sz] = True
    P = np.pad(closed, 1, constant_values=False)
    nb = (P[1:-1, :-2, 1:-1] | P[1:-1, 2:, 1:-1] | P[:-2, 1:-1, 1:-1] | P[2:, 1:-1, 1:-1] |
          P[1:-1, 1:-1, :-2] | P[1:-1, 1:-1, 2:])
    keep = closed | (nb & np.isfinite(cost))
    return np.where(keep, Tf, np.inf)


def gdm3d(T, init, end, tau=0.5, max_out=None):
    """FastMarching3D.getPathGDM :198-271 -> (path (K,3), status)."""
    T = _f64(T)
    H, W, L = T.shape
    steps = int(round(15000 / tau))
    max_out = max_out or steps + 4
    out = np.empty((max_out, 3))
    n, st = i64(0), C.c_int(0)
    lib().orc_gdm3d(T, H, W, L, _f64(init), _f64(end), float(tau), out, max_out, C.byref(n), C.byref(st))
    return out[: n.value].copy(), st.value


def fmm2d_batch(costs, goals, nthreads=1):
    """Full 2D fields of B independent maps (one map per thread)."""
    costs = _f64(costs)
    B, H, W = costs.shape
    T = np.empty_like(costs)
    _chk(lib().orc_fmm2d_batch(costs, B, H, W, np.ascontiguousarray(goals, dtype=np.int64), T, int(nthreads)))
    return T
