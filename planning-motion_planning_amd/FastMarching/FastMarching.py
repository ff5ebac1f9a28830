"""Drop-in ``FastMarching.FastMarching`` (reference: src/FastMarching/FastMarching.py).

Same function names, argument meaning and return types as the reference; the Eikonal solves,
the gradient and the path extraction run on the GPU (libeikonal.so via ctypes):

  computeTmap(costMap, goal, start)      FastMarching.py:92-112   -> GPU block-FIM, full field
  biComputeTmap(costMap, goal, start)    FastMarching.py:114-162  -> GPU fields + GPU join
  getPathGDM(T, init, end, tau)          FastMarching.py:164-236  -> GPU path kernel
  computeGradient(cost, point=[])        FastMarching.py:242-300  -> GPU gradient kernel

Scalar/list helpers that the reference exposes at module level keep their reference
semantics on the host (they operate on Python scalars and lists the caller owns):
  getEikonal :17-29, getNeighbours :31-42, updateNode :44-80, getMinNB :82-89,
  interpolatePoint :305-338.

Differences from the reference, by design:
  * computeTmap returns the full converged field (the reference raises ValueError at :107);
    with a `start` the values of every cell the reference would have closed are identical.
  * biComputeTmap returns the reference's PARTIAL goal/start fields (closed cells at their
    final values, the band at its final value where the reference holds a tentative one, the
    rest inf) and the join read from the two fronts' pop ranks.
  * the reference raises StopIteration on some tied decrease-keys (:72-73); the GPU solver has
    no narrow band and returns the intended field.  The host helper updateNode keeps that
    behaviour (and the IndexError of a search that runs past the band's end).
  * dtype: fields are computed in float64 by default (EIKONAL_DTYPE=float32 for fp32 speed).
"""
import bisect
import math
import os

import numpy as np

from eikonal import default_context, PATH_ERROR
from eikonal._lib import OPT_EXACT_BAND

_DTYPE = np.float32 if os.environ.get("EIKONAL_DTYPE", "float64") in ("float32", "f32") else np.float64


def _ctx():
    return default_context(int(os.environ.get("EIKONAL_DEVICE", "0")))


# ------------------------------------------------------------------ scalar / list helpers
def getEikonal(Thor, Tver, cost):
    """FastMarching.py:17-29 (scalar 2D Godunov update)."""
    if np.isinf(Thor):
        if np.isinf(Tver):
            return np.inf
        return Tver + cost
    if np.isinf(Tver):
        return Thor + cost
    if cost < np.abs(Thor - Tver):
        return np.minimum(Thor, Tver) + cost
    return .5 * (Thor + Tver + math.sqrt(2 * np.power(cost, 2) - np.power(Thor - Tver, 2)))


def getNeighbours(nodeTarget, closedMap):
    """FastMarching.py:31-42 (unused by the reference planner)."""
    out = []
    for d in ([-1, 0], [1, 0], [0, -1], [0, 1]):
        n = np.add(nodeTarget[0:2], d)
        if closedMap[n[1], n[0]] == 0:
            out.append(n)
    return out


def _band_index(nbNodes, lo, c):
    """The band search of FastMarching.py:73: enumerate(nbNodes[lo-1:], lo) visits the indices
    lo .. lo + len(nbNodes[lo-1:]) - 1.  For lo >= 1 that is lo .. len(nbNodes) (the last one is
    past the end: IndexError if c was not found before it); for lo == 0 the slice [-1:] holds one
    entry, so only index 0 is tested (StopIteration if c is not first)."""
    count = min(1, len(nbNodes)) if lo == 0 else len(nbNodes) - lo + 1
    for k in range(lo, lo + count):
        if np.array_equal(c, nbNodes[k]):
            return k
    raise StopIteration


def updateNode(nodeTarget, costMap, Tmap, nbT, nbNodes, closedMap):
    """FastMarching.py:44-80: narrow-band update of the four children of nodeTarget.
    Host bookkeeping on the caller's lists; the GPU solver does not use a narrow band."""
    for d in ([0, -1], [0, 1], [-1, 0], [1, 0]):
        c = np.add(nodeTarget, d)
        if closedMap[c[1], c[0]] != 0:
            continue
        Thor = np.minimum(Tmap[c[1], c[0] + 1], Tmap[c[1], c[0] - 1])
        Tver = np.minimum(Tmap[c[1] + 1, c[0]], Tmap[c[1] - 1, c[0]])
        T = getEikonal(Thor, Tver, costMap[c[1], c[0]])
        if np.isinf(Tmap[c[1], c[0]]):
            i = bisect.bisect_left(nbT, T)
            nbT.insert(i, T)
            nbNodes.insert(i, c)
            Tmap[c[1], c[0]] = T
        elif T < Tmap[c[1], c[0]]:
            i = _band_index(nbNodes, bisect.bisect_left(nbT, Tmap[c[1], c[0]]), c)
            del nbT[i]
            del nbNodes[i]
            i = bisect.bisect_left(nbT, T)
            nbT.insert(i, T)
            nbNodes.insert(i, c)
            Tmap[c[1], c[0]] = T
    return Tmap, nbT, nbNodes


def getMinNB(nbT, nbNodes):
    """FastMarching.py:82-89: pop the smallest entry of the sorted narrow band."""
    node = nbNodes.pop(0)
    del nbT[0]
    return node, nbT, nbNodes


def interpolatePoint(point, mapI):
    """FastMarching.py:305-338 (scalar bilinear interpolation with the reference's branches)."""
    i = np.uint32(np.fix(point[0]))
    j = np.uint32(np.fix(point[1]))
    a = point[0] - i
    b = point[1] - j
    m, n = np.uint32(mapI.shape)
    if i == n:
        if j == m:
            return mapI[j, i]
        return b * mapI[j + 1, i] + (1 - b) * mapI[j, i]
    if j == m:
        return a * mapI[j, i + 1] + (1 - a) * mapI[j, i]
    a00 = mapI[j, i]
    a10 = mapI[j, i + 1] - mapI[j, i]
    a01 = mapI[j + 1, i] - mapI[j, i]
    a11 = mapI[j + 1, i + 1] + mapI[j, i] - mapI[j, i + 1] - mapI[j + 1, i]
    if a == 0:
        return a00 if b == 0 else a00 + a01 * b
    return a00 + a10 * a if b == 0 else a00 + a10 * a + a01 * b + a11 * a * b


# ---------------------------------------------------------------------------- GPU paths
def _node(p):
    return int(p[0]), int(p[1])


def computeTmap(costMap, goal, start=None):
    """FastMarching.py:92-112 -> arrival-time field T (float64, inf = unreached)."""
    cost = np.ascontiguousarray(costMap, dtype=_DTYPE)
    T = _ctx().tmap2d(cost, _node(goal), dtype=_DTYPE)
    return T.astype(np.float64, copy=False)


def biComputeTmap(costMap, goal, start):
    """FastMarching.py:114-162 -> (TmapG, TmapS, nodeJoin uint32[2]).  EIKONAL_EXACT_BAND=1: the
    reference's own band values and LIFO ties, bit for bit (EIK_OPT_EXACT_BAND, csrc/bidir_exact.hip;
    ~6x the default's time on a 4096^2 raster)."""
    cost = np.ascontiguousarray(costMap, dtype=np.float64)
    c = _ctx()
    c.set_option(OPT_EXACT_BAND, 1 if os.environ.get("EIKONAL_EXACT_BAND", "0") not in ("", "0") else 0)
    TG, TS, join = c.tmap2d_bidir(cost, _node(goal), _node(start))
    return TG, TS, np.uint32(join)


def getPathGDM(totalCostMap, initWaypoint, endWaypoint, tau):
    """FastMarching.py:164-236 -> (K, 2) float64 path, first row init, last row end
    (a NaN-gradient fallback returns the reference's truncated path, :217-218)."""
    init = np.asarray(initWaypoint, dtype=np.float64).reshape(-1)[:2]
    end = np.asarray(endWaypoint, dtype=np.float64).reshape(-1)[:2]
    path, status = _ctx().path2d(np.ascontiguousarray(totalCostMap, dtype=np.float64), init, end, float(tau))
    if status == PATH_ERROR:
        raise IndexError("getPathGDM: the descent left the field (the reference raises here too)")
    return path


def computeGradient(cost, point=[]):
    """FastMarching.py:242-300 -> (Gnx, Gny): inf-aware normalised gradient; with a point only
    the window [int(p)-3, int(p)+3) is filled (zeros elsewhere), as in the reference."""
    T = np.ascontiguousarray(cost, dtype=np.float64)
    gx, gy = _ctx().gradient2d(T)
    if len(point) != 0:
        m, n = T.shape
        jmax, imax = min(m, int(point[1]) + 3), min(n, int(point[0]) + 3)
        jmin, imin = max(0, int(point[1] - 3)), max(0, int(point[0] - 3))
        mask = np.zeros_like(T, dtype=bool)
        mask[jmin:jmax, imin:imax] = True
        gx = np.where(mask, gx, 0.0)
        gy = np.where(mask, gy, 0.0)
    return gx, gy
