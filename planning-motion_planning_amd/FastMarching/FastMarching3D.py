"""Drop-in ``FastMarching.FastMarching3D`` (reference: src/FastMarching/FastMarching3D.py).

  computeTmap(costMap, goal, start)   FastMarching3D.py:126-145 -> GPU 3D block-FIM + early exit
  getPathGDM(T, init, end, tau)       FastMarching3D.py:198-271 -> GPU path kernel
Host-side scalar/list helpers keep their reference semantics: updateNode :19-101,
sumlist :103-107, getMinNB :109-123, interpolatePoint :275-314.

Layout as in the reference: cost[y, x, z], nodes (x, y, z).  computeTmap returns the reference's
PARTIAL field: its loop breaks once `start` is popped (:141), so cells popped before `start`
(T < T[start]) and `start` hold their final values (same as the full field, <= 1e-9), the narrow
band holds a tentative value (here: its converged full-field value, <= the reference's, whose
value depends on its sequential update order: within 3 %, tests/band.py) and every other cell +inf.  getPathGDM's np.gradient
(:200) sees those +inf cells, which is why the planner's end-effector path needs this field and
not the full one (tests/golden/fm3d_early.npz: identical paths on cubes and arm volumes).
start == goal, outside the volume or unreachable: the reference never pops it -> full field.
"""
import bisect
import os

import numpy as np
from numpy import array

from eikonal import default_context, PATH_ERROR
from eikonal._lib import OPT_EXACT_BAND

_DTYPE = np.float32 if os.environ.get("EIKONAL_DTYPE", "float64") in ("float32", "f32") else np.float64


def _ctx():
    return default_context(int(os.environ.get("EIKONAL_DEVICE", "0")))


def sumlist(listNum):
    """FastMarching3D.py:103-107 (right-associated sum)."""
    if len(listNum) == 1:
        return listNum[0]
    return listNum[0] + sumlist(listNum[1:])


def _solve(Tx, Ty, Tz, C):
    Tarray = [Tx, Ty, Tz]
    Tr = np.inf
    while Tr == np.inf:
        n = len(Tarray)
        Tmax = max(Tarray)
        sumT = 0
        for a in range(n):
            sumT = sumT + (Tmax - Tarray[a]) ** 2
        if C ** 2 > sumT:
            Tr = (sumlist(Tarray) + np.sqrt(n * C ** 2 + sumlist(Tarray) ** 2 - n * sumlist(array(Tarray) ** 2))) / n
        Tarray.remove(Tmax)
    return Tr


def _band_index(nbNodes, lo, c):
    """The band search of FastMarching3D.py:89 (same form as FastMarching.py:73): indices
    lo .. len(nbNodes) for lo >= 1 (IndexError past the end), only index 0 for lo == 0
    (StopIteration if c is not first)."""
    count = min(1, len(nbNodes)) if lo == 0 else len(nbNodes) - lo + 1
    for k in range(lo, lo + count):
        if np.array_equal(c, nbNodes[k]):
            return k
    raise StopIteration


def updateNode(nodeTarget, costMap, Tmap, nbT, nbNodes, closedMap):
    """FastMarching3D.py:19-101 narrow-band update (host bookkeeping on the caller's lists)."""
    for d in ([0, 0, -1], [0, 0, 1], [-1, 0, 0], [1, 0, 0], [0, 1, 0], [0, -1, 0]):
        c = np.add(nodeTarget, d)
        if closedMap[c[1], c[0], c[2]] != 0:
            continue
        T = _solve(min(Tmap[c[1], c[0] - 1, c[2]], Tmap[c[1], c[0] + 1, c[2]]),
                   min(Tmap[c[1] - 1, c[0], c[2]], Tmap[c[1] + 1, c[0], c[2]]),
                   min(Tmap[c[1], c[0], c[2] - 1], Tmap[c[1], c[0], c[2] + 1]), costMap[c[1], c[0], c[2]])
        if np.isinf(Tmap[c[1], c[0], c[2]]):
            i = bisect.bisect_left(nbT, T)
            nbT.insert(i, T)
            nbNodes.insert(i, c)
            Tmap[c[1], c[0], c[2]] = T
        elif T < Tmap[c[1], c[0], c[2]]:
            i = _band_index(nbNodes, bisect.bisect_left(nbT, Tmap[c[1], c[0], c[2]]), c)
            del nbT[i]
            del nbNodes[i]
            i = bisect.bisect_left(nbT, T)
            nbT.insert(i, T)
            nbNodes.insert(i, c)
            Tmap[c[1], c[0], c[2]] = T
    return Tmap, nbT, nbNodes


def getMinNB(nbT, nbNodes):
    """FastMarching3D.py:109-123"""
    node = nbNodes.pop(0)
    del nbT[0]
    return node, nbT, nbNodes


def interpolatePoint(point, mapI):
    """FastMarching3D.py:275-314 (trilinear, with the reference's a7 coefficient)."""
    i = np.uint32(np.fix(point[0]))
    j = np.uint32(np.fix(point[1]))
    k = np.uint32(np.fix(point[2]))
    a, b, c = point[0] - i, point[1] - j, point[2] - k
    a0 = mapI[j, i, k]
    a1 = mapI[j, i + 1, k] - mapI[j, i, k]
    a2 = mapI[j + 1, i, k] - mapI[j, i, k]
    a3 = mapI[j, i, k + 1] - mapI[j, i, k]
    a4 = mapI[j + 1, i + 1, k] + mapI[j, i, k] - mapI[j, i + 1, k] - mapI[j + 1, i, k]
    a5 = mapI[j, i + 1, k + 1] + mapI[j, i, k] - mapI[j, i + 1, k] - mapI[j, i, k + 1]
    a6 = mapI[j + 1, i, k + 1] + mapI[j, i, k] - mapI[j + 1, i, k] - mapI[j, i, k + 1]
    a7 = mapI[j + 1, i + 1, k + 1] + mapI[j, i, k] - mapI[j + 1, i, k] - mapI[j, i, k + 1] - mapI[j, i + 1, k]
    m, n, o = np.uint32(mapI.shape)
    if i == n:
        if j == m:
            return mapI[j, i, k] if k == o else c * mapI[j, i, k + 1] + (1 - c) * mapI[j, i, k]
        if k == o:
            return b * mapI[j + 1, i, k] + (1 - b) * mapI[j, i, k]
    elif j == m and k == o:
        return a * mapI[j, i + 1, k] + (1 - a) * mapI[j, i, k]
    return a0 + a1 * a + a2 * b + a3 * c + a4 * a * b + a5 * a * c + a6 * b * c + a7 * a * b * c


def computeTmap(costMap, goal, start=None):
    """FastMarching3D.py:126-145 -> T[y, x, z] (float64, inf = unreached), early exit at `start`
    (:141); start=None (no reference counterpart) returns the full field.  EIKONAL_EXACT_BAND=1 (fp64):
    the early-exit field's band values and ties exactly as the reference's sequential band
    (EIK_OPT_EXACT_BAND, csrc/bidir_exact.hip)."""
    cost = np.ascontiguousarray(costMap, dtype=_DTYPE)
    g = np.asarray(goal, dtype=np.int64).reshape(-1)[:3]
    s = None if start is None else np.asarray(start, dtype=np.int64).reshape(-1)[:3]
    c = _ctx()
    c.set_option(OPT_EXACT_BAND, 1 if os.environ.get("EIKONAL_EXACT_BAND", "0") not in ("", "0") else 0)
    return c.tmap3d(cost, g, dtype=_DTYPE, start=s).astype(np.float64, copy=False)


def getPathGDM(totalCostMap, initWaypoint, endWaypoint, tau):
    """FastMarching3D.py:198-271 -> (K, 3) float64 path."""
    path, status = _ctx().path3d(np.ascontiguousarray(totalCostMap, dtype=np.float64),
                                 np.asarray(initWaypoint, np.float64).reshape(-1)[:3],
                                 np.asarray(endWaypoint, np.float64).reshape(-1)[:3], float(tau))
    if status == PATH_ERROR:
        raise IndexError("getPathGDM (3D): the descent left the volume (the reference raises here too)")
    return path
