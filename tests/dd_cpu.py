"""CPU local solver for the domain-decomposition tests (TEST INFRASTRUCTURE, numpy).

Implements the duck-typed local-solver protocols of eikonal/dd.py (start / iterate /
pack_edges / merge_ghost / active for dd.solve; launch / begin / sync / end / release for
dd.solve_live over dd.P2PHalo) with a vectorised Jacobi Godunov iteration on one block
plus its ghost strips, so the rank-exchange logic of dd.solve can be exercised with the gloo
backend on CPU.  The GPU path plugs eikonal.Fim2d into the same driver (dd.GpuLocal).
"""
import numpy as np
import torch


def godunov(a, b, c):
    lo, hi = np.minimum(a, b), np.maximum(a, b)
    with np.errstate(invalid="ignore"):
        d = hi - lo
        t2 = 0.5 * (lo + hi + np.sqrt(np.maximum(2 * c * c - d * d, 0.0)))
    return np.where((hi == np.inf) | (c < d), lo + c, t2)


class CpuLocal:
    def __init__(self, cost, ghosts):
        self.cost = np.asarray(cost, np.float64)
        self.ghosts = ghosts  # torch tensors or None, order N S W E
        self.T = None
        self.dirty = False

    def start(self, goal):
        self.T = np.full(self.cost.shape, np.inf)
        for g in self.ghosts:
            if g is not None:
                g.fill_(float("inf"))
        if goal[0] >= 0:
            self.T[goal[1], goal[0]] = 0.0
        self.dirty = True

    def _padded(self):
        h, w = self.T.shape
        P = np.full((h + 2, w + 2), np.inf)
        P[1:-1, 1:-1] = self.T
        for side, sl in ((0, (0, slice(1, -1))), (1, (-1, slice(1, -1))), (2, (slice(1, -1), 0)),
                         (3, (slice(1, -1), -1))):
            if self.ghosts[side] is not None:
                P[sl] = self.ghosts[side].numpy()
        return P

    def _sweep(self):
        """one Jacobi sweep; returns whether T changed"""
        P = self._padded()
        a = np.minimum(P[1:-1, :-2], P[1:-1, 2:])
        b = np.minimum(P[:-2, 1:-1], P[2:, 1:-1])
        nv = np.minimum(self.T, godunov(a, b, self.cost))
        if np.array_equal(nv, self.T):
            return False
        self.T = nv
        return True

    def iterate(self, k):
        if not self.dirty:
            return
        while self._sweep():
            pass
        self.dirty = False

    # live protocol (dd.solve_live): the "concurrently running kernel" advances live_sweeps
    # Jacobi sweeps per round, so fronts cross blocks mid-solve as on the GPU
    live_sweeps = 3

    def launch(self, halo=None):
        self.changed, self.snap = 0, 1

    def begin(self):
        for _ in range(self.live_sweeps):
            if not self.dirty:
                break
            self.dirty = self._sweep()
        self.snap, self.changed = int(self.dirty), 0

    def sync(self):
        pass

    def end(self):
        return self.snap, self.changed

    def release(self):
        return int(self.dirty)

    def pack_edges(self, n, s, w, e):
        for t, v in ((n, self.T[0]), (s, self.T[-1]), (w, self.T[:, 0]), (e, self.T[:, -1])):
            if t is not None:
                t.copy_(torch.from_numpy(np.ascontiguousarray(v)))

    def merge_ghost(self, side, recv):
        g = self.ghosts[side]
        m = torch.minimum(g, recv)
        n = int((m < g).sum())
        if n:
            self.dirty = True
            self.changed = getattr(self, "changed", 0) + n
        g.copy_(m)

    def active(self):
        return int(self.dirty)


def godunov3(a, b, c, C):
    """FastMarching3D's n-D local solve (:59-75) on the axis minima a, b, c (the 3D Godunov update:
    three axes when C^2 exceeds the spread to the largest, else two, else one)."""
    s = np.sort(np.stack([a, b, c]), axis=0)
    s0, s1, s2 = s[0], s[1], s[2]
    with np.errstate(invalid="ignore", over="ignore"):
        t1 = s0 + C
        d = s1 - s0
        t2 = 0.5 * (s0 + s1 + np.sqrt(np.maximum(2 * C * C - d * d, 0.0)))
        q3 = 3 * C * C - 2 * ((s1 - s0) ** 2 + (s2 - s0) ** 2 - (s1 - s0) * (s2 - s0))
        t3 = (s0 + s1 + s2 + np.sqrt(np.maximum(q3, 0.0))) / 3.0
        three = C * C > (s2 - s0) ** 2 + (s2 - s1) ** 2
        two = C > d
    return np.where(three, t3, np.where(two, t2, t1))


class CpuLocalLayered(CpuLocal):
    """The layered protocol of eikonal/dd.py on CPU: a block [h][w][nl] of a few-layer volume, ghost
    strips of nl values per edge cell ([i][z] flattened), Jacobi sweeps of the n-D update with the
    layer neighbours inside the cell (FastMarching3D.py:21-57's six neighbours)."""

    def __init__(self, cost, ghosts):
        super().__init__(cost, ghosts)
        self.nl = self.cost.shape[2]

    def start(self, goal):
        self.T = np.full(self.cost.shape, np.inf)
        for g in self.ghosts:
            if g is not None:
                g.fill_(float("inf"))
        if goal[0] >= 0:
            self.T[goal[1], goal[0], goal[2]] = 0.0
        self.dirty = True

    def _padded(self):
        h, w, nl = self.T.shape
        P = np.full((h + 2, w + 2, nl), np.inf)
        P[1:-1, 1:-1] = self.T
        for side, sl in ((0, (0, slice(1, -1))), (1, (-1, slice(1, -1))), (2, (slice(1, -1), 0)),
                         (3, (slice(1, -1), -1))):
            if self.ghosts[side] is not None:
                P[sl] = self.ghosts[side].numpy().reshape(-1, nl)
        return P

    def _sweep(self):
        P = self._padded()
        a = np.minimum(P[1:-1, :-2], P[1:-1, 2:])
        b = np.minimum(P[:-2, 1:-1], P[2:, 1:-1])
        Z = np.full((self.T.shape[0], self.T.shape[1], self.nl + 2), np.inf)
        Z[:, :, 1:-1] = self.T
        c = np.minimum(Z[:, :, :-2], Z[:, :, 2:])
        nv = np.minimum(self.T, godunov3(a, b, c, self.cost))
        if np.array_equal(nv, self.T):
            return False
        self.T = nv
        return True

    def pack_edges(self, n, s, w, e):
        for t, v in ((n, self.T[0]), (s, self.T[-1]), (w, self.T[:, 0]), (e, self.T[:, -1])):
            if t is not None:
                t.copy_(torch.from_numpy(np.ascontiguousarray(v).reshape(-1)))
