"""Domain decomposition of one raster over R ranks with a halo exchange.

Each rank owns a block of the global H x W map, solves it with a local FIM solver whose
out-of-block neighbours are GHOST strips, and every `exchange_every` outer iterations:
  1. packs its four edge rows/columns,
  2. exchanges them point-to-point with its (<= 4) neighbours (torch.distributed P2P: RCCL
     over xGMI on the GPU box, gloo in the CPU tests),
  3. min-merges what it received into its ghosts; a ghost cell that decreased re-activates
     the adjacent edge tile,
  4. all-reduces the number of active tiles; the solve ends when it is zero everywhere.
Updates are monotone min-merges, so stale ghosts only delay convergence, never change the
fixed point.  The local solver is duck-typed (eikonal.Fim2d on the GPU; a numpy solver in the
CPU tests) with start / iterate / pack_edges / merge_ghost / active.
"""
import torch
import torch.distributed as dist

N_, S_, W_, E_ = 0, 1, 2, 3
SPLITS = {1: (1, 1), 2: (2, 1), 4: (2, 2), 8: (4, 2), 16: (4, 4)}  # ranks -> (px, py)


class Block:
    """Rank r's block of a px x py rank grid over a global H x W raster (row-major ranks)."""

    def __init__(self, H, W, px, py, rank):
        self.H, self.W, self.px, self.py, self.rank = H, W, px, py, rank
        self.rx, self.ry = rank % px, rank // px
        self.x0, self.x1 = (W * self.rx) // px, (W * (self.rx + 1)) // px
        self.y0, self.y1 = (H * self.ry) // py, (H * (self.ry + 1)) // py
        self.h, self.w = self.y1 - self.y0, self.x1 - self.x0
        nb = [None] * 4
        if self.ry > 0:
            nb[N_] = rank - px
        if self.ry + 1 < py:
            nb[S_] = rank + px
        if self.rx > 0:
            nb[W_] = rank - 1
        if self.rx + 1 < px:
            nb[E_] = rank + 1
        self.nb = nb

    def local_goal(self, gx, gy):
        if self.x0 <= gx < self.x1 and self.y0 <= gy < self.y1:
            return gx - self.x0, gy - self.y0
        return -1, -1

    def strip_len(self, side):
        return self.w if side in (N_, S_) else self.h


def make_strips(block, dtype, device, fill):
    """send/recv strips and ghosts for the sides that have a neighbour (None elsewhere)."""
    send, recv, ghost = [None] * 4, [None] * 4, [None] * 4
    for s in range(4):
        if block.nb[s] is not None:
            n = block.strip_len(s)
            send[s] = torch.full((n,), fill, dtype=dtype, device=device)
            recv[s] = torch.full((n,), fill, dtype=dtype, device=device)
            ghost[s] = torch.full((n,), fill, dtype=dtype, device=device)
    return send, recv, ghost


def exchange(block, send, recv, group=None):
    ops = []
    for s in range(4):
        if block.nb[s] is not None:
            ops.append(dist.P2POp(dist.isend, send[s], block.nb[s], group))
            ops.append(dist.P2POp(dist.irecv, recv[s], block.nb[s], group))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()


def solve(local, block, send, recv, exchange_every=8, max_rounds=100000, group=None, count_device=None):
    """Iterate the local solver with periodic halo exchanges until globally converged.
    Returns the number of exchange rounds."""
    dev = count_device if count_device is not None else send[next(i for i in range(4) if send[i] is not None)].device \
        if any(s is not None for s in send) else "cpu"
    rounds = 0
    while rounds < max_rounds:
        rounds += 1
        local.iterate(exchange_every)
        local.pack_edges(*send)
        exchange(block, send, recv, group)
        for s in range(4):
            if block.nb[s] is not None:
                local.merge_ghost(s, recv[s])
        act = torch.tensor([float(local.active())], device=dev)
        dist.all_reduce(act, op=dist.ReduceOp.SUM, group=group)
        if act.item() == 0:
            return rounds
    raise RuntimeError("domain-decomposed solve did not converge")


class GpuLocal:
    """dd.solve adapter over eikonal.Fim2d with torch-owned device buffers."""

    def __init__(self, fim, ghosts):
        self.fim = fim
        self.ghosts = ghosts
        self.last_active = 1
        fim.set_ghosts(*[g.data_ptr() if g is not None else None for g in ghosts])

    def start(self, cost, T, goal, stream):
        for g in self.ghosts:
            if g is not None:
                g.fill_(float("inf"))
        self.fim.start(cost.data_ptr(), T.data_ptr(), [goal], stream)
        self.last_active = 1

    def iterate(self, k):
        if self.last_active:
            self.last_active = self.fim.iterate(k)

    def pack_edges(self, n, s, w, e):
        self.fim.pack_edges(*[t.data_ptr() if t is not None else None for t in (n, s, w, e)])

    def merge_ghost(self, side, recv):
        self.fim.merge_ghost(side, recv.data_ptr())

    def active(self):
        self.last_active = self.fim.active()
        return self.last_active
