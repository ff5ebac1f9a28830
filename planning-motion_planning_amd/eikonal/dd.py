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
CPU tests) with start / iterate / pack_edges / merge_ghost / active.  A few-layer 3D volume splits
the same way in x-y, its layers kept together (eikonal.Fim3dLayered / GpuLocalLayered: strips of
nl values per edge cell).

solve_live is the GPU-native schedule (the default of bench.py at N > 1): ONE persistent launch
per rank stays up for the whole solve, serving its tile FIFO, while the host runs halo rounds
beside it on a side stream -- the front crosses a rank boundary within one round (~0.1-0.3 ms)
instead of waiting for the neighbour's whole local solve.  Edges go straight into the
neighbours' receive strips (IpcHalo: peer stores over xGMI into hipIpc-shared memory,
double-buffered by round parity); one small vote per round -- a shared-memory all-reduce
(NodeVote) on one node, else a gloo all-reduce -- is both the barrier for those stores and the
convergence test.
"""
import datetime

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


def make_strips(block, dtype, device, fill, per_cell=1):
    """send/recv strips and ghosts for the sides that have a neighbour (None elsewhere).
    per_cell: values per edge cell (a layered volume's block: its nl solved layers, [i][z])."""
    send, recv, ghost = [None] * 4, [None] * 4, [None] * 4
    for s in range(4):
        if block.nb[s] is not None:
            n = block.strip_len(s) * per_cell
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


class GpuLocalLayered(GpuLocal):
    """dd.solve adapter over eikonal.Fim3dLayered: a block of a few-layer 3D volume (SURVEY §8(e),
    C5: split in x-y, the layers stay together); ghosts of nl values per edge cell.  goal: the
    block-local (x, y, z) or x < 0."""

    def start(self, cost, T, goal, stream):
        for g in self.ghosts:
            if g is not None:
                g.fill_(float("inf"))
        self.fim.start(cost.data_ptr(), T.data_ptr(), goal, stream)
        self.last_active = 1


class HostStaged:
    """dd.solve adapter for a gloo group between processes that share one GPU (the shared-GPU
    rehearsals and tests): the device strips of a block solver are staged through host tensors
    (gloo moves CPU tensors; RCCL cannot put two ranks on one device -- on a node the strips go over
    RCCL directly).  dsend / drecv: the device strips; dd.solve is handed the host ones."""

    def __init__(self, loc, dsend, drecv):
        self.loc, self.dsend, self.drecv = loc, dsend, drecv

    def iterate(self, k):
        self.loc.iterate(k)

    def pack_edges(self, *hsend):
        self.loc.pack_edges(*self.dsend)
        for h, d in zip(hsend, self.dsend):
            if h is not None:
                h.copy_(d)

    def merge_ghost(self, side, hrecv):
        self.drecv[side].copy_(hrecv)
        self.loc.merge_ghost(side, self.drecv[side])

    def active(self):
        return self.loc.active()


# ------------------------------------------------------------------------- live schedule
OPP = {N_: S_, S_: N_, W_: E_, E_: W_}
ERR_MARK = 1 << 40  # carried through the all-reduce when a rank's solve failed


def control_group(timeout_s=120):
    """A gloo group for the per-round control all-reduce (CPU tensors, no GPU kernel)."""
    if dist.get_backend() == "gloo":
        return None
    return dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=timeout_s))


class NodeVote:
    """Per-round sum vote through shared memory (eik_node_allreduce): every rank on one node.
    Rank 0 creates the segment, the others attach; the name travels over `group`."""

    def __init__(self, group=None, timeout_s=60.0):
        import uuid

        from . import _lib as L

        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        self.nbytes = 64 * self.world
        name = [f"/eik_dd_{uuid.uuid4().hex[:12]}" if self.rank == 0 else None]
        dist.broadcast_object_list(name, src=0, group=group)
        if self.rank == 0:
            self.addr = L.node_shm_open(name[0], self.nbytes, True)
        dist.barrier(group=group)
        if self.rank != 0:
            self.addr = L.node_shm_open(name[0], self.nbytes, False)
        dist.barrier(group=group)
        if self.rank == 0:
            L.node_shm_unlink(name[0])  # every rank is attached: the name can go (no leak on a crash)
        self.round, self.timeout_s, self._L = 0, timeout_s, L

    def __call__(self, value):
        self.round += 1
        return self._L.node_allreduce(self.addr, self.rank, self.world, self.round, value, self.timeout_s)

    def close(self):
        if self.addr:
            self._L.node_shm_close(self.addr, self.nbytes)
            self.addr = None


def solve_live(local, block, halo, group=None, max_rounds=1000000, vote=None):
    """Drive one live solve to global convergence; returns the number of halo rounds.

    Round r (parity p = r & 1):  send (snapshot A_r: tiles pending or busy; then pack this rank's
    edges into the neighbours' strips of parity p)  ->  all-reduce of C_{r-1} (barrier for those
    stores; C = A + ghost cells lowered)  ->  merge the strips of parity p (C_r).
    C_{r-1} == 0 on every rank means: in round r-1 no tile was pending or busy anywhere when the
    edges were packed, and merging them lowered no ghost -- T was frozen from that snapshot on,
    so it is the global fixed point.  Stores of parity p land only after every rank has merged
    parity p of round r-2 (it has passed the all-reduce of round r-1)."""
    def total(v):
        if vote is not None:
            return vote(v)
        t = torch.tensor([v], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        return int(t.item())

    local.launch(halo)
    carry, rounds, ok, err = 1, 0, False, None
    try:
        while rounds < max_rounds:
            rounds += 1
            par = rounds & 1
            if err is None:
                try:
                    halo.send(local, par)
                except Exception as e:  # keep the collective schedule: the others must learn of it
                    err, carry = e, ERR_MARK
            tot = total(carry)
            if tot >= ERR_MARK:
                raise RuntimeError("live domain-decomposed solve failed on a rank") from err
            if tot == 0:
                ok = True
                return rounds
            try:
                a, c = halo.merge(local, par)
                carry = a + c
            except Exception as e:
                err, carry = e, ERR_MARK
        raise RuntimeError("live domain-decomposed solve did not converge")
    finally:
        rel_err = None
        try:
            left = local.release()
            if ok and left != 0:
                rel_err = RuntimeError(f"live solve released with {left} tiles still active")
        except Exception as e:
            rel_err = e
        if ok:
            # every rank left the round loop on the same vote; one more vote makes a release that
            # failed on ONE rank fail the solve on all of them (a caller that falls back -- bench.py --
            # must take the same branch everywhere)
            if total(ERR_MARK if rel_err is not None else 0) >= ERR_MARK:
                raise RuntimeError("live domain-decomposed solve: a rank's release failed") from rel_err


class P2PHalo:
    """Halo transport over torch.distributed P2P (gloo on CPU, RCCL on GPU): pack into local send
    strips, exchange, receive into the strip set of the round's parity.  The local solver exposes
    begin / pack_edges / sync / merge_ghost / end (tests/dd_cpu.py)."""

    def __init__(self, block, dtype, device, group=None):
        self.block, self.group = block, group
        self.send_strips, r0, _ = make_strips(block, dtype, device, float("inf"))
        _, r1, _ = make_strips(block, dtype, device, float("inf"))
        self._recv = (r0, r1)

    def send(self, local, par):
        local.begin()
        local.pack_edges(*self.send_strips)
        local.sync()
        exchange(self.block, self.send_strips, self._recv[par], self.group)

    def merge(self, local, par):
        for s in range(4):
            if self.block.nb[s] is not None:
                local.merge_ghost(s, self._recv[par][s])
        return local.end()


class IpcHalo:
    """Receive strips in hipIpc-shared device memory; the halo agent of a rank's live launch
    stores its edges directly into its neighbours' strips (peer stores over xGMI).  Strip
    (parity p, side s) of a block with sides h x w sits at byte ((p * 4 + s) * max(h, w)) * elem."""

    def __init__(self, ctx, block, elem_bytes, group=None):
        from . import _lib as L

        self.ctx, self.block, self.elem = ctx, block, elem_bytes
        slot = max(block.h, block.w) * elem_bytes
        self.buf = L.IpcBuffer(ctx, 8 * slot)
        self.base, self.slot = self.buf.ptr, slot
        handles = [None] * dist.get_world_size(group)
        dist.all_gather_object(handles, self.buf.handle, group=group)
        self.peers = {}
        self.targets = ([None] * 4, [None] * 4)
        self.recvs = ([None] * 4, [None] * 4)
        for s in range(4):
            nb = block.nb[s]
            if nb is None:
                continue
            if nb not in self.peers:
                self.peers[nb] = L.ipc_open(ctx, handles[nb])
            pb = Block(block.H, block.W, block.px, block.py, nb)
            pslot = max(pb.h, pb.w) * elem_bytes
            for par in (0, 1):
                self.targets[par][s] = self.peers[nb] + (par * 4 + OPP[s]) * pslot
                self.recvs[par][s] = self.base + (par * 4 + s) * slot

    def send(self, local, par):
        local.live_pack(par)

    def merge(self, local, par):
        return local.live_merge(par)

    def close(self):
        from . import _lib as L

        for p in self.peers.values():
            L.ipc_close(self.ctx, p)
        self.peers = {}
        self.buf.close()


class LiveGpuLocal(GpuLocal):
    """solve_live adapter over eikonal.Fim2d (persistent mode): one launch stays up per solve; its
    halo agent packs and merges on the host's command (halo.targets / halo.recvs strips)."""

    def launch(self, halo):
        self.fim.live_bind(halo.targets, halo.recvs)
        self.fim.launch(live=True)

    def live_pack(self, par):
        self.fim.live_pack(par)

    def live_merge(self, par):
        return self.fim.live_merge(par)

    def release(self):
        return self.fim.release()


class LiveGpuLocalLayered(LiveGpuLocal):
    """solve_live adapter over eikonal.Fim3dLayered: a block of a few-layer 3D volume
    on the live schedule -- the layered kernel's workgroup 0 is the halo agent, strips of nl values per
    edge cell (IpcHalo with elem_bytes = nl x the element size).  goal: the block-local (x, y, z) or
    x < 0."""

    def start(self, cost, T, goal, stream):
        GpuLocalLayered.start(self, cost, T, goal, stream)


def halo_consistent(block, T, ghosts, group=None):
    """After a converged solve every ghost strip equals the neighbour's final edge of T exactly
    (the last round packed the final edges and merged them).  Checks the halo transport end to
    end over `group` (CPU tensors); returns True on every rank iff it holds on all."""
    h, w = T.shape
    edges = [T[0, :], T[h - 1, :], T[:, 0], T[:, w - 1]]
    send = [edges[s].detach().cpu().contiguous() if block.nb[s] is not None else None for s in range(4)]
    recv = [torch.empty_like(send[s]) if send[s] is not None else None for s in range(4)]
    exchange(block, send, recv, group)
    ok = all(torch.equal(recv[s], ghosts[s].detach().cpu()) for s in range(4) if block.nb[s] is not None)
    t = torch.tensor([1 if ok else 0], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())
