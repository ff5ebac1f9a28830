"""Analyse a tools/trace.hip event log: every visit's phases and the solve's critical chain.

    python tools/trace_an.py out.bin

Event = type:4 | aux:8 | tile:20 | time:32 (10 ns ticks).  Types: 1..8 probe 0..7 (thread 0),
9 grab (aux = trigger bits), 10 activation of `tile` (aux = its state word before the OR).
The chain walks back from the last-retired visit through the activation that made each visit
pending (or the previous visit of the same tile for a self revisit) to the goal tile's first
visit, and splits every hop into wait (activation -> grab), stage (grab -> staged) and work
(staged -> the activation that triggered the next hop, counting passes).
"""
import sys
import numpy as np

kPending, kBusy, kSelf = 1, 2, 64


def load(path):
    with open(path, "rb") as f:
        N, grid, cap, ntx = np.frombuffer(f.read(16), dtype=np.int32)
        ev = np.frombuffer(f.read(), dtype=np.uint64).reshape(grid, cap)
    return int(N), int(grid), int(cap), int(ntx), ev


class Visit:
    __slots__ = ("wg", "tile", "trig", "grab", "start", "staged", "passes", "end", "fin", "acts", "cause")

    def __init__(self, wg, tile, trig, grab):
        self.wg, self.tile, self.trig, self.grab = wg, tile, trig, grab
        self.start = self.staged = self.end = self.fin = None
        self.passes = []   # [swept, drained]
        self.acts = []     # (time, target, old, passes_done)
        self.cause = None  # (time, producer Visit) or ("self", Visit)


def parse(ev):
    visits = []
    t0 = None
    for wg in range(ev.shape[0]):
        row = ev[wg]
        row = row[row != 0]
        typ = (row >> np.uint64(60)).astype(np.int64)
        aux = ((row >> np.uint64(52)) & np.uint64(0xff)).astype(np.int64)
        tile = ((row >> np.uint64(32)) & np.uint64(0xfffff)).astype(np.int64)
        tm = (row & np.uint64(0xffffffff)).astype(np.int64)
        cur = nxt = ret = None
        retiring = False
        for k in range(len(row)):
            ty, ax, tl, t = typ[k], aux[k], tile[k], tm[k]
            if ty == 9:
                nxt = Visit(wg, tl, ax, t)
            elif ty == 7:  # probe 6: after the grab barrier
                if nxt is not None:
                    cur, nxt = nxt, None
                    visits.append(cur)
                else:
                    cur = None
            elif ty == 1 and cur is not None:
                cur.start = t
            elif ty == 2 and cur is not None:
                cur.staged = t
            elif ty == 3 and cur is not None:
                cur.passes.append([t, None])
            elif ty == 8 and cur is not None and cur.passes:
                cur.passes[-1][1] = t
            elif ty == 4 and cur is not None:
                cur.end = t
                ret = cur
            elif ty == 5:
                retiring = True
            elif ty == 6:
                retiring = False
                if ret is not None:
                    ret.fin = t
                    ret = None
            elif ty == 10:
                v = ret if retiring else cur
                if v is not None:
                    v.acts.append((t, tl, ax, len(v.passes)))
    return visits


def main():
    N, grid, cap, ntx, ev = load(sys.argv[1])
    visits = parse(ev)
    if not visits:
        print("no visits")
        return
    # unwrap time relative to the first event (32-bit ticks; a solve lasts far less than 42 s)
    base = min(v.grab for v in visits)
    for v in visits:
        for f in ("grab", "start", "staged", "end", "fin"):
            x = getattr(v, f)
            if x is not None:
                setattr(v, f, (x - base) & 0xffffffff)
        v.passes = [[(a - base) & 0xffffffff, None if b is None else (b - base) & 0xffffffff] for a, b in v.passes]
        v.acts = [((t - base) & 0xffffffff, tl, ax, n) for t, tl, ax, n in v.acts]
    us = 0.01  # tick = 10 ns
    tend = max(v.fin or v.end or 0 for v in visits)
    print(f"N={N} grid={grid}: {len(visits)} visits, {sum(len(v.passes) for v in visits)} passes, span {tend * us:.1f} us")
    # phase statistics
    st = np.array([v.staged - v.grab for v in visits if v.staged is not None]) * us
    p1 = np.array([v.passes[0][0] - v.staged for v in visits if v.passes and v.staged is not None]) * us
    dr = np.array([v.passes[0][1] - v.passes[0][0] for v in visits if v.passes and v.passes[0][1] is not None]) * us
    ip = []
    for v in visits:
        for i in range(1, len(v.passes)):
            if v.passes[i - 1][1] is not None:
                ip.append(v.passes[i][0] - v.passes[i - 1][1])
    ip = np.array(ip) * us
    print(f"  grab->staged  mean {st.mean():6.2f} us  p50 {np.median(st):6.2f}")
    print(f"  first sweep   mean {p1.mean():6.2f} us  p50 {np.median(p1):6.2f}")
    print(f"  wback+drain   mean {dr.mean():6.2f} us  p50 {np.median(dr):6.2f}")
    if len(ip):
        print(f"  in-place pass (drained -> next swept) mean {ip.mean():6.2f} us  p50 {np.median(ip):6.2f}  n={len(ip)}")
    # causes
    by_tile = {}
    for v in visits:
        by_tile.setdefault(v.tile, []).append(v)
    acts_on = {}
    for v in visits:
        for (t, tl, ax, n) in v.acts:
            acts_on.setdefault(tl, []).append((t, ax, v, n))
    for tl in acts_on:
        acts_on[tl].sort(key=lambda x: x[0])
    for tl, vs in by_tile.items():
        vs.sort(key=lambda v: v.grab)
        prev_grab = -1
        for i, v in enumerate(vs):
            cand = [a for a in acts_on.get(tl, []) if prev_grab < a[0] <= v.grab and not (a[1] & kPending)]
            if cand:
                v.cause = ("act",) + cand[0]
            elif i > 0:
                v.cause = ("self", vs[i - 1])
            prev_grab = v.grab
    wait = np.array([v.grab - v.cause[1] for v in visits if v.cause and v.cause[0] == "act"]) * us
    print(f"  activation->grab mean {wait.mean():6.2f} us p50 {np.median(wait):6.2f}  (n={len(wait)}); self revisits {sum(1 for v in visits if v.cause and v.cause[0] == 'self')}")
    # critical chain from the last retirement
    last = max(visits, key=lambda v: v.fin or v.end or 0)
    chain = []
    v = last
    out_t = v.fin or v.end
    out_n = len(v.passes)
    seen = set()
    while v is not None and id(v) not in seen:
        seen.add(id(v))
        c = v.cause
        rec = {"tile": v.tile, "grab": v.grab, "staged": v.staged, "out": out_t, "npass": out_n,
               "in": None, "kind": "seed" if c is None else c[0], "trig": v.trig}
        if c is None:
            chain.append(rec)
            break
        if c[0] == "act":
            _, t, ax, prod, n = c
            rec["in"] = t
            rec["busy"] = bool(ax & kBusy)
            chain.append(rec)
            v, out_t, out_n = prod, t, n
        else:
            prev = c[1]
            rec["in"] = prev.fin or prev.end
            chain.append(rec)
            v, out_t, out_n = prev, prev.fin or prev.end, len(prev.passes)
    chain.reverse()
    W = sum((r["grab"] - r["in"]) for r in chain if r["in"] is not None) * us
    S = sum((r["staged"] - r["grab"]) for r in chain if r["staged"] is not None) * us
    K = sum((r["out"] - r["staged"]) for r in chain if r["staged"] is not None) * us
    npass = [r["npass"] for r in chain]
    kinds = {}
    for r in chain:
        kinds[r["kind"]] = kinds.get(r["kind"], 0) + 1
    print(f"  critical chain: {len(chain)} visits {kinds}, end {chain[-1]['out'] * us:.1f} us: wait {W:.1f} + stage {S:.1f} + work {K:.1f} us;"
          f" passes before hand-off mean {np.mean(npass):.2f}")
    wb = [(r["grab"] - r["in"]) * us for r in chain if r.get("busy") and r["in"] is not None]
    wf = [(r["grab"] - r["in"]) * us for r in chain if r.get("busy") is False and r["in"] is not None]
    print(f"  chain hops whose activation found the tile busy: {len(wb)} (wait mean {np.mean(wb) if wb else 0:.1f} us), "
          f"idle: {len(wf)} (wait mean {np.mean(wf) if wf else 0:.1f} us)")
    # every visit caused by an activation: the wait split the same way
    ab = [(v.grab - v.cause[1]) * us for v in visits if v.cause and v.cause[0] == "act" and (v.cause[2] & kBusy)]
    af = [(v.grab - v.cause[1]) * us for v in visits if v.cause and v.cause[0] == "act" and not (v.cause[2] & kBusy)]
    print(f"  all visits: busy at activation {len(ab)} (wait p50 {np.median(ab) if ab else 0:.1f} us), "
          f"idle {len(af)} (wait p50 {np.median(af) if af else 0:.1f} us)")
    first = chain[0]
    print(f"  chain start: grab {first['grab'] * us:.1f} us")
    for r in chain[:: max(1, len(chain) // 24)]:
        ty, tx = divmod(r["tile"], ntx)
        print(f"    tile ({ty:3d},{tx:3d}) {r['kind']:4s} trig {r['trig']:3d} in {('%.1f' % (r['in'] * us)) if r['in'] is not None else '-':>8s}"
              f" grab {r['grab'] * us:8.1f} staged {r['staged'] * us if r['staged'] is not None else -1:8.1f} out {r['out'] * us:8.1f} passes {r['npass']}")
    # busy workgroups over time (10 buckets)
    nb = 10
    busy = np.zeros(nb)
    for v in visits:
        e = v.end if v.end is not None else v.grab
        a, b = v.grab / tend * nb, e / tend * nb
        for k in range(int(a), min(nb, int(b) + 1)):
            lo, hi = max(a, k), min(b, k + 1)
            if hi > lo:
                busy[k] += hi - lo
    print("  busy WGs by tenth of the span:", " ".join(f"{x:.0f}" for x in busy))


if __name__ == "__main__":
    main()
