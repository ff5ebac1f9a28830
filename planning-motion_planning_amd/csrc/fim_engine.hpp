// fim_engine.hpp -- the tile-queue engine shared by the 2D (fim2d.hip) and layered
// (fim2dl.hip) block-FIM solvers: per-tile queue state, coherent T access policy, activation of
// neighbour tiles (list mode / persistent FIFO) and the persistent driver's grab / finish.
// See fim2d.hip for the algorithm and the memory-model recipe these follow.
#pragma once
#include "eik_common.hpp"
#include "eik_kernels.hpp"

namespace eik {

// quadrant sweeps (fim2d.hip sweep_quadrant, fim2dl.hip sweep_layered): software pipeline depth
// in steps, and the +inf guard rows above and below the staged tile that its per-group row clamp
// needs
constexpr int kAhead = 4;
constexpr int kGuard = kAhead;

// per-tile queue state (persistent mode): pending / busy, plus what activated the tile since its
// last visit -- a halo side that improved (its information flows away from that side) or the
// tile itself (last visit changed it: every direction)
constexpr unsigned kPending = 1u, kBusy = 2u;
constexpr unsigned kFromN = 4u, kFromS = 8u, kFromW = 16u, kFromE = 32u, kSelf = 64u;
// set by the first grab of a tile and never cleared within a solve: a tile without it is FRESH --
// its T is still +inf everywhere, and its first activation is the front arriving
constexpr unsigned kVisited = 128u;

// Quadrant sweeps that can carry the triggering information: wave 0 (+x,+y) and 1 (-x,+y) move
// it away from the north edge, 2 and 3 from the south; 0 and 2 from the west, 1 and 3 from the
// east.  A visit that runs a subset and changes nothing is still a fixed point of the local
// update (every cell was evaluated against final neighbours); one that changes something
// re-activates itself with kSelf, i.e. all four.
__device__ __forceinline__ unsigned sweep_dirs(unsigned trig) {
    if (trig & kSelf) return 0xFu;
    unsigned d = 0;
    if (trig & kFromN) d |= 0x3u;
    if (trig & kFromS) d |= 0xCu;
    if (trig & kFromW) d |= 0x5u;
    if (trig & kFromE) d |= 0xAu;
    return d ? d : 0xFu;
}
// profiling hooks (tools/qprof.hip phase timers, tools/trace.hip event logs); no-ops here
#ifndef EIK_PROBE
#define EIK_PROBE(k) ((void)0)
#endif
#ifndef EIK_VISIT
#define EIK_VISIT(tile, trig, dirs) ((void)0)
#endif
#ifndef EIK_ACT
#define EIK_ACT(tile, old) ((void)0)
#endif
#ifndef EIK_KSTART
#define EIK_KSTART() ((void)0)
#endif

// ------------------------------------------------------------------- memory access policy
// Plain accesses (LIST mode) or coherent sc1 buffer accesses (PERSISTENT mode).
template <typename R, bool COH>
struct TMem;

template <typename R>
struct TMem<R, false> {
    R* p;
    TMem() = default;
    __device__ TMem(R* base, int64_t) : p(base) {}
    __device__ R ld(int64_t i) const { return p[i]; }
    __device__ void ld4(int64_t i, R (&v)[4]) const {
        if constexpr (sizeof(R) == 4) {
            const float4 t = *reinterpret_cast<const float4*>(p + i);
            v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
        } else {
            const double2 t0 = *reinterpret_cast<const double2*>(p + i);
            const double2 t1 = *reinterpret_cast<const double2*>(p + i + 2);
            v[0] = t0.x; v[1] = t0.y; v[2] = t1.x; v[3] = t1.y;
        }
    }
    __device__ void st(int64_t i, R v) const { p[i] = v; }
    __device__ void st4(int64_t i, const R (&v)[4]) const {
        if constexpr (sizeof(R) == 4) {
            *reinterpret_cast<float4*>(p + i) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
            *reinterpret_cast<double2*>(p + i) = make_double2(v[0], v[1]);
            *reinterpret_cast<double2*>(p + i + 2) = make_double2(v[2], v[3]);
        }
    }
};

constexpr int kSC1 = 16;  // aux cache-policy bits of the raw buffer builtins: sc1 (agent coherence)
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <typename R>
struct TMem<R, true> {
    __amdgpu_buffer_rsrc_t rs;
    // n * sizeof(R) < 2^32 is checked by the host before it selects this mode (fim2dl.hip: one
    // resource per layer and tile)
    TMem() = default;
    __device__ TMem(R* base, int64_t n)
        : rs(__builtin_amdgcn_make_buffer_rsrc(base, 0, (int)(uint32_t)(n * (int64_t)sizeof(R)), 0x00020000)) {}
    __device__ R ld(int64_t i) const {
        const unsigned off = (unsigned)(i * (int64_t)sizeof(R));
        if constexpr (sizeof(R) == 4) {
            return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, kSC1));
        } else {
            const u32x2 u = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, kSC1);
            return __longlong_as_double((long long)(((unsigned long long)u[1] << 32) | u[0]));
        }
    }
    __device__ void ld4(int64_t i, R (&v)[4]) const {
        const unsigned off = (unsigned)(i * (int64_t)sizeof(R));
        if constexpr (sizeof(R) == 4) {
            const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kSC1);
            v[0] = __uint_as_float(u[0]); v[1] = __uint_as_float(u[1]);
            v[2] = __uint_as_float(u[2]); v[3] = __uint_as_float(u[3]);
        } else {
            const u32x4 u0 = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kSC1);
            const u32x4 u1 = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, kSC1);
            v[0] = __longlong_as_double((long long)(((unsigned long long)u0[1] << 32) | u0[0]));
            v[1] = __longlong_as_double((long long)(((unsigned long long)u0[3] << 32) | u0[2]));
            v[2] = __longlong_as_double((long long)(((unsigned long long)u1[1] << 32) | u1[0]));
            v[3] = __longlong_as_double((long long)(((unsigned long long)u1[3] << 32) | u1[2]));
        }
    }
    __device__ void st(int64_t i, R v) const {
        const unsigned off = (unsigned)(i * (int64_t)sizeof(R));
        if constexpr (sizeof(R) == 4) {
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, off, 0, kSC1);
        } else {
            const unsigned long long b = (unsigned long long)__double_as_longlong(v);
            const u32x2 u = {(unsigned)b, (unsigned)(b >> 32)};
            __builtin_amdgcn_raw_buffer_store_b64(u, rs, off, 0, kSC1);
        }
    }
    __device__ void st4(int64_t i, const R (&v)[4]) const {
        const unsigned off = (unsigned)(i * (int64_t)sizeof(R));
        if constexpr (sizeof(R) == 4) {
            const u32x4 u = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
            __builtin_amdgcn_raw_buffer_store_b128(u, rs, off, 0, kSC1);
        } else {
            unsigned long long b[4];
            for (int k = 0; k < 4; ++k) b[k] = (unsigned long long)__double_as_longlong(v[k]);
            const u32x4 u0 = {(unsigned)b[0], (unsigned)(b[0] >> 32), (unsigned)b[1], (unsigned)(b[1] >> 32)};
            const u32x4 u1 = {(unsigned)b[2], (unsigned)(b[2] >> 32), (unsigned)b[3], (unsigned)(b[3] >> 32)};
            __builtin_amdgcn_raw_buffer_store_b128(u0, rs, off, 0, kSC1);
            __builtin_amdgcn_raw_buffer_store_b128(u1, rs, off + 16, 0, kSC1);
        }
    }
};

// Scoped loads / stores of one value (float or double) through its bit pattern.
template <typename R>
__device__ __forceinline__ R ld_agent(const R* p) {
    if constexpr (sizeof(R) == 4) {
        return __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT));
    } else {
        return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(p),
                                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
}
template <typename R>
__device__ __forceinline__ R ld_system(const R* p) {
    if constexpr (sizeof(R) == 4) {
        return __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_SYSTEM));
    } else {
        return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(p),
                                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    }
}
template <typename R>
__device__ __forceinline__ void st_scoped(R* p, R v, int scope) {
    if constexpr (sizeof(R) == 4) {
        if (scope == __HIP_MEMORY_SCOPE_SYSTEM)
            __hip_atomic_store(reinterpret_cast<unsigned*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        else
            __hip_atomic_store(reinterpret_cast<unsigned*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        const unsigned long long b = (unsigned long long)__double_as_longlong(v);
        if (scope == __HIP_MEMORY_SCOPE_SYSTEM)
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        else
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <typename R, bool COH>
__device__ __forceinline__ R load_T(const Fim2dArgs& a, const TMem<R, COH>& T, int64_t gy, int64_t gx) {
    constexpr R INF = Real<R>::inf();
    if (gy >= 0 && gy < a.H && gx >= 0 && gx < a.W) return T.ld(gy * a.W + gx);
    // ghost strips: the merge kernel lowers them between list launches, or DURING a live
    // persistent launch -- there they are read like T (agent-scope loads, L1 bypassed)
    auto g = [&](int side, int64_t i) -> R {
        const R* p = static_cast<const R*>(a.ghost[side]);
        if (!p) return INF;
        return COH ? ld_agent(p + i) : p[i];
    };
    if (gy == -1 && gx >= 0 && gx < a.W) return g(0, gx);
    if (gy == a.H && gx >= 0 && gx < a.W) return g(1, gx);
    if (gx == -1 && gy >= 0 && gy < a.H) return g(2, gy);
    if (gx == a.W && gy >= 0 && gy < a.H) return g(3, gy);
    return INF;
}

// -------------------------------------------------------------------- activation helpers
// LIST mode: append to the next iteration's list (dedup by mark).
__device__ __forceinline__ void enqueue(const Fim2dArgs& a, int tile, int list, unsigned stamp, float key) {
    if (a.delta < __builtin_inff()) {  // ordered mode only: keep the entering-T keys
        const unsigned kb = __float_as_uint(key);  // non-negative: float order == unsigned order
        atomicMin(&a.key[tile], kb);
        // one shared word per list: read first, so only a new minimum pays the contended atomic
        if (kb < __hip_atomic_load(&a.minkey[list], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            atomicMin(&a.minkey[list], kb);
    }
    if (atomicMax(&a.mark[tile], stamp) < stamp) {
        const int pos = atomicAdd(&a.counts[list], 1);
        a.lists[(int64_t)list * a.capacity + pos] = tile;
    }
}

// PERSISTENT mode: a FIFO of tiles, consumers take tickets (qgrab), producers append at the tail.
// A FRESH tile's first activation is the front advancing into it, and the front's advance is the
// solve's critical path (tools/trace.hip: on the 4096^2 DEM the chain of first visits from the
// goal to the far corner waited 766 us of a 2.1 ms solve behind re-visits of tiles the front had
// already passed).  So while the FIFO has a backlog (tail ahead of head: no workgroup waiting) a
// fresh tile takes the slot of the NEXT ticket to be issued -- a CAS on that slot's old entry,
// which is re-appended at the tail -- instead of queueing behind the backlog.  (A separate
// priority FIFO polled by every grabber was tried: hundreds of workgroups CAS-ing its head
// serialised for hundreds of microseconds.)
__device__ __forceinline__ void qslot_put(const Fim2dArgs& a, int tile) {
    const unsigned long long pos = atomicAdd(a.qtail, 1ull);
    __hip_atomic_store(&a.qslot[pos & a.qmask], (unsigned)tile + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void qslot_put_front(const Fim2dArgs& a, int tile) {
    const unsigned long long h = __hip_atomic_load(a.qhead, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long t = __hip_atomic_load(a.qtail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t > h + 1ull) {  // a backlog: slot h (the next ticket's) is filled, or about to be
        unsigned* slot = &a.qslot[h & a.qmask];
        const unsigned v = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // the ticket holder takes its slot with an exchange, so a CAS that wins lands before it
        if (v != 0u && atomicCAS(slot, v, (unsigned)tile + 1u) == v) {
            qslot_put(a, (int)(v - 1u));  // the displaced tile goes to the back (still pending)
            return;
        }
    }
    qslot_put(a, tile);
}
// Queue the tile unless it is already pending (nothing to do) or busy (its processor re-queues it
// when it finishes).
#ifndef EIK_ACT_SPLIT
#define EIK_ACT_SPLIT 1  // in-place passes use the split halves below (fim2d.hip, fim2dl.hip)
#endif
// Split in two halves (EIK_ACT_SPLIT): the state word's atomicOr (qpush_issue) and the queueing
// its old value decides (qpush_complete), so a busy tile's in-place pass can issue the first at the
// pass boundary and finish the second inside its next sweep.  Between the two the neighbour is
// PENDING but not yet queued: other activations of it do nothing (its entry is on the way), and
// the activating tile is still busy, so the active count stays above zero.
// ---------------------------------------------------------------- priority bands (EIK_OPT_PRIO)
// The FIFO serves tiles in activation order.  With a backlog (every workgroup busy, tiles waiting:
// the middle of a large solve) that order processes tiles far ahead of the front's settled region,
// whose halos are still coarse, and they are visited again.  tools/sched_sim.c (lock-step, 512
// workers): serving the waiting tiles lowest entering T first takes C2 108 -> 90 rounds and
// 40.6k -> 33.1k passes, an 8192^2 raster 265 -> 190 rounds (Dijkstra order at tile level; a
// bucket queue of width 250-1000 on C2 does as well as the exact heap).  The device form:
//  * a tile that becomes pending goes to the FIFO when a workgroup waits there (no backlog: order
//    is moot and the waiter takes it at once), else to band min(T / pdelta, kBands - 1): kBands
//    FIFOs of tile ids with their own head / tail words; pdelta = 64 x the geometric mean of the
//    finite costs (prio_delta_kernel; about one tile width of T) x EIK_OPT_PRIO;
//  * a pending tile activated again with a key a whole band lower gets a second entry in the lower
//    band (decrease-key: the sim's lazy re-push; a bucket that kept its first entry did worse than the
//    FIFO, 170 vs 108 rounds); whichever entry is taken first claims the tile, the others are stale
//    and are dropped when taken (the claim is a CAS pending -> busy on the state word);
//  * every workgroup looking for work takes a FIFO ticket; the oldest waiter (its ticket is the next
//    slot to be filled) moves up to 32 band entries to the FIFO's tail, lowest bands first
//    (band_dispatch), so the band heads see one claimant at a time.
// a.key[tile] holds the smallest key since the tile's last claim (atomicMin at each activation).
__device__ __forceinline__ unsigned band_of(const Fim2dArgs& a, float k) {
    const float q = k / *a.pdelta;  // k >= 0 (or +inf); a kernel-constant word (scalar cache)
    return q < float(kBands - 1) ? (unsigned)q : unsigned(kBands - 1);
}
#ifndef EIK_QDEBUG
#define EIK_QDEBUG 0
#endif
// queue counters for tools (eik_fim2d_qcount): a.visits[3 + i] -- 0 FIFO slot polls, 1 tail polls
// (priority mode), 2 band dispatch attempts, 3 / 4 claims won / stale entries dropped, 5 dispatches
// that moved entries, 6 decrease-key entries, 7 band entries put
__device__ __forceinline__ void qcount(const Fim2dArgs& a, int i) {
    if (EIK_QDEBUG) atomicAdd(a.visits + 3 + i, 1ull);
}
// A band is a ring of bmask + 1 slots (eikonal_api.cpp: a power of two >= 2 x the tiles,
// EIK_OPT_PRIO_RING).  At most ONE entry per (tile, band) exists at any time: a.bmem[tile] bit b is
// set by the put (an atomicOr whose old value says whether an entry is already there) and cleared
// by the workgroup that takes the entry from the FIFO, before its claim (qgrab_prio).  A put that
// finds the bit set is dropped -- the tile's entry already waiting in band b (stale from an earlier
// pending episode, or this episode's) is taken in its place, and since the put made the tile
// PENDING before its bit test, that entry's claim, which clears the bit before its CAS, serves it.
// So a band holds at most `tiles` entries and its ring cannot lap.  (Round 5 without the bits:
// stale entries of a long live DD launch's many episodes piled up in the bands until a ring of 2 x
// the tiles lapped -- the 4 x 2 live test's launch ended on qerror bit 4, profiles/
// r05as_tests_live_4x2_fail.log)  The lap check stays for a ring forced below the
// tile count (EIK_OPT_PRIO_RING, tests): qerror bit 4, and eik_fim2d_solve re-solves on the FIFO.
__device__ __forceinline__ void band_put_slot(const Fim2dArgs& a, unsigned b, int tile) {
    const unsigned long long hd = __hip_atomic_load(&a.bctl[16 * b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long pos = atomicAdd(&a.bctl[16 * b + 8], 1ull);
    if (pos > hd + a.bmask) atomicOr(a.qerror, 4u);
    __hip_atomic_store(&a.bslot[(size_t)b * (a.bmask + 1ull) + (pos & a.bmask)], (unsigned)tile + 1u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void band_put(const Fim2dArgs& a, unsigned b, int tile) {
    const unsigned long long bit = 1ull << b;
    if (atomicOr(&a.bmem[tile], bit) & bit) return;  // the tile's entry in band b serves this put
    qcount(a, 7);
    band_put_slot(a, b, tile);
}
// a newly pending tile with key k (priority mode): to a waiting workgroup (a ticket past the
// filled slots), else to its band.
__device__ __forceinline__ void prio_put(const Fim2dArgs& a, int tile, float k) {
    const unsigned long long h = __hip_atomic_load(a.qhead, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long t = __hip_atomic_load(a.qtail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (h > t)
        qslot_put(a, tile);
    else
        band_put(a, band_of(a, k), tile);
}
// The same with the membership bit set beside the head / tail loads (one round trip for both), given
// back when the tile goes to the FIFO instead -- meanwhile another put of this pending tile to band b
// is dropped, which is safe: the FIFO entry serves it.  For qfinish (a visit's retirement, off the
// sweeps' register peak); inside a sweep (qpush_complete in the split activations) the serial form
// above keeps the fp64 kernel at two workgroups per CU.
__device__ __forceinline__ void prio_put_overlap(const Fim2dArgs& a, int tile, float k) {
    const unsigned b = band_of(a, k);
    const unsigned long long bit = 1ull << b;
    const unsigned long long had = atomicOr(&a.bmem[tile], bit) & bit;
    const unsigned long long h = __hip_atomic_load(a.qhead, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long t = __hip_atomic_load(a.qtail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (h > t) {
        if (!had) atomicAnd(&a.bmem[tile], ~bit);
        qslot_put(a, tile);
    } else if (!had) {
        qcount(a, 7);
        band_put_slot(a, b, tile);
    }
}
// claim a taken entry: pending -> busy (stale entries -- the tile busy, or no longer pending -- fail).
// cleared: the entry came from a band and its membership bit was just cleared (qgrab_prio) -- that
// clear is in flight beside the state load below, which may have been served before it.  A put that
// still saw the bit made the tile pending before it (and returned), so when the load says "not
// claimable" the state is loaded again once the clear has completed: a pending tile whose put was
// dropped for this entry is served by this claim, never left without an entry.
__device__ __forceinline__ bool prio_claim(const Fim2dArgs& a, int tile, unsigned& trig, bool cleared = false) {
    unsigned old = __hip_atomic_load(&a.qstate[tile], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the clear, too)
    if (cleared && ((old & kBusy) || !(old & kPending)))
        old = __hip_atomic_load(&a.qstate[tile], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
        if ((old & kBusy) || !(old & kPending)) return false;
        const unsigned prev = atomicCAS(&a.qstate[tile], old, kBusy | kVisited);
        if (prev == old) {
            trig = old;
            __hip_atomic_store(&a.key[tile], 0x7f800000u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return true;
        }
        old = prev;
    }
}

__device__ __forceinline__ unsigned qpush_issue(const Fim2dArgs& a, int tile, unsigned trig) {
    const unsigned old = atomicOr(&a.qstate[tile], kPending | trig);
    EIK_ACT(tile, old);
    return old;
}
// priority mode: the key's atomicMin beside the state word's atomicOr (both in flight together)
__device__ __forceinline__ unsigned qpush_issue_key(const Fim2dArgs& a, int tile, unsigned trig, float k, unsigned& kold) {
    kold = atomicMin(&a.key[tile], __float_as_uint(k));  // k >= 0: float order == unsigned order
    return qpush_issue(a, tile, trig);
}
__device__ __forceinline__ void qpush_complete(const Fim2dArgs& a, int tile, unsigned old, float k = 0.f,
                                               unsigned kold = 0x7f800000u) {
    if ((old & (kPending | kBusy)) == 0u) {
        atomicAdd(a.qactive, 1);  // before the slot store: a waiter never sees "empty and idle"
        if (a.bctl)  // (EIK_OPT_FRESH_FIRST on the bands: a fresh tile -- the front advancing -- keyed 0)
            prio_put(a, tile, a.fresh_first && !(old & kVisited) ? 0.f : fminf(k, __uint_as_float(kold)));
        else if (!(old & kVisited) && a.fresh_first)
            qslot_put_front(a, tile);
        else
            qslot_put(a, tile);
    } else if (a.bctl && !(old & kBusy)) {  // queued: a lower band gets a second entry (decrease-key)
        const unsigned b = band_of(a, k);
        if (b < band_of(a, __uint_as_float(kold))) {
            qcount(a, 6);
            band_put(a, b, tile);
        }
    }
}
__device__ __forceinline__ void qpush(const Fim2dArgs& a, int tile, unsigned trig, float k = 0.f) {
    if (a.bctl) {
        unsigned kold;
        const unsigned old = qpush_issue_key(a, tile, trig, k, kold);
        qpush_complete(a, tile, old, k, kold);
        return;
    }
    qpush_complete(a, tile, qpush_issue(a, tile, trig));
}

__device__ __forceinline__ void activate(const Fim2dArgs& a, int tile, int list, unsigned stamp, float key,
                                         unsigned trig) {
    if (a.mode == kModePersistent)
        qpush(a, tile, trig, key);
    else
        enqueue(a, tile, list, stamp, key);
}

// Neighbour activations of a write-back with flags f: thread q in 1..4 handles one side (their
// atomics overlap); thread 0 flags changed subdomain edges for the halo exchange.  (`tid`: the
// caller's index for this role -- a lane of any one wave may serve, fim2d.hip's follow-through.)
__device__ __forceinline__ void activate_neighbours(const Fim2dArgs& a, int tile, unsigned f, const unsigned* key,
                                                    int list, unsigned stamp, int tid = threadIdx.x) {
    if (tid >= 5) return;
    const int map = tile / a.tiles_per_map;
    const int rem = tile - map * a.tiles_per_map;
    const int ty = rem / a.ntx, tx = rem - (rem / a.ntx) * a.ntx;
    const int base = map * a.tiles_per_map;
    const float kk = __uint_as_float(key[tid]);
    // (this tile's north edge is the north neighbour's south halo, ...)
    if (tid == 1 && (f & 1u) && ty > 0) activate(a, base + rem - a.ntx, list, stamp, kk, kFromS);
    if (tid == 2 && (f & 2u) && ty + 1 < a.nty) activate(a, base + rem + a.ntx, list, stamp, kk, kFromN);
    if (tid == 3 && (f & 4u) && tx > 0) activate(a, base + rem - 1, list, stamp, kk, kFromE);
    if (tid == 4 && (f & 8u) && tx + 1 < a.ntx) activate(a, base + rem + 1, list, stamp, kk, kFromW);
    if (tid == 0 && a.edge_dirty) {  // subdomain edges (domain decomposition)
        unsigned e = 0;
        if ((f & 1u) && ty == 0) e |= 1u;
        if (((f & 2u) || (f & 32u)) && ty + 1 == a.nty) e |= 2u;
        if ((f & 4u) && tx == 0) e |= 4u;
        if (((f & 8u) || (f & 64u)) && tx + 1 == a.ntx) e |= 8u;
        if (e) atomicOr(a.edge_dirty, e);
    }
}

// The issue half of a persistent in-place pass's activations (EIK_ACT_SPLIT): thread q in 1..4
// issues its side's state-word atomicOr and returns the neighbour (-1: none) with `old` to be
// passed to qpush_complete later; thread 0 flags changed subdomain edges as above.
__device__ __forceinline__ int activate_neighbours_issue(const Fim2dArgs& a, int tile, unsigned f, unsigned& old,
                                                         const unsigned* key, float& kq, unsigned& kold,
                                                         int tid = threadIdx.x) {
    old = 0u;
    if (tid >= 5) return -1;
    kq = __uint_as_float(key[tid]);  // priority mode: the side's smallest new edge value
    const int map = tile / a.tiles_per_map;
    const int rem = tile - map * a.tiles_per_map;
    const int ty = rem / a.ntx, tx = rem - (rem / a.ntx) * a.ntx;
    const int base = map * a.tiles_per_map;
    int nb = -1;
    unsigned trig = 0u;
    if (tid == 1 && (f & 1u) && ty > 0) { nb = base + rem - a.ntx; trig = kFromS; }
    if (tid == 2 && (f & 2u) && ty + 1 < a.nty) { nb = base + rem + a.ntx; trig = kFromN; }
    if (tid == 3 && (f & 4u) && tx > 0) { nb = base + rem - 1; trig = kFromE; }
    if (tid == 4 && (f & 8u) && tx + 1 < a.ntx) { nb = base + rem + 1; trig = kFromW; }
    if (nb >= 0) old = a.bctl ? qpush_issue_key(a, nb, trig, kq, kold) : qpush_issue(a, nb, trig);
    if (tid == 0 && a.edge_dirty) {
        unsigned e = 0;
        if ((f & 1u) && ty == 0) e |= 1u;
        if (((f & 2u) || (f & 32u)) && ty + 1 == a.nty) e |= 2u;
        if ((f & 4u) && tx == 0) e |= 4u;
        if (((f & 8u) || (f & 64u)) && tx + 1 == a.ntx) e |= 8u;
        if (e) atomicOr(a.edge_dirty, e);
    }
    return nb;
}

// ------------------------------------------------------------------- PERSISTENT driver
// Take a ticket and wait for its slot: the next queued tile, or -1 when the solve has ended
// (no tile pending or busy) or failed.  ONE lane polls (relaxed agent-scope loads = sc1) and takes
// the entry with an exchange (a producer may CAS a fresh tile into a filled slot, qslot_put_front).
__device__ __forceinline__ int qgrab(const Fim2dArgs& a, unsigned& trig) {
    if (__hip_atomic_load(a.qerror, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return -1;
    const unsigned long long pos = atomicAdd(a.qhead, 1ull);
    unsigned* slot = &a.qslot[pos & a.qmask];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned spin = 0;; ++spin) {
        const unsigned v = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        qcount(a, 0);
        if (v != 0u) {
            // free the slot BEFORE the tile can be re-queued (slot reuse).  Only fresh-first
            // producers write a filled slot (their CAS): then the entry is taken with an exchange.
            // Otherwise this ticket owns the slot alone (at most `grid` tickets are outstanding,
            // far fewer than the slots, so no other holder polls it and the tail is a lap away):
            // the value polled is the entry, and a relaxed store clears it -- one device-scope
            // round trip less per grab.
            int tile;
            if (a.fresh_first) {
                tile = (int)(atomicExch(slot, 0u) - 1u);
            } else {
                tile = (int)(v - 1u);
                __hip_atomic_store(slot, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            // pending -> busy before T is read: any activation from here on makes the finish
            // re-queue the tile, so no update is lost
            trig = atomicExch(&a.qstate[tile], kBusy | kVisited);  // consumed after the staging loads
            return tile;
        }
        if ((spin & 7u) == 7u) {
            // live DD: idle is not the end -- a halo merge may queue tiles until the host releases
            if (a.qhold ? __hip_atomic_load(a.qhold, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u
                        : __hip_atomic_load(a.qactive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
                return -1;
            if (__hip_atomic_load(a.qerror, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return -1;
            if (__builtin_amdgcn_s_memrealtime() - t0 > a.qtimeout) {  // never hang
                atomicOr(a.qerror, 1u);
                return -1;
            }
        }
        __builtin_amdgcn_s_sleep(8);
    }
}

// Visit budget (EIK_OPT_MAX_VISITS; negative costs on device buffers never converge): full
// visits (counter 0, flushed 64 at a time) and in-place passes (counter 1) are charged alike --
// an in-place pass sweeps the tile like a visit does.  One lane calls these.
__device__ __forceinline__ void charge_visits(const Fim2dArgs& a, unsigned long long n) {
    const unsigned long long v = atomicAdd(a.visits, n) + n;
    if (v + __hip_atomic_load(a.visits + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= a.qbudget)
        atomicOr(a.qerror, 2u);
}
__device__ __forceinline__ void charge_inplace_pass(const Fim2dArgs& a) {
    const unsigned long long p = atomicAdd(a.visits + 1, 1ull) + 1ull;
    if ((p & 63ull) == 0ull &&
        p + __hip_atomic_load(a.visits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= a.qbudget)
        atomicOr(a.qerror, 2u);
}

// Retire a visited tile (after its activations completed): re-queue it if it was activated
// while busy (it stays counted), else it stops counting as active.
__device__ __forceinline__ void qfinish(const Fim2dArgs& a, int tile) {
    const unsigned old = atomicAnd(&a.qstate[tile], ~kBusy);
    if (old & kPending) {
        if (a.bctl)  // its key: the smallest activation since its claim (0 for a self re-queue)
            prio_put_overlap(a, tile, __uint_as_float(__hip_atomic_load(&a.key[tile], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
        else
            qslot_put(a, tile);
    } else {
        atomicSub(a.qactive, 1);
    }
}

// inclusive prefix sum over the wave's 64 lanes
__device__ __forceinline__ unsigned wave_incl_sum(unsigned v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned u = __shfl_up(v, d);
        if (lane >= d) v += u;
    }
    return v;
}

// Priority mode, one wave (all lanes; the oldest FIFO waiter): move up to kDispatch entries of the
// lowest non-empty bands, in band order, to the FIFO's tail -- each band's share claimed by one CAS
// of its head (one lane per band, all at once) -- so the waiters take them lowest key first.  Only
// the oldest waiter does this, so the band heads see little contention (a first design where every
// idle workgroup CAS-ed the lowest band's head lost ~900k CASes per C2 solve and ran 20x slower),
// and the batch is the bands' throughput: C4 takes ~9 tiles per us, and one band per dispatch (a few
// entries each, ~3 round trips) held narrow bands to a fraction of that (C4 2.7 vs 10.9 Gcells/s).
// The batch a dispatch moves: Fim2dArgs::disp, set per solve (eikonal_api.cpp, EIK_OPT_PRIO_DISPATCH),
// else kDispatch; at most kMaxDispatch = 128 (two entries per lane).  128 on maps of >= kWideTiles tiles:
// C4 at one GPU 13.8-14.3 (32) -> 15.5-15.7 (48) -> 16.3-16.7 (64) -> 17.3-17.6 Gcells/s (128; 96: 17.0-17.3,
// round 6, profiles/r06s7/r06s7_disp_ab.log); 16 below: C2 2.22-2.27 (32) -> 2.16-2.19 ms (8:
// 2.20-2.22, 48: 2.31) -- a larger batch leaves a FIFO backlog that no longer follows the bands'
// order, a smaller one dispatches more often.  (A batch limited to the waiting workgroups, qhead -
// qtail: C4 10.6 -- the backlog is what feeds a busy chip.  profiles/r05x_dispatch_ab.log,
// r05z2_dispatch_sweep.log.)
constexpr unsigned kDispatch = 32;
constexpr unsigned kMaxDispatch = 128;  // two entries per lane
__device__ __forceinline__ bool band_dispatch(const Fim2dArgs& a) {
    const int lane = threadIdx.x & 63;
    unsigned long long h = 0, t = 0;
    if (lane < kBands) {
        h = __hip_atomic_load(&a.bctl[16 * lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        t = __hip_atomic_load(&a.bctl[16 * lane + 8], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) qcount(a, 2);  // (EIK_QDEBUG: dispatch attempts, 2 x 64 band words read each)
    const unsigned lim = a.disp ? (a.disp < kMaxDispatch ? a.disp : kMaxDispatch) : kDispatch;
    const unsigned avail = t > h ? (unsigned)(t - h < lim ? t - h : lim) : 0u;
    if (!__ballot(avail != 0u)) return false;
    // lowest bands first.  (Reserving a quarter of the batch for the highest band -- the front's
    // first visits -- was measured and removed: C4 at one GPU 14 -> 2.6-6 Gcells/s, C2 no gain,
    // profiles/r05h_prio_planar_ab.log.)
    const unsigned before = wave_incl_sum(avail) - avail;  // entries of the lower bands
    const unsigned take = before >= lim ? 0u : (avail < lim - before ? avail : lim - before);
    const unsigned got = take && atomicCAS(&a.bctl[16 * lane], h, h + take) == h ? take : 0u;
    const unsigned end = wave_incl_sum(got), start = end - got;
    const unsigned total = __shfl(end, 63);
    if (total == 0u) return false;  // another dispatcher moved first: look again at the next poll
    if (lane == 0) qcount(a, 5);
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(a.qtail, (unsigned long long)total);
    base = __shfl(base, 0);
    // entry e < total: lane e, and lane e - 64 for a batch past 64 -- band b where start_b <= e < end_b,
    // offset e - start_b
    const unsigned long long gotmask = __ballot(got != 0u);
    auto move = [&](unsigned e) {
        int b = -1;
        unsigned long long src = 0;
        unsigned long long mask = gotmask;
        while (mask) {
            const int j = __builtin_ctzll(mask);
            mask &= mask - 1;
            const unsigned sj = __shfl(start, j), ej = __shfl(end, j);
            const unsigned long long hj = __shfl(h, j);
            if (e >= sj && e < ej) {
                b = j;
                src = hj + (e - sj);
            }
        }
        if (b >= 0) {
            // the entry's producer may still be storing it (it took the tail first)
            unsigned* slot = &a.bslot[(size_t)b * (a.bmask + 1ull) + (src & a.bmask)];
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            unsigned v;
            while ((v = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0u) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > a.qtimeout) {
                    atomicOr(a.qerror, 1u);
                    v = 1u;  // (the error flag ends the solve; the FIFO slot gets a harmless entry)
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            __hip_atomic_store(slot, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // tagged with its band: the taker clears the tile's membership bit (qgrab_prio)
            __hip_atomic_store(&a.qslot[(base + e) & a.qmask], v | ((unsigned)b + 1u) << kBandTagShift, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    move((unsigned)lane);
    if (total > 64u) move((unsigned)lane + 64u);  // (uniform)
    return true;
}

// Priority mode: qgrab for one whole wave.  Every workgroup takes a FIFO ticket; pushes go to the
// FIFO while tickets wait, else to the bands, and the oldest waiter moves band entries to the FIFO
// in band order.  Entries are claimed by a CAS (stale ones dropped: take another ticket).
#ifndef EIK_PRIO_SLEEP
#define EIK_PRIO_SLEEP 4  // s_sleep between a waiter's polls (x 64 cycles)
#endif
__device__ __forceinline__ int qgrab_prio(const Fim2dArgs& a, unsigned& trig) {
    const int lane = threadIdx.x & 63;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (__hip_atomic_load(a.qerror, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return -1;
        unsigned long long pos = 0;
        if (lane == 0) pos = atomicAdd(a.qhead, 1ull);
        pos = __shfl(pos, 0);
        unsigned* slot = &a.qslot[pos & a.qmask];
        for (unsigned spin = 0;; ++spin) {
            unsigned v = 0;
            int oldest = 0;
            if (lane == 0) {
                v = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                qcount(a, 0);  // (EIK_QDEBUG: the polls' sc1 loads -- slot, then tail)
                if (!v) {
                    oldest = __hip_atomic_load(a.qtail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == pos;
                    qcount(a, 1);
                }
            }
            v = __shfl(v, 0);
            if (v != 0u) {
                int got = -1;
                unsigned tg = 0u;
                if (lane == 0) {
                    __hip_atomic_store(slot, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const int tl = (int)((v & kSlotTileMask) - 1u);
                    const unsigned tag = v >> kBandTagShift;
                    // an entry from band tag - 1: its membership bit is cleared before the claim
                    // decides (a put that still saw the bit made the tile pending first, so this
                    // claim serves it; a put after the clear makes a new entry).  Issued beside the
                    // claim's state load (prio_claim re-loads the state when that load came first).
                    if (tag) atomicAnd(&a.bmem[tl], ~(1ull << (tag - 1u)));
                    got = prio_claim(a, tl, tg, tag != 0u) ? tl : -1;
                    qcount(a, got >= 0 ? 3 : 4);
                }
                got = __shfl(got, 0);
                trig = __shfl(tg, 0);
                if (got >= 0) return got;
                break;  // a stale entry: this ticket is spent, take another
            }
            // the next slot filled is this one: feed the FIFO from the bands, then poll again at once
            // (an empty dispatch falls through to the end / error checks and the sleep)
            if (__shfl(oldest, 0) && band_dispatch(a)) continue;
            if ((spin & 7u) == 7u) {
                int stop = 0;
                if (lane == 0) {
                    // (live DD: idle is not the end -- a halo merge may queue tiles until the release)
                    stop = (a.qhold ? __hip_atomic_load(a.qhold, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u
                                    : __hip_atomic_load(a.qactive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) ||
                           __hip_atomic_load(a.qerror, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
                    if (!stop && __builtin_amdgcn_s_memrealtime() - t0 > a.qtimeout) {
                        atomicOr(a.qerror, 1u);
                        stop = 1;
                    }
                }
                if (__shfl(stop, 0)) return -1;
            }
            __builtin_amdgcn_s_sleep(EIK_PRIO_SLEEP);
        }
    }
}

// ------------------------------------------------------------------ live DD halo agent
// The mailbox protocol of a live launch's halo agent (workgroup 0 -- the first one dispatched, so it
// runs even when other work on the device keeps some of the launch's workgroups from being resident;
// those start late and find the solve over).  The host posts one command at a time in pinned memory
// (LiveBox, eik_kernels.hpp): PACK (snapshot the tiles pending or busy, then `pack(par, skip_busy)`
// stores this block's edges into the neighbours' receive strips of parity par, system-scope stores
// and a system release fence), MERGE (system acquire, then `merge(par, count)` min-merges the
// received strips into the ghosts, queues the edge tiles whose ghost dropped and adds the dropped
// cells to *count) and RELEASE (end the launch).  Every wait is bounded by qtimeout.  The solver
// supplies pack / merge (fim2d.hip: one value per edge cell; fim2dl.hip: nl values).
template <class Pack, class Merge>
__device__ __forceinline__ void live_agent_loop(const Fim2dArgs& a, unsigned* sh, Pack&& pack, Merge&& merge) {
    LiveBox* box = a.live;
    const int tid = threadIdx.x;
    unsigned last = 0;
    for (;;) {
        if (tid == 0) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            unsigned s;
            for (;;) {
                s = __hip_atomic_load(&box->seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
                if (s != last) break;
                if (__hip_atomic_load(a.qerror, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u ||
                    __builtin_amdgcn_s_memrealtime() - t0 > a.qtimeout) {
                    atomicOr(a.qerror, 1u);
                    s = ~0u;
                    break;
                }
                __builtin_amdgcn_s_sleep(4);
            }
            sh[0] = s;
            sh[1] = s == ~0u ? 0u : __hip_atomic_load(&box->cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            sh[2] = (unsigned)__hip_atomic_load(a.qactive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sh[3] = 0u;
        }
        __syncthreads();
        const unsigned s = sh[0], op = sh[1] & 0xffu, par = (sh[1] >> 8) & 1u;
        if (s == ~0u) {  // timed out: make the solvers leave too
            if (tid == 0) __hip_atomic_store(a.qhold, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        last = s;
        if (op == kLivePack) {  // the snapshot (sh[2]) was taken before any T load
            pack(par, a.live_pack && sh[2] != 0u);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: peer stores complete
        } else if (op == kLiveMerge) {
            // the strips were stored by peer GPUs: drop any stale cached copy before reading
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            merge(par, &sh[3]);
        }
        __syncthreads();
        if (tid == 0) {
            if (op == kLivePack) __hip_atomic_store(&box->active, sh[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (op == kLiveMerge) __hip_atomic_store(&box->changed, sh[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (op == kLiveRelease) __hip_atomic_store(a.qhold, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&box->error, __hip_atomic_load(a.qerror, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&box->done, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (op == kLiveRelease) return;
        __syncthreads();  // sh[] is rewritten by the next command
    }
}

}  // namespace eik
