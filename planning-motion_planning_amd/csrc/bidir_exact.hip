// bidir_exact.hip -- biComputeTmap's nodeJoin and partial fields exactly as the reference's
// sequential narrow band forms them (EIK_OPT_EXACT_BAND = 1), by replaying its update events in pop
// order on the device.
//
// The reference (FastMarching.py:44-89, :141-162) pops the band's minimum, closes it, and updates
// each open 4-neighbour y of it (children y-1, y+1, x-1, x+1, :46-54) from the values y's
// neighbours hold AT THAT MOMENT -- popped neighbours their final values, band neighbours their
// tentative ones, the rest +inf (:57-63).  An update is kept only when smaller (:64-79), and equal T
// pop in LIFO insertion order (bisect_left, :65 / :76).  So every value it returns is an EVENT
//     g(y, d) = getEikonal over y's neighbours as of time t = rank(c), c = y's neighbour in direction d,
// where a cell z holds, as of time t,
//     V(z, t) = 0 for the source;  +inf for a +inf-cost cell;  else the min over z's events with
//               time < min(t, rank(z))  (+inf without any),
// a popped cell's value is V(y, rank y) and a band cell's at the meeting k is V(y, k + 1).  An event
// reads only events of strictly earlier times (z's events precede t; two neighbours of y are never
// neighbours of each other), so the events are a DAG in pop order with one solution; and the pop
// order follows the popped values with the list's LIFO rule: equal T pop latest insertion first, and
// an insertion made by a pop of the same T pops next (a stack, exact_ties_kernel).  Both are solved by
// fixed-point iteration from the converged fields, which solve_fronts computes in the reference's
// own getEikonal arithmetic for this mode (fim2d.hip sweep_quadrant REF), so that the popped cells'
// final values mostly start exact:
//  1. init:    every event from the field's values (an estimate: the fixed point does not depend on it);
//  2. relax:   chunks of kChunk pops in rank order, every event of a chunk swept in place across the
//              GPU until a sweep changes no event's bits (earlier chunks are final), each event's
//              inputs resolved once per chunk;
//  3. re-rank: key every popped cell (value, seq) and sort the ranks from the first one relaxed, then
//              re-form the runs of exactly equal T as stacks (seq reads earlier runs' ranks: one tie
//              level per launch, on the device); if a rank moved against the relaxation's order,
//              relax again from it (the relaxed events are the start) and re-rank;
//  4. join:    bidir.hip's min over max(rankG, rankS) on the exact ranks;
//  5. fields:  popped cells V(y, rank y), band cells V(y, k + 1), every other cell +inf.
// getEikonal is the reference's own arithmetic (eik_ref, eik_common.hpp: its operation order, IEEE
// fp64 without contraction, correctly rounded sqrt), so the values are the reference's bits.  The
// fields and the join are checked bit for bit against the reference's biComputeTmap fixtures (ties
// included) and the oracle's sequential band on seeded rasters (tests/test_gpu_bidir_exact.py).
// Cost: profiles/r06m_exact_ab.log (the bench's planner step 1, 4096^2, 2.1 M pops per front).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "eik_common.hpp"
#include "eik_kernels.hpp"

namespace eik {

namespace {

constexpr unsigned kNoRank = 0xFFFFFFFFu;
constexpr unsigned kMaxPasses = 1u << 16;
constexpr int kTieBatch = 16;
constexpr unsigned kMaxTieBatches = 1u << 16;

struct Front {
    const double* cost;  // the raster / volume
    double* T;           // the converged field on entry (init values); the partial field on exit (2D)
    unsigned* rank;      // per cell: pop rank, kNoRank = not among the m ranked cells
    unsigned* ord;       // m: the cell of each rank
    double* ev;          // K per cell: events [cell][d], d = the direction of the popping neighbour
    int64_t src;         // the front's source (closed before the first pop)
    unsigned m;
    unsigned from;       // this pass: first rank relaxed / re-keyed
};

struct Ctl {
    unsigned chunk[2], done[2], changed[2], arrive[2], fresh[2];  // the relaxation's chunk walk
    unsigned act[2];        // fronts still re-ranking
    unsigned sweeps[2];     // chunk sweeps of the relaxation (per pass)
    unsigned first_bad[2];  // this pass: first rank that moved against the relaxation's order
    unsigned longrun;       // a run of equal T too long for exact_ties_kernel (1), or not closed (2)
    unsigned msel;          // FM3D: cells selected for ranking
    double thr;             // FM3D: the selection's bound on T
    unsigned long long nmin[2];  // biComputeTmap: bits of the smallest field value of an unranked finite cell
    unsigned edge;               // biComputeTmap: the meeting's value is not clear of that bound
};

// The grids.  Children (= neighbours) in the reference's updateNode order, opposite directions
// paired (d ^ 1); `solve` is its local update over the K neighbours' values as of a pop.
// 2D, FastMarching.py:46-63: y - 1, y + 1, x - 1, x + 1; getEikonal(min(T[x+1], T[x-1]),
// min(T[y+1], T[y-1]), cost).  Cells [y][x].
struct Geo2 {
    int64_t H, W;
    static constexpr int K = 4;
    struct Co {
        int64_t x, y;
    };
    __device__ Co co(int64_t i) const {
        const int64_t y = (unsigned)i / (unsigned)W;
        return {i - y * W, y};
    }
    __device__ int64_t nb(int64_t i, Co c, int d) const {
        switch (d) {
            case 0: return c.y > 0 ? i - W : -1;
            case 1: return c.y + 1 < H ? i + W : -1;
            case 2: return c.x > 0 ? i - 1 : -1;
            default: return c.x + 1 < W ? i + 1 : -1;
        }
    }
    __device__ Co step(Co c, int d) const {
        return d < 2 ? Co{c.x, c.y + (d == 0 ? -1 : 1)} : Co{c.x + (d == 2 ? -1 : 1), c.y};
    }
    __device__ double solve(const double* v, double cost) const {
        return eik_ref(__builtin_fmin(v[3], v[2]), __builtin_fmin(v[1], v[0]), cost);
    }
};
// 3D, FastMarching3D.py:21-75: z - 1, z + 1, x - 1, x + 1, y + 1, y - 1 (node = [x, y, z]); Tx = Tx1 <
// Tx2 ? Tx1 : Tx2 with Tx1 = T[x-1] (likewise y, z), then the n-D update solve3_ref(Tx, Ty, Tz, C).
// Cells [y][x][z].
struct Geo3 {
    int64_t H, W, L;
    static constexpr int K = 6;
    struct Co {
        int64_t x, y, z;
    };
    __device__ Co co(int64_t i) const {
        const int64_t xy = (unsigned)i / (unsigned)L, y = (unsigned)xy / (unsigned)W;
        return {xy - y * W, y, i - xy * L};
    }
    __device__ int64_t nb(int64_t i, Co c, int d) const {
        switch (d) {
            case 0: return c.z > 0 ? i - 1 : -1;
            case 1: return c.z + 1 < L ? i + 1 : -1;
            case 2: return c.x > 0 ? i - L : -1;
            case 3: return c.x + 1 < W ? i + L : -1;
            case 4: return c.y + 1 < H ? i + W * L : -1;
            default: return c.y > 0 ? i - W * L : -1;
        }
    }
    __device__ Co step(Co c, int d) const {
        switch (d) {
            case 0: return {c.x, c.y, c.z - 1};
            case 1: return {c.x, c.y, c.z + 1};
            case 2: return {c.x - 1, c.y, c.z};
            case 3: return {c.x + 1, c.y, c.z};
            case 4: return {c.x, c.y + 1, c.z};
            default: return {c.x, c.y - 1, c.z};
        }
    }
    __device__ double solve(const double* v, double cost) const {
        const double tx = v[2] < v[3] ? v[2] : v[3], ty = v[5] < v[4] ? v[5] : v[4], tz = v[0] < v[1] ? v[0] : v[1];
        return solve3_ref(tx, ty, tz, cost);
    }
};

// the min over z's events whose time (the popping neighbour's rank) is below lim
template <class G>
__device__ __forceinline__ double events_below(const G& g, const Front& F, int64_t z, typename G::Co c, unsigned lim) {
    double v = Real<double>::inf();
    for (int d = 0; d < G::K; ++d) {
        const int64_t j = g.nb(z, c, d);
        if (j >= 0 && F.rank[j] < lim) v = __builtin_fmin(v, F.ev[G::K * z + d]);
    }
    return v;
}

// is y updated by the pop of rank r?  open: not popped before, not +inf cost, not the source
__device__ __forceinline__ bool child_open(const Front& F, int64_t y, unsigned r) {
    return y >= 0 && F.rank[y] > r && y != F.src && F.cost[y] < Real<double>::inf();
}

__global__ void exact_order_kernel(Front F0, Front F1, int64_t n) {
    const Front& F = blockIdx.y ? F1 : F0;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned r = F.rank[i];
    if (r < F.m) F.ord[r] = (unsigned)i;
}

// 1. every child slot of every ranked pop from the field's values -- valid under the current ranks
//    or not, so that a slot a later pass's ranks make valid never holds garbage (later passes keep
//    the relaxed values as their start)
template <class G>
__global__ __launch_bounds__(256) void exact_init_kernel(Front F0, Front F1, G g) {
    const Front& F = blockIdx.y ? F1 : F0;
    const double inf = Real<double>::inf();
    const int64_t e1 = (int64_t)G::K * F.m;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < e1; e += (int64_t)gridDim.x * blockDim.x) {
        const unsigned r = (unsigned)(e / G::K);
        const int k = (int)(e - (int64_t)r * G::K);
        const int64_t c = F.ord[r];
        const typename G::Co cc = g.co(c);
        const int64_t y = g.nb(c, cc, k);
        if (y < 0 || y == F.src || !(F.cost[y] < inf)) continue;
        const typename G::Co yc = g.step(cc, k);
        double v[G::K];
        for (int d = 0; d < G::K; ++d) {
            const int64_t j = g.nb(y, yc, d);
            v[d] = j < 0 ? inf : F.T[j];
        }
        F.ev[G::K * y + (k ^ 1)] = g.solve(v, F.cost[y]);
    }
}

// 2. relaxation, chunk by chunk in rank order: each launch sweeps every event of the current chunk of
//    kChunk pops of each front in place (all of the GPU), and the front's last workgroup advances the
//    chunk when the sweep changed no event's bits -- the chunk's events are then the unique solution
//    given the earlier chunks (an event reads only events of earlier ranks).  A chunk's first sweep
//    resolves every event's inputs (EvDesc: slot, cost, per neighbour its events row, which of them
//    precede the pop, source / never updated) and stores them; later sweeps of the chunk reload them,
//    so a sweep is one level of descriptor loads and one of event loads.
//    History (profiles/r06m_exact_ab.log, the bench's planner query: 4096^2, 2.1 M pops per front):
//    one in-order workgroup per front (Gauss-Seidel groups of 256 pops) 297 ms -- it settles a group
//    per latency period where a GPU-wide sweep settles a chunk; GPU-wide Jacobi sweeps over ALL events
//    1.95 s (1513 launches: the band's tentative values chain along the front).
constexpr unsigned kChunk = 16384;  // pops per chunk (4 / 6 events each)
constexpr int kBatch = 32;          // sweeps queued between two reads of the done flags
constexpr unsigned long long kMaxSweeps = 1ull << 24;
template <class G>
struct EvDesc {
    double* slot;  // nullptr: the child is not open (no event)
    double cost;
    const double* zev[G::K];
    unsigned long long mask;  // K bits per neighbour: its events that precede the pop
    unsigned kinds;           // 2 bits per neighbour: 0 events, 1 source, 2 +inf (never updated, outside)
};
template <class G>
__device__ __forceinline__ void make_desc(const G& g, const Front& F, unsigned e, EvDesc<G>& D) {
    const unsigned r = e / G::K;
    const int k = (int)(e - r * G::K);
    const int64_t c = F.ord[r];
    const typename G::Co cc = g.co(c);
    const int64_t y = g.nb(c, cc, k);
    D.slot = nullptr;
    if (!child_open(F, y, r)) return;
    const typename G::Co yc = g.step(cc, k);
    D.slot = F.ev + G::K * y + (k ^ 1);
    D.cost = F.cost[y];
    D.mask = 0ull;
    D.kinds = 0u;
#pragma unroll
    for (int d = 0; d < G::K; ++d) {
        const int64_t z = g.nb(y, yc, d);
        D.zev[d] = nullptr;
        if (z < 0 || (z != F.src && !(F.cost[z] < Real<double>::inf()))) {
            D.kinds |= 2u << (2 * d);
            continue;
        }
        if (z == F.src) {
            D.kinds |= 1u << (2 * d);
            continue;
        }
        const unsigned rz = F.rank[z], lim = rz < r ? rz : r;  // V(z, t): events of time < min(t, rank z)
        const typename G::Co zc = g.step(yc, d);
        D.zev[d] = F.ev + G::K * z;
        for (int q = 0; q < G::K; ++q) {
            const int64_t w = g.nb(z, zc, q);
            if (w >= 0 && F.rank[w] < lim) D.mask |= 1ull << (G::K * d + q);
        }
    }
}
template <class G>
__device__ __forceinline__ double desc_value(const G& g, const EvDesc<G>& D) {
    double v[G::K];
#pragma unroll
    for (int d = 0; d < G::K; ++d) {
        const unsigned kd = (D.kinds >> (2 * d)) & 3u;
        double m = kd == 1u ? 0.0 : Real<double>::inf();
        if (kd == 0u) {
#pragma unroll
            for (int q = 0; q < G::K; ++q)
                if ((D.mask >> (G::K * d + q)) & 1ull) m = __builtin_fmin(m, D.zev[d][q]);
        }
        v[d] = m;
    }
    return g.solve(v, D.cost);
}
template <class G>
__global__ __launch_bounds__(256) void exact_sweep_kernel(Front F0, Front F1, G g, Ctl* ctl, EvDesc<G>* desc0,
                                                          EvDesc<G>* desc1) {
    const int f = blockIdx.y;
    const Front& F = f ? F1 : F0;
    EvDesc<G>* desc = f ? desc1 : desc0;
    __shared__ unsigned s_chunk, s_done, s_fresh;
    if (threadIdx.x == 0) {
        s_done = ctl->done[f];
        s_chunk = ctl->chunk[f];
        s_fresh = ctl->fresh[f];
    }
    __syncthreads();
    if (s_done) return;
    const unsigned r0 = s_chunk * kChunk, r1 = min(r0 + kChunk, F.m);
    bool ch = false;
    for (unsigned e = G::K * r0 + blockIdx.x * blockDim.x + threadIdx.x; e < G::K * r1; e += gridDim.x * blockDim.x) {
        EvDesc<G> D;
        if (s_fresh) {
            make_desc(g, F, e, D);
            desc[e - G::K * r0] = D;
        } else {
            D = desc[e - G::K * r0];
        }
        if (!D.slot) continue;
        const double v = desc_value(g, D);
        if (__double_as_longlong(*D.slot) != __double_as_longlong(v)) {
            *D.slot = v;
            ch = true;
        }
    }
    const int any = __syncthreads_or(ch);
    if (threadIdx.x == 0) {
        if (any) atomicOr(&ctl->changed[f], 1u);
        __threadfence();
        if (atomicAdd(&ctl->arrive[f], 1u) == gridDim.x - 1) {  // the front's last workgroup
            __threadfence();
            const unsigned chg = atomicOr(&ctl->changed[f], 0u);
            ctl->sweeps[f] += 1u;
            if (!chg) {
                ctl->chunk[f] = s_chunk + 1u;
                ctl->fresh[f] = 1u;
                if ((unsigned long long)(s_chunk + 1u) * kChunk >= F.m) ctl->done[f] = 1u;
            } else {
                ctl->fresh[f] = 0u;
            }
            ctl->changed[f] = 0u;
            ctl->arrive[f] = 0u;
        }
    }
}

// the LIFO key of the cell y popped at rank r: its value (the min over its events before r) and seq
// = K x the time of the first event reaching that value (the last strict decrease) + y's child
// index in that update -- the later the insertion, the earlier among equal T (bisect_left)
template <class G>
__device__ __forceinline__ double pop_key(const G& g, const Front& F, int64_t y, unsigned r, unsigned* seq) {
    if (y == F.src) {
        *seq = ~0u;  // pops first
        return 0.0;
    }
    const typename G::Co c = g.co(y);
    double best = Real<double>::inf();
    unsigned bt = kNoRank, s = 0u;
    for (int d = 0; d < G::K; ++d) {
        const int64_t nb = g.nb(y, c, d);
        if (nb < 0) continue;
        const unsigned t = F.rank[nb];
        if (t >= r) continue;
        const double v = F.ev[G::K * y + d];
        if (v < best || (v == best && t < bt)) {
            best = v;
            bt = t;
            s = (unsigned)G::K * t + (unsigned)(d ^ 1);
        }
    }
    *seq = s;
    return best;
}

// 3a. the keys of every pop of rank >= from.  The value key is max(value, its setter's value): a pop
//     can give a neighbour a value below its own by rounding (an inversion: the reference's c3 cube
//     drops 2.8e-14 at its pop 1484), and the list then pops that neighbour NEXT -- so it sorts into
//     its setter's run, whose stack order (exact_ties_kernel) puts it right after the setter
template <class G>
__global__ void exact_keys_kernel(Front F, G g, unsigned long long* kT, unsigned* kS, unsigned* val) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t cnt = (int64_t)F.m - F.from;
    if (j >= cnt) return;
    const unsigned r = F.from + (unsigned)j;
    unsigned seq;
    double t = pop_key(g, F, F.ord[r], r, &seq);
    if (seq != ~0u) {
        const unsigned bt = seq / G::K;  // the setter's rank
        unsigned sq;
        const double ts = pop_key(g, F, F.ord[bt], bt, &sq);
        t = ts > t ? ts : t;
    }
    kT[j] = (unsigned long long)__double_as_longlong(t);  // T >= 0 (or +inf): orders as unsigned
    kS[j] = ~seq;                                         // ascending ~seq = most recent insertion first
    val[j] = r;
}

__global__ void exact_gather_kernel(const unsigned long long* kT, const unsigned* perm, unsigned from, int64_t cnt,
                                    unsigned long long* out) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < cnt) out[j] = kT[perm[j] - from];
}

// 3b. the new order by the sorted positions (ord2: staging)
__global__ void exact_moved_kernel(Front F, const unsigned* sorted, int64_t cnt, unsigned* ord2) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= cnt) return;
    ord2[j] = F.ord[sorted[j]];
}

// 3c. runs of equal keys pop as the reference's list does: entries of equal T pop most recent
//     insertion first (bisect_left), and a pop may insert a child at exactly its own T (getEikonal's
//     two-sided form at |Thor - Tver| = cost gives Thor) or, by rounding, below it -- which then
//     pops NEXT, before older entries.  So a run is a stack: its roots (members whose value was set
//     by a pop before the run) pushed in insertion order (seq), then each pop pushes, in updateNode's
//     child order, the members it set (their value's first event is its update).  A member's value
//     and setter are read over the events of every pop up to the run's end (an equal or larger value
//     from a later pop is no strict decrease).  seq reads the ranks of earlier pops, themselves
//     possibly in a run, so a tie level settles once the levels below it have: each launch re-forms
//     every run (its first thread, runs are short) from the current ranks until a launch moves
//     nothing.  The events stay as the relaxation left them; the pass's final check (every rank
//     against the relaxation's order) catches any exception.  Launch s returns at once when launch
//     s - 1 moved nothing.
constexpr int64_t kMaxRun = 4096;
template <class G>
__global__ void exact_ties_kernel(Front F, G g, const unsigned long long* kT, int64_t cnt, unsigned* flags, int s,
                                  unsigned* longrun, unsigned* out_buf, unsigned* stack_buf, unsigned* pushed_buf) {
    if (s > 0 && flags[s - 1] == 0u) return;
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j + 1 >= cnt || kT[j + 1] != kT[j] || (j > 0 && kT[j - 1] == kT[j])) return;  // run starts only
    int64_t e = j + 2;
    while (e < cnt && kT[e] == kT[j] && e - j <= kMaxRun) ++e;
    if (e - j > kMaxRun) {
        atomicOr(longrun, 1u);  // (the replay reports it: the run's order would be unchecked)
        return;
    }
    const int L = (int)(e - j);
    const unsigned r0 = F.from + (unsigned)j, r1 = r0 + (unsigned)L;
    unsigned* out = out_buf + j;
    unsigned* stk = stack_buf + j;
    unsigned* pushed = pushed_buf + j;  // per member (the run's own slice of a free buffer, no scratch)
    for (int a = 0; a < L; ++a) pushed[a] = 0u;
    // roots in ascending seq: the top of the stack is the latest insertion
    int sp = 0;
    unsigned* sseq = out;  // (the roots' seq, beside the stack, until the output is written)
    for (int a = 0; a < L; ++a) {
        const int64_t y = F.ord[r0 + a];
        unsigned sq;
        (void)pop_key(g, F, y, r1, &sq);
        if (sq != ~0u && sq / G::K >= r0) continue;  // set by a run member: pushed by its pop
        int b = sp++;
        while (b > 0 && sseq[b - 1] > sq) {
            stk[b] = stk[b - 1];
            sseq[b] = sseq[b - 1];
            --b;
        }
        stk[b] = (unsigned)y;
        sseq[b] = sq;
        pushed[a] = 1u;
    }
    // pop: the output overwrites sseq from the front, which the stack no longer needs (sseq[i] is
    // only read while sorting the roots in)
    int no = 0;
    while (sp > 0) {
        const int64_t p = stk[--sp];
        const typename G::Co pc = g.co(p);
        const unsigned rp = F.rank[p];
        out[no++] = (unsigned)p;
        for (int k = 0; k < G::K; ++k) {
            const int64_t y = g.nb(p, pc, k);
            if (y < 0) continue;
            const unsigned ry = F.rank[y];
            if (ry < r0 || ry >= r1) continue;  // not in this run
            const int a = (int)(ry - r0);
            if (pushed[a]) continue;
            unsigned sq;
            (void)pop_key(g, F, y, r1, &sq);
            if (sq != (unsigned)G::K * rp + (unsigned)k) continue;  // p's update did not set y's value
            pushed[a] = 1u;
            stk[sp++] = (unsigned)y;
        }
    }
    if (no != L) {  // a member no pop of the run reached (never on valid input): reported
        atomicOr(longrun, 2u);
        return;
    }
    bool moved = false;
    for (int a = 0; a < L; ++a) {
        const unsigned y = out[a];
        if (F.ord[r0 + a] != y) {
            moved = true;
            F.ord[r0 + a] = y;
            F.rank[y] = r0 + (unsigned)a;
        }
    }
    if (moved) flags[s] = 1u;
}

// 3d. the first rank whose cell differs from the order the relaxation used
__global__ void exact_cmp_kernel(Front F, const unsigned* ordp, int64_t cnt, unsigned* first_bad) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < cnt && F.ord[F.from + j] != ordp[j]) atomicMin(first_bad, F.from + (unsigned)j);
}

__global__ void exact_apply_kernel(Front F, const unsigned* ord2, int64_t cnt) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= cnt) return;
    const unsigned r = F.from + (unsigned)j, i = ord2[j];
    F.ord[r] = i;
    F.rank[i] = r;
}

// 5. the returned field after the pop of rank k: popped cells (rank <= k) their value, band cells
//    (an open cell with a popped neighbour) their value as of that pop, every other cell +inf.
//    biComputeTmap: k = the meeting iteration (*best >> 30), each front in place.  FM3D's early
//    exit: k = the rank of `start` (kNoRank: never popped -- the full field), into Te.
template <class G>
__device__ __forceinline__ double field_value(const G& g, const Front& F, int64_t i, unsigned k) {
    if (i == F.src) return 0.0;
    if (!(F.cost[i] < Real<double>::inf())) return Real<double>::inf();
    const unsigned r = F.rank[i];
    const unsigned lim = r <= k ? r : (k == kNoRank ? kNoRank : k + 1u);
    return events_below(g, F, i, g.co(i), lim);  // (+inf when no neighbour popped)
}

// biComputeTmap ranks only the join's member prefix (every cell of field value up to a bucket edge);
// the replay's order is valid if no unranked cell could pop before the meeting: the meeting's exact
// value must stay below every unranked finite cell's field value by more than their ~1e-13 agreement
__global__ __launch_bounds__(256) void exact_nmin_kernel(Front F0, Front F1, int64_t n, Ctl* ctl) {
    const int f = blockIdx.y;
    const Front& F = f ? F1 : F0;
    unsigned long long m = ~0ull;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double t = F.T[i];
        if (F.rank[i] == kNoRank && t < Real<double>::inf()) {
            const unsigned long long v = (unsigned long long)__double_as_longlong(t);
            m = v < m ? v : m;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(m, off, 64);
        m = o < m ? o : m;
    }
    if ((threadIdx.x & 63) == 0 && m != ~0ull) atomicMin(&ctl->nmin[f], m);
}
__global__ void exact_edge_kernel(Front F0, Front F1, Geo2 g, const unsigned long long* best, Ctl* ctl) {
    const unsigned long long b = *best;
    if (threadIdx.x >= 2 || b == ~0ull) return;
    const Front& F = threadIdx.x ? F1 : F0;
    const unsigned k = (unsigned)(b >> 30);
    if (k >= F.m) {
        ctl->edge = 1u;
        return;
    }
    const unsigned long long nm = ctl->nmin[threadIdx.x];
    if (nm == ~0ull) return;  // every finite cell is ranked
    unsigned sq;
    const double t = pop_key(g, F, F.ord[k], k, &sq);
    if (!(t < __longlong_as_double((long long)nm) * (1.0 - 0x1p-30))) ctl->edge = 1u;
}

__global__ void exact_fields_bidir_kernel(Front F0, Front F1, Geo2 g, const unsigned long long* best) {
    const Front& F = blockIdx.y ? F1 : F0;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long b = *best;
    if (i >= g.H * g.W || b == ~0ull) return;  // never met: the caller reports it
    F.T[i] = field_value(g, F, i, (unsigned)(b >> 30));
}

__global__ void exact_fields_early_kernel(Front F, Geo3 g, int64_t start, double* __restrict__ Te) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= g.H * g.W * g.L) return;
    Te[i] = field_value(g, F, i, F.rank[start]);
}

// FM3D: the cells ranked -- T <= T[start] x (1 + 2^-30), every cell the replay can pop up to start
// (the converged field is within a few ulps of the reference's values); all finite cells when start
// is unreachable (the reference then empties its band)
__global__ void exact_thr_kernel(const double* T, int64_t start, Ctl* ctl) {
    const double ts = T[start];
    ctl->thr = ts < Real<double>::inf() ? ts * (1.0 + 0x1p-30) : Real<double>::inf();
}
struct Fm3dMember {
    const double* T;
    const Ctl* ctl;
    __device__ bool operator()(const unsigned& i) const {
        const double t = T[i];
        return t < Real<double>::inf() && t <= ctl->thr;
    }
};
__global__ void exact_tkeys_kernel(const double* T, const unsigned* list, int64_t m, unsigned long long* keys) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m) keys[j] = (unsigned long long)__double_as_longlong(T[list[j]]);
}
__global__ void exact_scatter_rank_kernel(const unsigned* ord, int64_t m, unsigned* rank) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m) rank[ord[j]] = (unsigned)j;
}

struct ExactLayout {
    unsigned* rank[2];
    unsigned* ord[2];
    double* ev[2];
    unsigned long long *kT, *kT2, *kT3;
    unsigned *kS, *kS2, *val, *val2, *val3, *ord2, *ordp, *flags;
    void* desc[2];  // EvDesc per event of the current chunk
    char* cub_tmp;
    size_t cub_bytes;
    Ctl* ctl;
    size_t total;
};

size_t align256(size_t b) { return (b + 255) & ~size_t(255); }

// K events per cell; per-front arrays only for fronts with members; sel: room for FM3D's selection
ExactLayout exact_layout(void* work, int64_t n, int K, int64_t m0, int64_t m1, bool sel) {
    ExactLayout L{};
    const int64_t mx = std::max<int64_t>(1, std::max(m0, m1));
    size_t sort64 = 0, sort32 = 0, sel_b = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort32, (unsigned*)nullptr, (unsigned*)nullptr, (unsigned*)nullptr,
                                             (unsigned*)nullptr, (int)mx, 0, 32, (hipStream_t)0);
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort64, (unsigned long long*)nullptr,
                                             (unsigned long long*)nullptr, (unsigned*)nullptr, (unsigned*)nullptr,
                                             (int)mx, 0, 64, (hipStream_t)0);
    if (sel)
        (void)hipcub::DeviceSelect::If(nullptr, sel_b, hipcub::CountingInputIterator<unsigned>(0u), (unsigned*)nullptr,
                                       (unsigned*)nullptr, n, Fm3dMember{nullptr, nullptr}, (hipStream_t)0);
    L.cub_bytes = align256(std::max(std::max(sort32, sort64), sel_b));
    char* p = static_cast<char*>(work);
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char* q = p ? p + off : nullptr;
        off += align256(bytes);
        return q;
    };
    const int64_t m[2] = {m0, m1};
    for (int f = 0; f < 2; ++f) {
        const bool on = m[f] > 0;
        L.ev[f] = reinterpret_cast<double*>(take(sizeof(double) * (on ? (size_t)K * n : 1)));
        L.rank[f] = reinterpret_cast<unsigned*>(take(sizeof(unsigned) * (on ? (size_t)n : 1)));
        L.ord[f] = reinterpret_cast<unsigned*>(take(sizeof(unsigned) * (size_t)std::max<int64_t>(1, m[f])));
        L.desc[f] = take(on ? (K == Geo2::K ? sizeof(EvDesc<Geo2>) : sizeof(EvDesc<Geo3>)) * (size_t)K * kChunk : 1);
    }
    L.kT = reinterpret_cast<unsigned long long*>(take(8 * (size_t)mx));
    L.kT2 = reinterpret_cast<unsigned long long*>(take(8 * (size_t)mx));
    L.kT3 = reinterpret_cast<unsigned long long*>(take(8 * (size_t)mx));
    L.kS = reinterpret_cast<unsigned*>(take(4 * (size_t)mx));
    L.kS2 = reinterpret_cast<unsigned*>(take(4 * (size_t)mx));
    L.val = reinterpret_cast<unsigned*>(take(4 * (size_t)mx));
    L.val2 = reinterpret_cast<unsigned*>(take(4 * (size_t)mx));
    L.val3 = reinterpret_cast<unsigned*>(take(4 * (size_t)mx));
    L.ord2 = reinterpret_cast<unsigned*>(take(4 * (size_t)mx));
    L.ordp = reinterpret_cast<unsigned*>(take(4 * (size_t)mx));
    L.flags = reinterpret_cast<unsigned*>(take(4 * (size_t)64));
    L.cub_tmp = take(L.cub_bytes);
    L.ctl = reinterpret_cast<Ctl*>(take(sizeof(Ctl)));
    L.total = off;
    return L;
}

__global__ void exact_ctl_kernel(Ctl* ctl, unsigned a0, unsigned a1, unsigned c0, unsigned c1) {
    ctl->act[0] = a0;
    ctl->act[1] = a1;
    ctl->chunk[0] = c0;
    ctl->chunk[1] = c1;
    ctl->done[0] = a0 ? 0u : 1u;
    ctl->done[1] = a1 ? 0u : 1u;
    ctl->fresh[0] = ctl->fresh[1] = 1u;
    ctl->changed[0] = ctl->changed[1] = 0u;
    ctl->arrive[0] = ctl->arrive[1] = 0u;
    ctl->first_bad[0] = ctl->first_bad[1] = kNoRank;
    ctl->longrun = 0u;
}

// steps 1-3 for nf fronts (F[0..nf-1]) whose rank / ord arrays hold a first order of their m cells
template <class G>
hipError_t replay(const G& g, Front F[2], int nf, const ExactLayout& L, hipStream_t st, unsigned long long info[4]) {
    hipError_t e = hipSuccess;  // (the caller cleared Ctl)
    {
        const int64_t mx = std::max(F[0].m, nf > 1 ? F[1].m : 0u);
        const unsigned gi = (unsigned)std::max<int64_t>(1, std::min<int64_t>(4096, ((int64_t)G::K * mx + 255) / 256));
        hipLaunchKernelGGL(exact_init_kernel<G>, dim3(gi, nf), dim3(256), 0, st, F[0], F[1], g);
    }
    bool active[2] = {F[0].m > 0, nf > 1 && F[1].m > 0};
    static const bool debug = getenv("EIK_EXACT_DEBUG") != nullptr;  // per-pass trace on stderr (diagnostics)
    unsigned passes = 0;
    for (;;) {
        if (++passes > kMaxPasses) {
            if (debug) fprintf(stderr, "[exact] no fixed point after %u passes\n", kMaxPasses);
            return hipErrorNotReady;
        }
        hipLaunchKernelGGL(exact_ctl_kernel, dim3(1), dim3(1), 0, st, L.ctl, active[0] ? 1u : 0u, active[1] ? 1u : 0u,
                           F[0].from / kChunk, F[1].from / kChunk);
        unsigned long long sweeps = 0;
        for (;;) {  // relax until every active front's last chunk settled
            for (int q = 0; q < kBatch; ++q)
                hipLaunchKernelGGL(exact_sweep_kernel<G>, dim3(G::K * kChunk / 256, nf), dim3(256), 0, st, F[0], F[1], g,
                                   L.ctl, reinterpret_cast<EvDesc<G>*>(L.desc[0]), reinterpret_cast<EvDesc<G>*>(L.desc[1]));
            sweeps += kBatch;
            unsigned done[2] = {0, 0};
            e = hipMemcpyAsync(done, L.ctl->done, sizeof done, hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess) return e;
            if (done[0] && done[1]) break;
            if (sweeps > kMaxSweeps) {
                if (debug) fprintf(stderr, "[exact] the relaxation did not settle (pass %u)\n", passes);
                return hipErrorNotReady;
            }
        }
        // re-rank every active front from its first relaxed rank
        for (int f = 0; f < nf; ++f) {
            if (!active[f]) continue;
            const int64_t cnt = (int64_t)F[f].m - F[f].from;
            if (cnt <= 0) continue;
            const unsigned gk = (unsigned)((cnt + 255) / 256);
            hipLaunchKernelGGL(exact_keys_kernel<G>, dim3(gk), dim3(256), 0, st, F[f], g, L.kT, L.kS, L.val);
            size_t b = L.cub_bytes;
            e = hipcub::DeviceRadixSort::SortPairs(L.cub_tmp, b, L.kS, L.kS2, L.val, L.val2, (int)cnt, 0, 32, st);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL(exact_gather_kernel, dim3(gk), dim3(256), 0, st, L.kT, L.val2, F[f].from, cnt, L.kT2);
            b = L.cub_bytes;
            e = hipcub::DeviceRadixSort::SortPairs(L.cub_tmp, b, L.kT2, L.kT3, L.val2, L.val3, (int)cnt, 0, 64, st);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL(exact_moved_kernel, dim3(gk), dim3(256), 0, st, F[f], L.val3, cnt, L.ord2);
            e = hipMemcpyAsync(L.ordp, F[f].ord + F[f].from, sizeof(unsigned) * (size_t)cnt, hipMemcpyDeviceToDevice, st);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL(exact_apply_kernel, dim3(gk), dim3(256), 0, st, F[f], L.ord2, cnt);
            // the tie runs, in batches of kTieBatch launches until one moves nothing
            for (unsigned tb = 0;; ++tb) {
                if (tb >= kMaxTieBatches) return hipErrorNotReady;
                e = hipMemsetAsync(L.flags, 0, sizeof(unsigned) * kTieBatch, st);
                if (e != hipSuccess) return e;
                for (int q = 0; q < kTieBatch; ++q)
                    hipLaunchKernelGGL(exact_ties_kernel<G>, dim3(gk), dim3(256), 0, st, F[f], g, L.kT3, cnt, L.flags, q,
                                       &L.ctl->longrun, L.ord2, L.val2, L.val3);
                unsigned hf[kTieBatch];
                e = hipMemcpyAsync(hf, L.flags, sizeof hf, hipMemcpyDeviceToHost, st);
                if (e == hipSuccess) e = hipStreamSynchronize(st);
                if (e != hipSuccess) return e;
                int q = 0;
                while (q < kTieBatch && hf[q]) ++q;
                info[3] += (unsigned long long)(q < kTieBatch ? q + 1 : kTieBatch);
                if (q < kTieBatch) break;
                if (debug && (tb & (tb - 1)) == 0)
                    fprintf(stderr, "[exact] pass %u front %d: tie runs still moving after %u batches\n", passes, f, tb + 1);
            }
            // ordp: the relaxation's order (the old ord after the copy above)
            hipLaunchKernelGGL(exact_cmp_kernel, dim3(gk), dim3(256), 0, st, F[f], L.ordp, cnt, &L.ctl->first_bad[f]);
        }
        Ctl h{};
        e = hipMemcpyAsync(&h, L.ctl, sizeof h, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return e;
        if (h.longrun) return hipErrorNotSupported;
        info[1] += h.sweeps[0];
        info[2] += h.sweeps[1];
        if (debug)
            fprintf(stderr, "[exact] pass %u from %u/%u sweeps so far %llu/%llu m %u/%u first moved %d/%d tie launches %llu\n",
                    passes, F[0].from, F[1].from, info[1], info[2], F[0].m, F[1].m,
                    h.first_bad[0] == kNoRank ? -1 : (int)h.first_bad[0], h.first_bad[1] == kNoRank ? -1 : (int)h.first_bad[1],
                    info[3]);
        e = hipMemsetAsync(L.ctl->sweeps, 0, sizeof h.sweeps, st);
        if (e != hipSuccess) return e;
        for (int f = 0; f < nf; ++f) {
            if (!active[f]) continue;
            if (h.first_bad[f] == kNoRank) active[f] = false;
            else F[f].from = h.first_bad[f];
        }
        if (!active[0] && !active[1]) break;
    }
    info[0] = passes;
    return hipSuccess;
}

}  // namespace

size_t bidir_exact_work_bytes(int64_t n, int64_t m0, int64_t m1) {
    return exact_layout(nullptr, n, Geo2::K, m0, m1, false).total;
}

hipError_t bidir_exact(double* d_TG, double* d_TS, const double* d_cost, int64_t H, int64_t W, int64_t gnode,
                       int64_t snode, const unsigned* d_rg, const unsigned* d_rs, const int64_t members[2],
                       void* d_work, size_t work_bytes, unsigned long long* d_best, hipStream_t st,
                       unsigned long long info[4]) {
    const int64_t n = H * W;
    if (n >= (1ll << 29) || members[0] < 0 || members[1] < 0 || members[0] > n || members[1] > n)
        return hipErrorInvalidValue;
    const ExactLayout L = exact_layout(d_work, n, Geo2::K, members[0], members[1], false);
    if (L.total > work_bytes) return hipErrorOutOfMemory;
    const Geo2 g{H, W};
    Front F[2];
    double* T[2] = {d_TG, d_TS};
    const int64_t src[2] = {gnode, snode};
    const unsigned* rin[2] = {d_rg, d_rs};
    hipError_t e = hipSuccess;
    for (int f = 0; f < 2; ++f) {
        F[f] = Front{d_cost, T[f], L.rank[f], L.ord[f], L.ev[f], src[f], (unsigned)members[f], 0u};
        if (members[f] > 0) e = hipMemcpyAsync(L.rank[f], rin[f], sizeof(unsigned) * (size_t)n, hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) return e;
    }
    if (members[0] <= 0 || members[1] <= 0) return hipErrorInvalidValue;  // (the join found no meeting)
    const unsigned ng = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(exact_order_kernel, dim3(ng, 2), dim3(256), 0, st, F[0], F[1], n);
    e = hipMemsetAsync(L.ctl, 0, sizeof(Ctl), st);
    if (e == hipSuccess) e = hipMemsetAsync(L.ctl->nmin, 0xFF, sizeof(L.ctl->nmin), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(exact_nmin_kernel, dim3((unsigned)std::min<int64_t>(1024, ng), 2), dim3(256), 0, st, F[0], F[1], n,
                       L.ctl);
    e = replay(g, F, 2, L, st, info);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(d_best, 0xFF, sizeof(unsigned long long), st);
    if (e != hipSuccess) return e;
    e = bidir_join_min(L.rank[0], L.rank[1], n, d_best, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(exact_edge_kernel, dim3(1), dim3(64), 0, st, F[0], F[1], g, d_best, L.ctl);
    {
        unsigned edge = 0;
        e = hipMemcpyAsync(&edge, &L.ctl->edge, sizeof edge, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return e;
        if (edge) return hipErrorIllegalState;
    }
    hipLaunchKernelGGL(exact_fields_bidir_kernel, dim3(ng, 2), dim3(256), 0, st, F[0], F[1], g, d_best);
    return hipGetLastError();
}

size_t fm3d_exact_work_bytes(int64_t n) { return exact_layout(nullptr, n, Geo3::K, n, 0, true).total; }

hipError_t fm3d_exact(const double* d_cost, const double* d_T, double* d_Te, int64_t H, int64_t W, int64_t L3,
                      int64_t goal_off, int64_t start_off, void* d_work, size_t work_bytes, hipStream_t st,
                      unsigned long long info[4]) {
    const int64_t n = H * W * L3;
    if (n >= (1ll << 29) || goal_off < 0 || goal_off >= n || start_off < 0 || start_off >= n) return hipErrorInvalidValue;
    const ExactLayout L = exact_layout(d_work, n, Geo3::K, n, 0, true);
    if (L.total > work_bytes) return hipErrorOutOfMemory;
    const Geo3 g{H, W, L3};
    hipError_t e = hipMemsetAsync(L.ctl, 0, sizeof(Ctl), st);
    if (e != hipSuccess) return e;
    // the cells to rank (node order), their first order by T (stable: ties by node)
    hipLaunchKernelGGL(exact_thr_kernel, dim3(1), dim3(1), 0, st, d_T, start_off, L.ctl);
    size_t b = L.cub_bytes;
    e = hipcub::DeviceSelect::If(L.cub_tmp, b, hipcub::CountingInputIterator<unsigned>(0u), L.val, &L.ctl->msel,
                                            n, Fm3dMember{d_T, L.ctl}, st);
    if (e != hipSuccess) return e;
    unsigned m = 0;
    e = hipMemcpyAsync(&m, &L.ctl->msel, sizeof m, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return e;
    if (m == 0) return hipErrorInvalidValue;  // (the goal is always selected)
    const unsigned gm = (unsigned)((m + 255) / 256);
    hipLaunchKernelGGL(exact_tkeys_kernel, dim3(gm), dim3(256), 0, st, d_T, L.val, (int64_t)m, L.kT);
    b = L.cub_bytes;
    e = hipcub::DeviceRadixSort::SortPairs(L.cub_tmp, b, L.kT, L.kT2, L.val, L.ord[0], (int)m, 0, 64, st);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(L.rank[0], 0xFF, sizeof(unsigned) * (size_t)n, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(exact_scatter_rank_kernel, dim3(gm), dim3(256), 0, st, L.ord[0], (int64_t)m, L.rank[0]);
    Front F[2];
    F[0] = Front{d_cost, const_cast<double*>(d_T), L.rank[0], L.ord[0], L.ev[0], goal_off, m, 0u};
    F[1] = Front{d_cost, nullptr, L.rank[1], L.ord[1], L.ev[1], -1, 0u, 0u};
    e = replay(g, F, 1, L, st, info);
    if (e != hipSuccess) return e;
    const unsigned gn = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(exact_fields_early_kernel, dim3(gn), dim3(256), 0, st, F[0], g, start_off, d_Te);
    return hipGetLastError();
}

}  // namespace eik
