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
//  2. relax:   one workgroup per front walks the pops in rank order, groups of kGroup swept in place
//              until a sweep changes no event's bits (earlier groups are final; the band's tentative
//              values chain along the front, which in-order groups resolve as they go);
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
// Cost (profiles/r06m_exact_ab.log): the bench's planner step 1 (4096^2, 2.1 M pops per front)
// 12.7 ms -> ~0.39 s, of which the relaxation is ~95 % (one event's chain of dependent loads per
// group sweep, ~11 us, times ~33 k sweeps); an opt-in for bit-identity, not the default.
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
    const double* cost;  // H*W
    double* T;           // the converged field on entry (init values); the partial field on exit
    unsigned* rank;      // H*W: pop rank, kNoRank = not among the m ranked cells
    unsigned* ord;       // m: the cell of each rank
    double* ev;          // 4*H*W: events [cell][d], d = the direction of the popping neighbour
    int64_t src;         // the front's source (closed before the first pop, :120 / :123)
    unsigned m;
    unsigned from;       // this pass: first rank re-initialised / re-keyed
};

struct Ctl {
    unsigned act[2];        // fronts still re-ranking
    unsigned sweeps[2];     // group sweeps of the relaxation (accumulated over passes)
    unsigned first_bad[2];  // this pass: first rank that moved against the relaxation's order
    unsigned stuck[2];      // a group did not settle within kGroupSweepCap sweeps
    unsigned longrun;       // a run of equal T too long for exact_ties_kernel (1), or not closed (2)
};

// children / neighbours in the reference's order (:46-54): y - 1, y + 1, x - 1, x + 1
__device__ __forceinline__ int64_t nb_of(int64_t i, int64_t x, int64_t y, int d, int64_t H, int64_t W) {
    switch (d) {
        case 0: return y > 0 ? i - W : -1;
        case 1: return y + 1 < H ? i + W : -1;
        case 2: return x > 0 ? i - 1 : -1;
        default: return x + 1 < W ? i + 1 : -1;
    }
}
__device__ __forceinline__ int64_t dx_of(int d) { return d < 2 ? 0 : (d == 2 ? -1 : 1); }
__device__ __forceinline__ int64_t dy_of(int d) { return d >= 2 ? 0 : (d == 0 ? -1 : 1); }

// the min over z's events whose time (the popping neighbour's rank) is below lim
__device__ __forceinline__ double events_below(const Front& F, int64_t z, int64_t x, int64_t y, unsigned lim,
                                               int64_t H, int64_t W) {
    double v = Real<double>::inf();
    for (int d = 0; d < 4; ++d) {
        const int64_t j = nb_of(z, x, y, d, H, W);
        if (j >= 0 && F.rank[j] < lim) v = __builtin_fmin(v, F.ev[4 * z + d]);
    }
    return v;
}

// V(z, t): what cell z holds when the t-th pop updates its neighbours
__device__ __forceinline__ double value_at(const Front& F, int64_t z, int64_t x, int64_t y, unsigned t, int64_t H,
                                           int64_t W) {
    if (z == F.src) return 0.0;                                      // :132 / :135
    if (!(F.cost[z] < Real<double>::inf())) return Real<double>::inf();  // closed from the start (:121 / :124)
    const unsigned rz = F.rank[z];
    return events_below(F, z, x, y, rz < t ? rz : t, H, W);
}

// the update of y made by the t-th pop (updateNode :56-63): Thor = min(T[x+1], T[x-1]), Tver =
// min(T[y+1], T[y-1]) as of that pop
__device__ __forceinline__ double event_value(const Front& F, int64_t y, int64_t x, int64_t yy, unsigned t, double cy,
                                              int64_t H, int64_t W) {
    const double inf = Real<double>::inf();
    double v[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const int64_t j = nb_of(y, x, yy, d, H, W);
        v[d] = j < 0 ? inf : value_at(F, j, x + dx_of(d), yy + dy_of(d), t, H, W);
    }
    return eik_ref(__builtin_fmin(v[3], v[2]), __builtin_fmin(v[1], v[0]), cy);
}

// is y updated by the pop of rank r (y = child k of that pop)?  open (:56): not popped before, not
// +inf cost, not the source
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
__global__ __launch_bounds__(256) void exact_init_kernel(Front F0, Front F1, int64_t H, int64_t W) {
    const Front& F = blockIdx.y ? F1 : F0;
    const double inf = Real<double>::inf();
    const int64_t e1 = 4ll * F.m;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < e1; e += (int64_t)gridDim.x * blockDim.x) {
        const unsigned r = (unsigned)(e >> 2);
        const int k = (int)(e & 3);
        const int64_t c = F.ord[r], cyy = (unsigned)c / (unsigned)W, cx = c - cyy * W;
        const int64_t y = nb_of(c, cx, cyy, k, H, W);
        if (y < 0 || y == F.src || !(F.cost[y] < inf)) continue;
        const int64_t x = cx + dx_of(k), yy = cyy + dy_of(k);
        double v[4];
        for (int d = 0; d < 4; ++d) {
            const int64_t j = nb_of(y, x, yy, d, H, W);
            v[d] = j < 0 ? inf : F.T[j];
        }
        F.ev[4 * y + (k ^ 1)] = eik_ref(__builtin_fmin(v[3], v[2]), __builtin_fmin(v[1], v[0]), F.cost[y]);
    }
}

// 2. relaxation in rank order, Gauss-Seidel: one workgroup per front walks its pops from `from` in
//    groups of kGroup, sweeping each group's events in place until a sweep changes no event's bits.
//    An event reads only events of earlier ranks: the groups before are final, so a group settles in
//    (its own dependency depth + 1) sweeps -- a correction crosses a whole group per sweep instead of
//    one dependency step per GPU-wide launch.  One workgroup: its waves share the CU's L1, so a
//    barrier orders their global stores and loads (workgroup scope, no cache maintenance).
// pops per group, one event per thread: a group sweep is bound by one event's chain of dependent
// loads (~11 us), so short groups win -- on the bench's planner query (4096^2, 2.1 M pops per front)
// 256 / 512 / 1024 / 2048 / 4096 took 376 / 473 / 438 / 477 / 575 ms (33.4 / 24.1 / 11.1 / 6.4 / 3.7 k
// sweeps); global Jacobi sweeps over all events instead needed 1513 launches, 1.95 s: the band's
// tentative values chain along the front (profiles/r06m_exact_ab.log)
constexpr unsigned kGroup = 256;
constexpr unsigned kGroupSweepCap = 1u << 16;
__global__ __launch_bounds__(1024) void exact_relax_kernel(Front F0, Front F1, int64_t H, int64_t W, Ctl* ctl) {
    const int f = blockIdx.y;
    const Front& F = f ? F1 : F0;
    if (!ctl->act[f]) return;
    unsigned sweeps = 0;
    for (unsigned g0 = (F.from / kGroup) * kGroup; g0 < F.m; g0 += kGroup) {
        const unsigned g1 = min(g0 + kGroup, F.m);
        for (unsigned it = 0;; ++it) {
            bool ch = false;
            for (unsigned e = 4u * g0 + threadIdx.x; e < 4u * g1; e += blockDim.x) {
                const unsigned r = e >> 2;
                const int k = (int)(e & 3u);
                const int64_t c = F.ord[r], cyy = (unsigned)c / (unsigned)W, cx = c - cyy * W;
                const int64_t y = nb_of(c, cx, cyy, k, H, W);
                if (!child_open(F, y, r)) continue;
                const double g = event_value(F, y, cx + dx_of(k), cyy + dy_of(k), r, F.cost[y], H, W);
                double* slot = F.ev + 4 * y + (k ^ 1);
                if (__double_as_longlong(*slot) != __double_as_longlong(g)) {
                    *slot = g;
                    ch = true;
                }
            }
            ++sweeps;
            if (!__syncthreads_or(ch)) break;
            if (it >= kGroupSweepCap) {  // a DAG settles within its depth: never on valid input
                if (threadIdx.x == 0) ctl->stuck[f] = 1u;
                return;
            }
        }
    }
    if (threadIdx.x == 0) ctl->sweeps[f] += sweeps;
}

// the LIFO key of the cell y popped at rank r: its value (the min over its events before r) and seq
// = 4 x the time of the first event reaching that value (the last strict decrease, :70) + y's child
// index in that update -- the later the insertion, the earlier among equal T (bisect_left, :76)
__device__ __forceinline__ double pop_key(const Front& F, int64_t y, unsigned r, int64_t H, int64_t W, unsigned* seq) {
    if (y == F.src) {
        *seq = ~0u;  // pops first
        return 0.0;
    }
    const int64_t yy = (unsigned)y / (unsigned)W, x = y - yy * W;
    double best = Real<double>::inf();
    unsigned bt = kNoRank, s = 0u;
    for (int d = 0; d < 4; ++d) {
        const int64_t nb = nb_of(y, x, yy, d, H, W);
        if (nb < 0) continue;
        const unsigned t = F.rank[nb];
        if (t >= r) continue;
        const double v = F.ev[4 * y + d];
        if (v < best || (v == best && t < bt)) {
            best = v;
            bt = t;
            s = 4u * t + (unsigned)(d ^ 1);
        }
    }
    *seq = s;
    return best;
}

// 3a. the keys of every pop of rank >= from
__global__ void exact_keys_kernel(Front F, int64_t H, int64_t W, unsigned long long* kT, unsigned* kS,
                                  unsigned* val) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t cnt = (int64_t)F.m - F.from;
    if (j >= cnt) return;
    const unsigned r = F.from + (unsigned)j;
    unsigned seq;
    const double t = pop_key(F, F.ord[r], r, H, W, &seq);
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

// 3c. runs of exactly equal T v pop as the reference's list does: entries of equal T pop most recent
//     insertion first (bisect_left), and a pop may insert a child at exactly v (getEikonal's two-sided
//     form at |Thor - Tver| = cost gives Thor), which then pops NEXT, before older entries of v.  So
//     a run is a stack: its roots (members whose value v was set by a pop below the run) pushed in
//     insertion order (seq), then each pop pushes its children in updateNode's order (:46-54) whose
//     update from it is exactly v and that are not on the stack yet (an equal value is no strict
//     decrease, :70).  seq reads the ranks of earlier pops, themselves possibly in a run, so a tie
//     level settles once the levels below it have: each launch re-forms every run (its first
//     thread, runs are short) from the current ranks until a launch moves nothing.  The events stay
//     as the relaxation left them (a cell's value does not depend on the order of equal-T pops); the
//     pass's final check (every rank against the relaxation's order) catches any exception.
//     Launch s returns at once when launch s - 1 moved nothing.
constexpr int64_t kMaxRun = 4096;
__global__ void exact_ties_kernel(Front F, int64_t H, int64_t W, const unsigned long long* kT, int64_t cnt,
                                  unsigned* flags, int s, unsigned* longrun, unsigned* out_buf, unsigned* stack_buf) {
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
    const unsigned r0 = F.from + (unsigned)j;
    const double v = __longlong_as_double((long long)kT[j]);
    unsigned* out = out_buf + j;
    unsigned* stk = stack_buf + j;
    unsigned pushed[kMaxRun / 32];
    for (int w = 0; w < kMaxRun / 32; ++w) pushed[w] = 0u;
    // roots in ascending seq: the top of the stack is the latest insertion
    int sp = 0;
    unsigned* sseq = out;  // (the roots' seq, beside the stack, until the output is written)
    for (int a = 0; a < L; ++a) {
        const int64_t y = F.ord[r0 + a], yy = (unsigned)y / (unsigned)W, x = y - yy * W;
        unsigned bt = kNoRank, sq = 0u;
        if (y == F.src) {
            bt = 0u;
            sq = ~0u;
        } else {
            for (int d = 0; d < 4; ++d) {
                const int64_t nb = nb_of(y, x, yy, d, H, W);
                if (nb < 0) continue;
                const unsigned t = F.rank[nb];
                if (t < r0 && t < bt && F.ev[4 * y + d] == v) {
                    bt = t;
                    sq = 4u * t + (unsigned)(d ^ 1);
                }
            }
        }
        if (bt == kNoRank) continue;  // a child of a run member
        int b = sp++;
        while (b > 0 && sseq[b - 1] > sq) {
            stk[b] = stk[b - 1];
            sseq[b] = sseq[b - 1];
            --b;
        }
        stk[b] = (unsigned)y;
        sseq[b] = sq;
        pushed[a >> 5] |= 1u << (a & 31);
    }
    // pop: the output overwrites sseq from the front, which the stack no longer needs (sseq[i] is
    // only read while sorting the roots in)
    int no = 0;
    while (sp > 0) {
        const int64_t p = stk[--sp], py = (unsigned)p / (unsigned)W, px = p - py * W;
        out[no++] = (unsigned)p;
        for (int k = 0; k < 4; ++k) {
            const int64_t y = nb_of(p, px, py, k, H, W);
            if (y < 0) continue;
            const unsigned ry = F.rank[y];
            if (ry < r0 || ry >= r0 + (unsigned)L) continue;  // not in this run
            const int a = (int)(ry - r0);
            if (pushed[a >> 5] & (1u << (a & 31))) continue;
            if (F.ev[4 * y + (k ^ 1)] != v) continue;  // p's update of y is not exactly v
            pushed[a >> 5] |= 1u << (a & 31);
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

// 5. biComputeTmap's returned fields at the meeting k: popped cells (rank <= k) their value,
//    band cells (an open cell with a popped neighbour) their value as of the last pop, else +inf
__global__ void exact_fields_kernel(Front F0, Front F1, int64_t H, int64_t W, const unsigned long long* best) {
    const Front& F = blockIdx.y ? F1 : F0;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long b = *best;
    if (i >= H * W || b == ~0ull) return;  // never met: the caller reports it
    const unsigned k = (unsigned)(b >> 30);
    const int64_t yy = i / W, x = i - yy * W;
    const unsigned r = F.rank[i];
    double t = Real<double>::inf();
    if (i == F.src) {
        t = 0.0;
    } else if (F.cost[i] < Real<double>::inf()) {
        t = events_below(F, i, x, yy, r <= k ? r : k + 1u, H, W);  // (+inf when no neighbour popped)
    }
    F.T[i] = t;
}

struct ExactLayout {
    unsigned* rank[2];
    unsigned* ord[2];
    double* ev[2];
    unsigned long long *kT, *kT2, *kT3;
    unsigned *kS, *kS2, *val, *val2, *val3, *ord2, *ordp, *flags;
    char* cub_tmp;
    size_t cub_bytes;
    Ctl* ctl;
    size_t total;
};

size_t align256(size_t b) { return (b + 255) & ~size_t(255); }

ExactLayout exact_layout(void* work, int64_t n, int64_t m0, int64_t m1) {
    ExactLayout L{};
    const int64_t mx = std::max<int64_t>(1, std::max(m0, m1));
    size_t sort64 = 0, sort32 = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort32, (unsigned*)nullptr, (unsigned*)nullptr, (unsigned*)nullptr,
                                             (unsigned*)nullptr, (int)mx, 0, 32, (hipStream_t)0);
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort64, (unsigned long long*)nullptr,
                                             (unsigned long long*)nullptr, (unsigned*)nullptr, (unsigned*)nullptr,
                                             (int)mx, 0, 64, (hipStream_t)0);
    L.cub_bytes = align256(std::max(sort32, sort64));
    char* p = static_cast<char*>(work);
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char* q = p ? p + off : nullptr;
        off += align256(bytes);
        return q;
    };
    const int64_t m[2] = {m0, m1};
    for (int f = 0; f < 2; ++f) {
        L.ev[f] = reinterpret_cast<double*>(take(sizeof(double) * 4 * (size_t)n));
        L.rank[f] = reinterpret_cast<unsigned*>(take(sizeof(unsigned) * (size_t)n));
        L.ord[f] = reinterpret_cast<unsigned*>(take(sizeof(unsigned) * (size_t)std::max<int64_t>(1, m[f])));
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

__global__ void exact_ctl_kernel(Ctl* ctl, unsigned a0, unsigned a1) {
    ctl->act[0] = a0;
    ctl->act[1] = a1;
    ctl->first_bad[0] = ctl->first_bad[1] = kNoRank;
    ctl->longrun = 0u;
}

}  // namespace

size_t bidir_exact_work_bytes(int64_t n, int64_t m0, int64_t m1) { return exact_layout(nullptr, n, m0, m1).total; }

hipError_t bidir_exact(double* d_TG, double* d_TS, const double* d_cost, int64_t H, int64_t W, int64_t gnode,
                       int64_t snode, const unsigned* d_rg, const unsigned* d_rs, const int64_t members[2],
                       void* d_work, size_t work_bytes, unsigned long long* d_best, hipStream_t st,
                       unsigned long long info[4]) {
    const int64_t n = H * W;
    if (n >= (1ll << 29) || members[0] < 0 || members[1] < 0 || members[0] > n || members[1] > n)
        return hipErrorInvalidValue;
    const ExactLayout L = exact_layout(d_work, n, members[0], members[1]);
    if (L.total > work_bytes) return hipErrorOutOfMemory;
    Front F[2];
    double* T[2] = {d_TG, d_TS};
    const int64_t src[2] = {gnode, snode};
    const unsigned* rin[2] = {d_rg, d_rs};
    hipError_t e = hipSuccess;
    for (int f = 0; f < 2; ++f) {
        F[f] = Front{d_cost, T[f], L.rank[f], L.ord[f], L.ev[f], src[f], (unsigned)members[f], 0u};
        e = hipMemcpyAsync(L.rank[f], rin[f], sizeof(unsigned) * (size_t)n, hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) return e;
    }
    const unsigned ng = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(exact_order_kernel, dim3(ng, 2), dim3(256), 0, st, F[0], F[1], n);
    e = hipMemsetAsync(L.ctl, 0, sizeof(Ctl), st);
    if (e != hipSuccess) return e;
    {
        const int64_t mx = std::max(members[0], members[1]);
        const unsigned gi = (unsigned)std::max<int64_t>(1, std::min<int64_t>(4096, (4 * mx + 255) / 256));
        hipLaunchKernelGGL(exact_init_kernel, dim3(gi, 2), dim3(256), 0, st, F[0], F[1], H, W);
    }
    bool active[2] = {members[0] > 0, members[1] > 0};
    static const bool debug = getenv("EIK_EXACT_DEBUG") != nullptr;  // per-pass trace on stderr (diagnostics)
    unsigned passes = 0;
    for (;;) {
        if (++passes > kMaxPasses) return hipErrorNotReady;
        hipLaunchKernelGGL(exact_ctl_kernel, dim3(1), dim3(1), 0, st, L.ctl, active[0] ? 1u : 0u, active[1] ? 1u : 0u);
        hipLaunchKernelGGL(exact_relax_kernel, dim3(1, 2), dim3(1024), 0, st, F[0], F[1], H, W, L.ctl);
        // re-rank every active front from its first relaxed rank
        for (int f = 0; f < 2; ++f) {
            if (!active[f]) continue;
            const int64_t cnt = (int64_t)F[f].m - F[f].from;
            if (cnt <= 0) continue;
            const unsigned g = (unsigned)((cnt + 255) / 256);
            hipLaunchKernelGGL(exact_keys_kernel, dim3(g), dim3(256), 0, st, F[f], H, W, L.kT, L.kS, L.val);
            size_t b = L.cub_bytes;
            e = hipcub::DeviceRadixSort::SortPairs(L.cub_tmp, b, L.kS, L.kS2, L.val, L.val2, (int)cnt, 0, 32, st);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL(exact_gather_kernel, dim3(g), dim3(256), 0, st, L.kT, L.val2, F[f].from, cnt, L.kT2);
            b = L.cub_bytes;
            e = hipcub::DeviceRadixSort::SortPairs(L.cub_tmp, b, L.kT2, L.kT3, L.val2, L.val3, (int)cnt, 0, 64, st);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL(exact_moved_kernel, dim3(g), dim3(256), 0, st, F[f], L.val3, cnt, L.ord2);
            e = hipMemcpyAsync(L.ordp, F[f].ord + F[f].from, sizeof(unsigned) * (size_t)cnt, hipMemcpyDeviceToDevice, st);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL(exact_apply_kernel, dim3(g), dim3(256), 0, st, F[f], L.ord2, cnt);
            // the tie runs, in batches of kTieBatch launches until one moves nothing
            for (unsigned tb = 0;; ++tb) {
                if (tb >= kMaxTieBatches) return hipErrorNotReady;
                e = hipMemsetAsync(L.flags, 0, sizeof(unsigned) * kTieBatch, st);
                if (e != hipSuccess) return e;
                for (int q = 0; q < kTieBatch; ++q)
                    hipLaunchKernelGGL(exact_ties_kernel, dim3(g), dim3(256), 0, st, F[f], H, W, L.kT3, cnt, L.flags, q,
                                       &L.ctl->longrun, L.ord2, L.val2);
                unsigned hf[kTieBatch];
                e = hipMemcpyAsync(hf, L.flags, sizeof hf, hipMemcpyDeviceToHost, st);
                if (e == hipSuccess) e = hipStreamSynchronize(st);
                if (e != hipSuccess) return e;
                int q = 0;
                while (q < kTieBatch && hf[q]) ++q;
                info[3] += (unsigned long long)(q < kTieBatch ? q + 1 : kTieBatch);
                if (q < kTieBatch) break;
            }
            // ordp: the relaxation's order (the old ord after the copy above)
            hipLaunchKernelGGL(exact_cmp_kernel, dim3(g), dim3(256), 0, st, F[f], L.ordp, cnt, &L.ctl->first_bad[f]);
        }
        Ctl h{};
        e = hipMemcpyAsync(&h, L.ctl, sizeof h, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return e;
        if (h.stuck[0] || h.stuck[1]) return hipErrorNotReady;
        if (h.longrun) return hipErrorNotSupported;
        const unsigned* bad = h.first_bad;
        const unsigned* sw = h.sweeps;
        info[1] += sw[0];
        info[2] += sw[1];
        if (debug)
            fprintf(stderr, "[exact] pass %u from %u/%u sweeps so far %llu/%llu m %u/%u first moved %d/%d tie launches %llu\n",
                    passes, F[0].from, F[1].from, info[1], info[2], F[0].m, F[1].m, bad[0] == kNoRank ? -1 : (int)bad[0],
                    bad[1] == kNoRank ? -1 : (int)bad[1], info[3]);
        e = hipMemsetAsync(L.ctl->sweeps, 0, sizeof h.sweeps, st);
        if (e != hipSuccess) return e;
        for (int f = 0; f < 2; ++f) {
            if (!active[f]) continue;
            if (bad[f] == kNoRank) active[f] = false;
            else F[f].from = bad[f];
        }
        if (!active[0] && !active[1]) break;
    }
    info[0] = passes;
    e = hipMemsetAsync(d_best, 0xFF, sizeof(unsigned long long), st);
    if (e != hipSuccess) return e;
    e = bidir_join_min(L.rank[0], L.rank[1], n, d_best, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(exact_fields_kernel, dim3(ng, 2), dim3(256), 0, st, F[0], F[1], H, W, d_best);
    return hipGetLastError();
}

}  // namespace eik
