// bidir.hip -- nodeJoin of biComputeTmap (FastMarching.py:114-162) from two full fields.
//
// The reference advances a goal front and a start front one pop each per iteration and stops
// at iteration k when the goal front's k-th pop g_k is already closed by the start front
// (rankS(g_k) <= k, :150-152) or the start front's k-th pop s_k is closed by the goal front
// (rankG(s_k) <= k, :153-155).  A front pops nodes in increasing T, so with
//     rankG(n) = position of n in ascending TG,  rankS(n) = position in ascending TS
// the stopping iteration is k* = min_n max(rankG(n), rankS(n)), and the join is g_{k*} when it
// qualifies (the G test runs first), else s_{k*}.  Ties of exactly equal T are ranked by node
// index (the reference breaks them LIFO by insertion time, which a field does not record --
// SURVEY.md §7 "join approximated").
//
// Only the cells the fronts pop before they meet need a rank, so the join does not sort the
// raster.  It bounds k* first and ranks only the cells under the bound:
//   1. seed:   n0 = argmin over cells of max(TG, TS) (both finite) -> k* <= K0 = max(rankG(n0),
//              rankS(n0)), both ranks counted exactly in one pass beside a 256-bin coarse
//              histogram of each field over [0, 4 max(TG(n0), TS(n0))) (+ one overflow bin);
//              then n1 = argmin of the larger of the two histogram rank estimates, whose exact
//              ranks give K1; the bound is K = min(K0, K1)
//   2. select: per field the smallest value bucket holding >= K+1 cells (coarse scan, then a
//              1024-bin histogram inside that coarse bin) -> the member set {bucket(T) <=
//              threshold}, a prefix of the field's pop order that holds every cell of rank <= K
//   3. rank:   compact the members in node order (stable select), radix-sort them by T rounded to
//              float (stable: ties stay in node order), then put each run of equal floats in (T,
//              node) order -> their exact ranks; non-members keep rank UINT_MAX
//   4. join:   min over cells of max(rankG, rankS) as before.
// A non-member has rank > K >= k*, so it can be neither the join nor a closed cell of a partial
// field, and the members' ranks equal their ranks in the whole field (every cell below a member
// in pop order is a member).  The bucket function is monotone in T, so the member set is a prefix.
// The sort then covers ~K cells instead of H*W (the cells the fronts popped, plus one bucket).
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "eik_common.hpp"
#include "eik_kernels.hpp"

namespace eik {

constexpr int kCoarse = 256;   // coarse value buckets over [0, 4M) per field, the last one open-ended
constexpr int kFine = 1024;    // fine buckets inside the threshold's coarse bucket
constexpr unsigned kNone = 0xFFFFFFFFu;

// device control block of one join, in the work buffer after the sort scratch
struct JoinSel {
    unsigned long long n0;  // (bits(max(TG,TS)) with the low 29 bits cleared) | node; ~0: fronts never meet
    unsigned r0[2];         // exact ranks of n0 in TG / TS
    double scale;           // coarse buckets per unit of T: kCoarse / (4 M)
    int cb[2];              // threshold coarse bucket per field (-1: no member; kCoarse-1: every finite cell)
    int fb[2];              // threshold fine bucket inside cb
    unsigned need[2];       // members still needed inside cb (K0 + 1 - cells of lower coarse buckets)
    unsigned m[2];          // member count per field (select output)
    unsigned nb[2];         // band cells listed for the band relaxation (bidir_partial with a cost)
    unsigned sweeps[2];     // the band relaxation's sweeps
    unsigned longrun[2];    // a run of equal float keys longer than kFixupRun: sort that field by 64-bit keys
    unsigned long long n1;  // rank-aware seed: (estimated max rank) << 29 | node; ~0: none
    unsigned r1[2];         // exact ranks of n1
    unsigned pre[2][kCoarse];  // cells below each coarse bucket
    unsigned hc[2][kCoarse];
    unsigned hf[2][kFine];
};

__device__ __forceinline__ bool fin(double t) { return t < Real<double>::inf(); }

__device__ __forceinline__ int coarse_of(double t, double s) {
    const double q = t * s;
    return q >= double(kCoarse - 1) ? kCoarse - 1 : (int)q;
}

__device__ __forceinline__ int fine_of(double t, double s, int c) {
    const double q = (t * s - double(c)) * double(kFine);
    return q >= double(kFine - 1) ? kFine - 1 : (q <= 0.0 ? 0 : (int)q);
}

// the member test (monotone in t): a prefix of the field's pop order
struct JoinMember {
    const double* T;
    const JoinSel* sel;
    int f;
    __device__ bool operator()(const unsigned& i) const {
        const double t = T[i];
        const int tc = sel->cb[f];
        if (tc < 0 || !fin(t)) return false;
        const int c = coarse_of(t, sel->scale);
        if (c != tc) return c < tc;
        return tc == kCoarse - 1 || fine_of(t, sel->scale, c) <= sel->fb[f];
    }
};

template <typename V>
__device__ __forceinline__ V wave_min(V v) {
    for (int off = 32; off > 0; off >>= 1) {
        const V o = __shfl_xor(v, off, 64);
        v = o < v ? o : v;
    }
    return v;
}

__device__ __forceinline__ unsigned wave_sum(unsigned v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// LDS histogram add, aggregated over the wave: neighbouring cells mostly share a bucket, so the
// lanes agreeing with the first valid lane's bucket add once; the rest add one by one.  Called by
// every lane of the wave (uniform control flow).
__device__ __forceinline__ void hist_add(unsigned* h, int bin, bool valid) {
    const unsigned long long vm = __ballot(valid);
    if (!vm) return;
    const int src = __ffsll((long long)vm) - 1;
    const int b0 = __shfl(bin, src, 64);
    const bool same = valid && bin == b0;
    const unsigned long long sm = __ballot(same);
    if (same) {
        if ((int)(threadIdx.x & 63) == src) atomicAdd(&h[b0], (unsigned)__popcll(sm));
    } else if (valid) {
        atomicAdd(&h[bin], 1u);
    }
}

constexpr int kPassBlocks = 1024;  // grid-stride passes over the raster: 4 workgroups per CU

// 1a. n0: argmin of max(TG, TS) over the cells both fronts reach, to 2^-23 relative (the low 29
//     bits of the value carry the node) -- any such cell bounds k*, the closest only tightens it
__global__ __launch_bounds__(256) void join_seed_kernel(const double* __restrict__ TG, const double* __restrict__ TS,
                                                        int64_t n, JoinSel* __restrict__ sel) {
    __shared__ unsigned long long wmin[4];
    unsigned long long v = ~0ull;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const double a = TG[i], b = TS[i];
        if (fin(a) && fin(b)) {
            const unsigned long long m = (unsigned long long)__double_as_longlong(a > b ? a : b);
            const unsigned long long c = (m & ~((1ull << 29) - 1)) | (unsigned long long)i;
            v = c < v ? c : v;
        }
    }
    v = wave_min(v);
    if ((threadIdx.x & 63) == 0) wmin[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long m = wmin[0];
        for (int w = 1; w < 4; ++w) m = wmin[w] < m ? wmin[w] : m;
        if (m != ~0ull) atomicMin(&sel->n0, m);
    }
}

// 1b. the exact ranks of n0 in both fields (cells before it in (T, node) order) and the coarse
//     histograms (the scale join_scale_kernel derived from n0)
__global__ __launch_bounds__(256) void join_count_kernel(const double* __restrict__ TG, const double* __restrict__ TS,
                                                         int64_t n, JoinSel* __restrict__ sel) {
    __shared__ unsigned h[2][kCoarse];
    __shared__ unsigned wsum[2][4];
    const unsigned long long p = sel->n0;
    if (p == ~0ull) return;
    const int64_t node = (int64_t)(p & ((1ull << 29) - 1));
    const double g0 = TG[node], s0 = TS[node];
    const double s = sel->scale;
    for (int b = threadIdx.x; b < 2 * kCoarse; b += blockDim.x) (&h[0][0])[b] = 0;
    __syncthreads();
    unsigned cg = 0, cs = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x; i0 < n; i0 += stride) {
        const int64_t i = i0 + threadIdx.x;
        const bool in = i < n;
        const double a = in ? TG[i] : Real<double>::inf(), b = in ? TS[i] : Real<double>::inf();
        cg += (a < g0 || (a == g0 && i < node)) ? 1u : 0u;
        cs += (b < s0 || (b == s0 && i < node)) ? 1u : 0u;
        const bool fa = fin(a), fb = fin(b);
        hist_add(h[0], fa ? coarse_of(a, s) : 0, fa);
        hist_add(h[1], fb ? coarse_of(b, s) : 0, fb);
    }
    __syncthreads();
    cg = wave_sum(cg);
    cs = wave_sum(cs);
    if ((threadIdx.x & 63) == 0) {
        wsum[0][threadIdx.x >> 6] = cg;
        wsum[1][threadIdx.x >> 6] = cs;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        const unsigned t = wsum[threadIdx.x][0] + wsum[threadIdx.x][1] + wsum[threadIdx.x][2] + wsum[threadIdx.x][3];
        if (t) atomicAdd(&sel->r0[threadIdx.x], t);
    }
    for (int b = threadIdx.x; b < 2 * kCoarse; b += blockDim.x) {
        const unsigned v = (&h[0][0])[b];
        if (v) atomicAdd(&(&sel->hc[0][0])[b], v);
    }
}

// 2a. per field the first coarse bucket whose running count reaches K0 + 1 (one thread per field)
// 1c. a rank-aware seed: the value-space n0 can sit far from the meeting when the fronts grow at
//     different rates (a front in a corner or a corridor).  Each field's rank is estimated from its
//     coarse histogram (cells below the bucket + the bucket's share by linear position), and n1 =
//     argmin of the larger estimate; its exact ranks then give a second bound K1 (usually far
//     tighter), and the join keeps min(K0, K1).
__global__ void join_prefix_kernel(JoinSel* __restrict__ sel) {
    const int f = threadIdx.x;
    if (f >= 2) return;
    unsigned cum = 0;
    for (int b = 0; b < kCoarse; ++b) {
        sel->pre[f][b] = cum;
        cum += sel->hc[f][b];
    }
}

__device__ __forceinline__ unsigned rank_estimate(const JoinSel* sel, int f, double t) {
    const double q = t * sel->scale;
    const int b = coarse_of(t, sel->scale);
    const double frac = b == kCoarse - 1 ? 1.0 : (q - double(b) < 0.0 ? 0.0 : q - double(b));
    return sel->pre[f][b] + (unsigned)(frac * double(sel->hc[f][b]));
}

__global__ __launch_bounds__(256) void join_seed2_kernel(const double* __restrict__ TG, const double* __restrict__ TS,
                                                         int64_t n, JoinSel* __restrict__ sel) {
    __shared__ unsigned long long wmin[4];
    unsigned long long v = ~0ull;
    if (sel->n0 != ~0ull) {
        const int64_t stride = (int64_t)gridDim.x * blockDim.x;
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
            const double a = TG[i], b = TS[i];
            if (fin(a) && fin(b)) {
                const unsigned ea = rank_estimate(sel, 0, a), eb = rank_estimate(sel, 1, b);
                const unsigned long long c = ((unsigned long long)(ea > eb ? ea : eb) << 29) | (unsigned long long)i;
                v = c < v ? c : v;
            }
        }
    }
    v = wave_min(v);
    if ((threadIdx.x & 63) == 0) wmin[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long m = wmin[0];
        for (int w = 1; w < 4; ++w) m = wmin[w] < m ? wmin[w] : m;
        if (m != ~0ull) atomicMin(&sel->n1, m);
    }
}

// exact ranks of n1 (as join_count_kernel's of n0, without the histograms)
__global__ __launch_bounds__(256) void join_count2_kernel(const double* __restrict__ TG, const double* __restrict__ TS,
                                                          int64_t n, JoinSel* __restrict__ sel) {
    __shared__ unsigned wsum[2][4];
    const unsigned long long p = sel->n1;
    if (p == ~0ull) return;
    const int64_t node = (int64_t)(p & ((1ull << 29) - 1));
    const double g0 = TG[node], s0 = TS[node];
    unsigned cg = 0, cs = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const double a = TG[i], b = TS[i];
        cg += (a < g0 || (a == g0 && i < node)) ? 1u : 0u;
        cs += (b < s0 || (b == s0 && i < node)) ? 1u : 0u;
    }
    cg = wave_sum(cg);
    cs = wave_sum(cs);
    if ((threadIdx.x & 63) == 0) {
        wsum[0][threadIdx.x >> 6] = cg;
        wsum[1][threadIdx.x >> 6] = cs;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        const unsigned t = wsum[threadIdx.x][0] + wsum[threadIdx.x][1] + wsum[threadIdx.x][2] + wsum[threadIdx.x][3];
        if (t) atomicAdd(&sel->r1[threadIdx.x], t);
    }
}

__global__ void join_coarse_scan_kernel(JoinSel* __restrict__ sel) {
    const int f = threadIdx.x;
    if (f >= 2) return;
    if (sel->n0 == ~0ull) {
        sel->cb[f] = -1;
        return;
    }
    unsigned k0 = sel->r0[0] > sel->r0[1] ? sel->r0[0] : sel->r0[1];
    if (sel->n1 != ~0ull) {
        const unsigned k1 = sel->r1[0] > sel->r1[1] ? sel->r1[0] : sel->r1[1];
        k0 = k1 < k0 ? k1 : k0;
    }
    unsigned cum = 0;
    int c = kCoarse - 1;
    for (int b = 0; b < kCoarse; ++b) {
        if (cum + sel->hc[f][b] >= k0 + 1) {
            c = b;
            break;
        }
        cum += sel->hc[f][b];
    }
    sel->cb[f] = c;
    sel->need[f] = k0 + 1 - cum;
    sel->fb[f] = kFine - 1;
}

// 2b. fine histogram of the cells inside the threshold coarse bucket
__global__ __launch_bounds__(256) void join_fine_kernel(const double* __restrict__ TG, const double* __restrict__ TS,
                                                        int64_t n, JoinSel* __restrict__ sel) {
    __shared__ unsigned h[2][kFine];
    const int c0 = sel->cb[0], c1 = sel->cb[1];
    const bool w0 = c0 >= 0 && c0 < kCoarse - 1, w1 = c1 >= 0 && c1 < kCoarse - 1;
    if (!w0 && !w1) return;
    const double s = sel->scale;
    for (int b = threadIdx.x; b < 2 * kFine; b += blockDim.x) (&h[0][0])[b] = 0;
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x; i0 < n; i0 += stride) {
        const int64_t i = i0 + threadIdx.x;
        const bool in = i < n;
        if (w0) {
            const double a = in ? TG[i] : Real<double>::inf();
            const bool v = fin(a) && coarse_of(a, s) == c0;
            hist_add(h[0], v ? fine_of(a, s, c0) : 0, v);
        }
        if (w1) {
            const double b = in ? TS[i] : Real<double>::inf();
            const bool v = fin(b) && coarse_of(b, s) == c1;
            hist_add(h[1], v ? fine_of(b, s, c1) : 0, v);
        }
    }
    __syncthreads();
    for (int b = threadIdx.x; b < 2 * kFine; b += blockDim.x) {
        const unsigned v = (&h[0][0])[b];
        if (v) atomicAdd(&(&sel->hf[0][0])[b], v);
    }
}

__global__ void join_fine_scan_kernel(JoinSel* __restrict__ sel) {
    const int f = threadIdx.x;
    if (f >= 2) return;
    const int c = sel->cb[f];
    if (c < 0 || c == kCoarse - 1) return;
    unsigned cum = 0;
    int t = kFine - 1;
    for (int b = 0; b < kFine; ++b) {
        cum += sel->hf[f][b];
        if (cum >= sel->need[f]) {
            t = b;
            break;
        }
    }
    sel->fb[f] = t;
}

// the scale both histograms and the member test use, from n0 (one thread)
__global__ void join_scale_kernel(const double* __restrict__ TG, const double* __restrict__ TS,
                                  JoinSel* __restrict__ sel) {
    const unsigned long long p = sel->n0;
    if (p == ~0ull) {
        sel->scale = 1.0;
        return;
    }
    const int64_t node = (int64_t)(p & ((1ull << 29) - 1));
    const double g0 = TG[node], s0 = TS[node];
    const double M = g0 > s0 ? g0 : s0;
    sel->scale = double(kCoarse) / (4.0 * (M > 0.0 ? M : 1.0));
}

// 3. keys of the compacted members (node order) for the stable sort: T rounded to float (monotone,
//    so the float order is the double order wherever the floats differ), 32-bit keys -- half the
//    radix passes of the doubles' bits; join_fixup_kernel then orders the runs of equal floats
__global__ void join_gather_kernel(const double* __restrict__ T, const unsigned* __restrict__ list, int64_t m,
                                   unsigned* __restrict__ keys, unsigned* __restrict__ idx) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const unsigned i = list[j];
    keys[j] = __float_as_uint((float)T[i]);  // T >= 0: the float bits order as unsigned
    idx[j] = i;
}

// After the stable sort by float key (ties in node order): each run of equal float keys is put in
// (T, node) order -- insertion sort by its first thread.  Runs are short (cells whose T agree to
// float precision); runs of exactly equal T are already in node order, so they cost one pass.  A
// run longer than kFixupRun (e.g. a zero-cost region, whose distinct T of ~2^-500 all round to the
// float 0) is left alone and flags the field (longrun): bidir_join then sorts that field again by
// the doubles' 64-bit patterns, so no run costs a quadratic insertion sort on one thread.
constexpr int64_t kFixupRun = 1024;
__global__ void join_fixup_kernel(const double* __restrict__ T, const unsigned* __restrict__ key, int64_t m,
                                  unsigned* __restrict__ idx, unsigned* __restrict__ longrun) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j + 1 >= m || key[j + 1] != key[j] || (j > 0 && key[j - 1] == key[j])) return;  // run starts only
    int64_t e = j + 2;
    while (e < m && key[e] == key[j] && e - j <= kFixupRun) ++e;
    if (e - j > kFixupRun) {
        atomicOr(longrun, 1u);
        return;
    }
    for (int64_t a = j + 1; a < e; ++a) {
        const unsigned ia = idx[a];
        const double ta = T[ia];
        int64_t b = a - 1;
        while (b >= j) {
            const unsigned ib = idx[b];
            const double tb = T[ib];
            if (tb < ta || (tb == ta && ib < ia)) break;
            idx[b + 1] = ib;
            --b;
        }
        idx[b + 1] = ia;
    }
}

// the fallback's keys: the doubles' bit patterns (T >= 0: they order as unsigned), exact
__global__ void join_gather64_kernel(const double* __restrict__ T, const unsigned* __restrict__ list, int64_t m,
                                     unsigned long long* __restrict__ keys, unsigned* __restrict__ idx) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const unsigned i = list[j];
    keys[j] = (unsigned long long)__double_as_longlong(T[i]);
    idx[j] = i;
}

// rank[sorted_idx[k]] = k for the members; every other cell keeps UINT_MAX (memset)
__global__ void scatter_rank_kernel(const unsigned* __restrict__ sidx, int64_t m, unsigned* __restrict__ rank) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    rank[sidx[k]] = (unsigned)k;
}

// packed = (2*max(rG,rS) + (rG == max ? 0 : 1)) << 29 | node ; the min identifies the join.
// Grid-stride over the cells, a wave then a workgroup (LDS) minimum, ONE atomicMin per workgroup:
// one atomic per wave on the single result word serialised ~260k device-scope atomics for a
// 4096^2 raster (2.98 ms, tools/rover_probe.py under rocprofv3).
__global__ __launch_bounds__(256) void join_min_kernel(const unsigned* __restrict__ rg, const unsigned* __restrict__ rs,
                                                       int64_t n, unsigned long long* __restrict__ best) {
    __shared__ unsigned long long wmin[4];
    unsigned long long v = ~0ull;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const unsigned a = rg[i], b = rs[i];
        if (a != kNone && b != kNone) {
            const unsigned long long m = a > b ? a : b;
            const unsigned long long c = ((2ull * m + (a == m ? 0ull : 1ull)) << 29) | (unsigned long long)i;
            v = c < v ? c : v;
        }
    }
    v = wave_min(v);
    if ((threadIdx.x & 63) == 0) wmin[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long m = wmin[0];
        for (int w = 1; w < 4; ++w) m = wmin[w] < m ? wmin[w] : m;
        if (m != ~0ull) atomicMin(best, m);
    }
}

namespace {

struct JoinLayout {
    unsigned long long *k_in, *k_out;
    unsigned *i_in, *i_out, *rg, *rs;
    char* cub_tmp;
    size_t cub_bytes;
    JoinSel* sel;
    size_t total;
};

size_t cub_scratch(int64_t n) {
    size_t sort_b = 0, sel_b = 0;
    size_t sort32_b = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort32_b, (unsigned*)nullptr, (unsigned*)nullptr,
                                             (unsigned*)nullptr, (unsigned*)nullptr, (int)n, 0, 32, (hipStream_t)0);
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort_b, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                             (unsigned*)nullptr, (unsigned*)nullptr, (int)n, 0, 64, (hipStream_t)0);
    (void)hipcub::DeviceSelect::If(nullptr, sel_b, hipcub::CountingInputIterator<unsigned>(0u), (unsigned*)nullptr,
                                   (unsigned*)nullptr, n, JoinMember{nullptr, nullptr, 0}, (hipStream_t)0);
    return (std::max(std::max(sort_b, sort32_b), sel_b) + 255) & ~size_t(255);
}

// k_in | k_out (n u64) | i_in | i_out | rg | rs (n u32) | cub scratch | JoinSel
JoinLayout layout(void* work, int64_t n) {
    JoinLayout L{};
    char* p = static_cast<char*>(work);
    L.k_in = reinterpret_cast<unsigned long long*>(p);
    L.k_out = L.k_in + n;
    L.i_in = reinterpret_cast<unsigned*>(L.k_out + n);
    L.i_out = L.i_in + n;
    L.rg = L.i_out + n;
    L.rs = L.rg + n;
    const size_t head = ((size_t)n * (2 * 8 + 4 * 4) + 255) & ~size_t(255);
    L.cub_tmp = p + head;
    L.cub_bytes = cub_scratch(n);
    L.sel = reinterpret_cast<JoinSel*>(L.cub_tmp + L.cub_bytes);
    L.total = head + L.cub_bytes + ((sizeof(JoinSel) + 255) & ~size_t(255));
    return L;
}

}  // namespace

// d_TG/d_TS: n doubles (full fields); d_work: bidir_join_work_bytes(n).  One host synchronisation
// (the member counts size the sorts).  members (optional, host): the two member-set sizes.
// steps 1-2 of the join: the bound K0 and each field's member threshold bucket, in sel
static hipError_t join_bound(const double* d_TG, const double* d_TS, int64_t n, JoinSel* sel, hipStream_t st) {
    hipError_t e = hipMemsetAsync(sel, 0, sizeof(JoinSel), st);
    if (e == hipSuccess) e = hipMemsetAsync(&sel->n0, 0xFF, sizeof(sel->n0), st);
    if (e == hipSuccess) e = hipMemsetAsync(&sel->n1, 0xFF, sizeof(sel->n1), st);
    if (e != hipSuccess) return e;
    const unsigned pgrid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(kPassBlocks, (n + 255) / 256));
    hipLaunchKernelGGL(join_seed_kernel, dim3(pgrid), dim3(256), 0, st, d_TG, d_TS, n, sel);
    hipLaunchKernelGGL(join_scale_kernel, dim3(1), dim3(1), 0, st, d_TG, d_TS, sel);
    hipLaunchKernelGGL(join_count_kernel, dim3(pgrid), dim3(256), 0, st, d_TG, d_TS, n, sel);
    hipLaunchKernelGGL(join_prefix_kernel, dim3(1), dim3(64), 0, st, sel);
    hipLaunchKernelGGL(join_seed2_kernel, dim3(pgrid), dim3(256), 0, st, d_TG, d_TS, n, sel);
    hipLaunchKernelGGL(join_count2_kernel, dim3(pgrid), dim3(256), 0, st, d_TG, d_TS, n, sel);
    hipLaunchKernelGGL(join_coarse_scan_kernel, dim3(1), dim3(64), 0, st, sel);
    hipLaunchKernelGGL(join_fine_kernel, dim3(pgrid), dim3(256), 0, st, d_TG, d_TS, n, sel);
    hipLaunchKernelGGL(join_fine_scan_kernel, dim3(1), dim3(64), 0, st, sel);
    return hipGetLastError();
}

hipError_t bidir_join(const double* d_TG, const double* d_TS, int64_t n, void* d_work, size_t work_bytes,
                      unsigned long long* d_best, hipStream_t st, int64_t* members) {
    if (n >= (1ll << 29)) return hipErrorInvalidValue;
    const JoinLayout L = layout(d_work, n);
    if (L.total > work_bytes) return hipErrorOutOfMemory;
    JoinSel* sel = L.sel;
    hipError_t e = join_bound(d_TG, d_TS, n, sel, st);
    if (e != hipSuccess) return e;
    // stable compaction of the members: G into i_in, S into rs (free until its ranks are scattered)
    const double* T[2] = {d_TG, d_TS};
    unsigned* lists[2] = {L.i_in, L.rs};
    for (int f = 0; f < 2; ++f) {
        size_t b = L.cub_bytes;
        e = hipcub::DeviceSelect::If(L.cub_tmp, b, hipcub::CountingInputIterator<unsigned>(0u), lists[f], &sel->m[f],
                                     n, JoinMember{T[f], sel, f}, st);
        if (e != hipSuccess) return e;
    }
    unsigned hm[2] = {0, 0};
    e = hipMemcpyAsync(hm, sel->m, sizeof hm, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return e;
    if (members) {
        members[0] = hm[0];
        members[1] = hm[1];
    }
    unsigned* rank[2] = {L.rg, L.rs};
    for (int f = 0; f < 2; ++f) {
        const int64_t m = hm[f];
        if (m > 0) {
            const unsigned g = (unsigned)((m + 255) / 256);
            hipLaunchKernelGGL(join_gather_kernel, dim3(g), dim3(256), 0, st, T[f], lists[f], m,
                               reinterpret_cast<unsigned*>(L.k_in), L.i_in);
        }
        e = hipMemsetAsync(rank[f], 0xFF, sizeof(unsigned) * (size_t)n, st);
        if (e != hipSuccess) return e;
        if (m > 0) {
            size_t b = L.cub_bytes;
            unsigned* k32_in = reinterpret_cast<unsigned*>(L.k_in);
            unsigned* k32_out = reinterpret_cast<unsigned*>(L.k_out);
            e = hipcub::DeviceRadixSort::SortPairs(L.cub_tmp, b, k32_in, k32_out, L.i_in, L.i_out, (int)m, 0, 32, st);
            if (e != hipSuccess) return e;
            const unsigned g = (unsigned)((m + 255) / 256);
            hipLaunchKernelGGL(join_fixup_kernel, dim3(g), dim3(256), 0, st, T[f], k32_out, m, L.i_out,
                               &sel->longrun[f]);
            hipLaunchKernelGGL(scatter_rank_kernel, dim3(g), dim3(256), 0, st, L.i_out, m, rank[f]);
        }
    }
    // a field with a run of equal float keys too long for the fix-up: its members again (the select
    // is stable and deterministic: the same list), sorted by the 64-bit patterns, ranks re-scattered
    unsigned lr[2] = {0, 0};
    e = hipMemcpyAsync(lr, sel->longrun, sizeof lr, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return e;
    for (int f = 0; f < 2; ++f) {
        const int64_t m = hm[f];
        if (!lr[f] || m <= 0) continue;
        size_t b = L.cub_bytes;
        e = hipcub::DeviceSelect::If(L.cub_tmp, b, hipcub::CountingInputIterator<unsigned>(0u), L.i_in, &sel->m[f], n,
                                     JoinMember{T[f], sel, f}, st);
        if (e != hipSuccess) return e;
        const unsigned g = (unsigned)((m + 255) / 256);
        hipLaunchKernelGGL(join_gather64_kernel, dim3(g), dim3(256), 0, st, T[f], L.i_in, m, L.k_in, L.i_in);
        b = L.cub_bytes;
        e = hipcub::DeviceRadixSort::SortPairs(L.cub_tmp, b, L.k_in, L.k_out, L.i_in, L.i_out, (int)m, 0, 64, st);
        if (e != hipSuccess) return e;
        e = hipMemsetAsync(rank[f], 0xFF, sizeof(unsigned) * (size_t)n, st);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(scatter_rank_kernel, dim3(g), dim3(256), 0, st, L.i_out, m, rank[f]);
    }
    e = hipMemsetAsync(d_best, 0xFF, sizeof(unsigned long long), st);
    if (e != hipSuccess) return e;
    const unsigned jgrid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(kPassBlocks, (n + 255) / 256));
    hipLaunchKernelGGL(join_min_kernel, dim3(jgrid), dim3(256), 0, st, L.rg, L.rs, n, d_best);
    return hipGetLastError();
}

// biComputeTmap returns the PARTIAL fields of the two fronts at the meeting iteration k
// (FastMarching.py:141-162): front f has popped its source and the next k nodes, i.e. the cells of
// rank <= k in its field (rank 0 = the source).  Those keep their final values; every cell that is
// neither popped nor in the narrow band (finite cost, a popped 4-neighbour) is +inf, as the
// reference leaves it.  A band cell holds the reference's TENTATIVE value: its last update, made
// when its last popped neighbour was popped, from the values its neighbours had then.  That
// depends on the sequential pop order and has no parallel form; it lies between the cell's
// full-field value (below) and the update from its popped neighbours alone (above).
//  * with the cost (tmap2d_bidir, the rover path): the band relaxation below -- the fixed point of
//    the local solve over popped + band cells with every other cell +inf, a tighter lower bound
//    (on the reference fixtures: exact on 82-100 % of the band cells against 78-100 % for the
//    full-field value; the largest excess stays 1.17 %, the others fall, e.g. 0.86 -> 0.48 %;
//    tools/band_analysis.py, profiles/r04v_band_analysis.log);
//  * without (eik_bidir_join_f64 on given fields): the full-field value.
// In place: a cell's own value changes only to +inf (or its relaxed value), its neighbours'
// closedness comes from the ranks.  (viol: the capped fronts' check, see FrontsCheck -- a band cell
// of finite cost left +inf by the cap would have had a finite value in the full field.)
__global__ void bidir_partial_kernel(double* __restrict__ T, const unsigned* __restrict__ rank, int64_t H, int64_t W,
                                     const unsigned long long* __restrict__ best, const double* __restrict__ cost,
                                     unsigned* __restrict__ viol, unsigned* __restrict__ blist,
                                     unsigned* __restrict__ bcount) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long b = *best;
    if (i >= H * W || b == ~0ull) return;  // fronts never met: the reference raises, fields unused
    const unsigned k = (unsigned)(b >> 30);
    if (rank[i] <= k) return;
    const int64_t y = i / W, x = i - y * W;
    const bool band = (x > 0 && rank[i - 1] <= k) || (x + 1 < W && rank[i + 1] <= k) ||
                      (y > 0 && rank[i - W] <= k) || (y + 1 < H && rank[i + W] <= k);
    if (!band) {
        T[i] = Real<double>::inf();
        return;
    }
    // (with a band list the value is recomputed from the closed cells below, so a cut-off value
    // does not survive and needs no fallback: the check is for the full-field band values only)
    if (viol && !blist && !fin(T[i]) && fin(cost[i])) atomicOr(viol, 1u);
    if (blist && fin(cost[i])) {
        // relaxed by bidir_band_kernel from the update over its closed neighbours alone (an upper
        // bound of the fixed point, already equal to it where the upwind neighbours are closed);
        // closed cells are never written here, so their values are final
        const double inf = Real<double>::inf();
        auto cv = [&](bool in, int64_t j) { return in && rank[j] <= k ? T[j] : inf; };
        const double l = cv(x > 0, i - 1), r = cv(x + 1 < W, i + 1), u = cv(y > 0, i - W), d = cv(y + 1 < H, i + W);
        T[i] = godunov2(l < r ? l : r, u < d ? u : d, cost[i]);
        blist[atomicAdd(bcount, 1u)] = (unsigned)i;
    }
}

// The band relaxation: sweeps over both fronts' band lists, one launch per sweep across the GPU,
// each cell updated in place (monotone from an upper bound: the fixed point does not depend on the
// order) until a sweep decreases nothing beyond rounding.  Sweep s records a change in flags[s];
// sweep s + 1 returns at once when sweep s changed nothing, so batches of sweeps are queued without
// waiting and the host reads the flags once per batch.
constexpr int kBandBatch = 16, kBandMaxBatches = 4096;
__global__ void bidir_band_sweep_kernel(double* __restrict__ TG, double* __restrict__ TS, const double* __restrict__ cost,
                                        int64_t H, int64_t W, const unsigned* __restrict__ listG,
                                        const unsigned* __restrict__ listS, const JoinSel* __restrict__ sel,
                                        unsigned* __restrict__ flags, int s) {
    if (s > 0 && flags[s - 1] == 0u) return;  // converged
    const unsigned nG = sel->nb[0], nS = sel->nb[1];
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= (int64_t)nG + nS) return;
    double* T = j < nG ? TG : TS;
    const int64_t i = j < nG ? listG[j] : listS[j - nG];
    const int64_t y = i / W, x = i - y * W;
    const double inf = Real<double>::inf();
    const double l = x > 0 ? T[i - 1] : inf, r = x + 1 < W ? T[i + 1] : inf;
    const double u = y > 0 ? T[i - W] : inf, d = y + 1 < H ? T[i + W] : inf;
    const double w = godunov2(l < r ? l : r, u < d ? u : d, cost[i]);  // getEikonal's branches
    const double t = T[i];
    if (w < t) {
        T[i] = w;
        // another sweep only for a decrease beyond rounding: cells that feed each other can
        // otherwise trade last-ulp decreases for many sweeps
        if (w < t * (1.0 - 0x1p-40)) flags[s] = 1u;
    }
}

hipError_t bidir_partial(double* d_TG, double* d_TS, int64_t H, int64_t W, const void* d_work,
                         const unsigned long long* d_best, hipStream_t st, const double* d_cost, unsigned* d_viol) {
    const int64_t n = H * W;
    const JoinLayout L = layout(const_cast<void*>(d_work), n);
    const unsigned grid = (unsigned)((n + 255) / 256);
    // band lists in the (now free) key arrays
    unsigned* lg = d_cost ? reinterpret_cast<unsigned*>(L.k_in) : nullptr;
    unsigned* ls = d_cost ? reinterpret_cast<unsigned*>(L.k_out) : nullptr;
    if (d_cost) {
        hipError_t e = hipMemsetAsync(L.sel->nb, 0, sizeof(L.sel->nb), st);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(bidir_partial_kernel, dim3(grid), dim3(256), 0, st, d_TG, L.rg, H, W, d_best, d_cost, d_viol, lg,
                       &L.sel->nb[0]);
    hipLaunchKernelGGL(bidir_partial_kernel, dim3(grid), dim3(256), 0, st, d_TS, L.rs, H, W, d_best, d_cost, d_viol, ls,
                       &L.sel->nb[1]);
    if (d_cost) {
        unsigned hnb[2] = {0, 0};  // the band sizes size the sweep launches
        hipError_t e = hipMemcpyAsync(hnb, L.sel->nb, sizeof hnb, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return e;
        const int64_t cnt = (int64_t)hnb[0] + hnb[1];
        if (cnt > 0) {
            unsigned* flags = L.i_in;  // free after the join
            const unsigned g = (unsigned)((cnt + 255) / 256);
            unsigned sweeps = 0;
            bool converged = false;
            // a sweep in place finalises every cell whose dependency chain through the band is no
            // longer than the sweeps so far, and no chain is longer than the band: cnt sweeps suffice
            const int64_t max_batches = std::min<int64_t>(kBandMaxBatches, cnt / kBandBatch + 2);
            for (int64_t batch = 0; batch < max_batches; ++batch) {
                e = hipMemsetAsync(flags, 0, sizeof(unsigned) * kBandBatch, st);
                if (e != hipSuccess) return e;
                for (int q = 0; q < kBandBatch; ++q)
                    hipLaunchKernelGGL(bidir_band_sweep_kernel, dim3(g), dim3(256), 0, st, d_TG, d_TS, d_cost, H, W, lg, ls,
                                       L.sel, flags, q);
                unsigned hf[kBandBatch];
                e = hipMemcpyAsync(hf, flags, sizeof hf, hipMemcpyDeviceToHost, st);
                if (e == hipSuccess) e = hipStreamSynchronize(st);
                if (e != hipSuccess) return e;
                int last = 0;
                while (last < kBandBatch && hf[last]) ++last;  // sweeps that changed something
                sweeps += (unsigned)(last < kBandBatch ? last + 1 : kBandBatch);
                if (last < kBandBatch) {
                    converged = true;
                    break;
                }
            }
            const unsigned sw[2] = {sweeps, sweeps};
            e = hipMemcpyAsync(L.sel->sweeps, sw, sizeof sw, hipMemcpyHostToDevice, st);  // (pageable: staged now)
            if (e != hipSuccess) return e;
            // not settled within the bound (never on valid input): the caller reports it as
            // EIK_ERR_NOCONVERGE instead of returning unrelaxed band values
            if (!converged) return hipErrorNotReady;
        }
    }
    return hipGetLastError();
}

// ------------------------------------------------------------ capped fronts (solve_fronts)
// The fronts only matter up to the meeting: every cell of rank <= k* and the band around them.
// eikonal_api.cpp's solve_fronts estimates each front's value at the meeting on a coarse copy of
// the raster (F x F blocks), solves the two full-resolution fronts with that value (+ margin) as
// an activation cap (Fim2dArgs::tcap), and checks the result here: every kept cell (T <= cap) is
// exact, so the join on the capped fields is the join on the full fields when the meeting rank is
// below both fronts' kept cell counts and no band cell was cut off.  Otherwise: the uncapped solve.

// coarse block cost: the mean finite cost of the F x F block, +inf when more than half of it is
// +inf; and the raster's largest finite cost (a band cell exceeds a closed neighbour by <= its cost)
__global__ __launch_bounds__(256) void coarse_cost_kernel(const double* __restrict__ cost, int64_t H, int64_t W, int F,
                                                          double* __restrict__ out, int64_t Hc, int64_t Wc,
                                                          FrontsCheck* __restrict__ chk) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double mx = 0.0;
    if (j < Hc * Wc) {
        const int64_t cy = j / Wc, cx = j - cy * Wc;
        const int64_t y1 = std::min<int64_t>(H, (cy + 1) * F), x1 = std::min<int64_t>(W, (cx + 1) * F);
        double sum = 0.0;
        int nf = 0, ni = 0;
        for (int64_t y = cy * F; y < y1; ++y)
            for (int64_t x = cx * F; x < x1; ++x) {
                const double v = cost[y * W + x];
                if (fin(v)) {
                    sum += v;
                    ++nf;
                    mx = v > mx ? v : mx;
                } else {
                    ++ni;
                }
            }
        out[j] = (nf == 0 || ni > nf) ? Real<double>::inf() : sum / nf;
    }
    unsigned long long b = (unsigned long long)__double_as_longlong(mx);
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(b, off, 64);
        b = o > b ? o : b;
    }
    if ((threadIdx.x & 63) == 0 && b) atomicMax(&chk->maxcost_bits, b);
}

// the capped fields: T above the map's cap -> +inf (an upper bound, not the converged value), and
// the kept (finite) cells per map
__global__ __launch_bounds__(256) void cap_clean_kernel(double* __restrict__ T, int64_t n, FrontsCheck* __restrict__ chk) {
    __shared__ unsigned ws[2][4];
    const double c0 = chk->caps[0], c1 = chk->caps[1];
    unsigned k0 = 0, k1 = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < 2 * n; i += stride) {
        const bool m1 = i >= n;
        const double v = T[i];
        if (fin(v)) {
            if (v > (m1 ? c1 : c0)) T[i] = Real<double>::inf();
            else if (m1) ++k1;
            else ++k0;
        }
    }
    k0 = wave_sum(k0);
    k1 = wave_sum(k1);
    if ((threadIdx.x & 63) == 0) {
        ws[0][threadIdx.x >> 6] = k0;
        ws[1][threadIdx.x >> 6] = k1;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        const unsigned t = ws[threadIdx.x][0] + ws[threadIdx.x][1] + ws[threadIdx.x][2] + ws[threadIdx.x][3];
        if (t) atomicAdd(&chk->kept[threadIdx.x], t);
    }
}

hipError_t fronts_coarse_cost(const double* d_cost, int64_t H, int64_t W, int F, double* d_out, int64_t Hc, int64_t Wc,
                              FrontsCheck* chk, hipStream_t st) {
    hipError_t e = hipMemsetAsync(chk, 0, sizeof(FrontsCheck), st);
    if (e != hipSuccess) return e;
    const int64_t nc = Hc * Wc;
    hipLaunchKernelGGL(coarse_cost_kernel, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, st, d_cost, H, W, F, d_out,
                       Hc, Wc, chk);
    return hipGetLastError();
}

// caps from the coarse fields' join bound alone (no ranks: no sort, no host synchronisation): the
// upper edge of each field's member threshold bucket is >= its T at rank K0 >= k*
__global__ void fronts_caps_bound_kernel(const JoinSel* __restrict__ sel, double F, double margin,
                                         FrontsCheck* __restrict__ chk) {
    const int f = threadIdx.x;
    if (f >= 2) return;
    const double mc = __longlong_as_double((long long)chk->maxcost_bits);
    const int cb = sel->cb[f];
    double cap = Real<double>::inf();  // fronts never met, or the threshold in the open bucket
    if (sel->n0 != ~0ull && cb >= 0 && cb < kCoarse - 1)
        cap = F * ((double(cb) + double(sel->fb[f] + 1) / double(kFine)) / sel->scale) * margin + mc;
    chk->caps[f] = cap;
    chk->best_c = sel->n0;
}

hipError_t fronts_estimate(const double* d_TG, const double* d_TS, int64_t n, void* d_work, double F, double margin,
                           FrontsCheck* chk, hipStream_t st) {
    if (n >= (1ll << 29)) return hipErrorInvalidValue;
    const JoinLayout L = layout(d_work, n);
    hipError_t e = join_bound(d_TG, d_TS, n, L.sel, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(fronts_caps_bound_kernel, dim3(1), dim3(64), 0, st, L.sel, F, margin, chk);
    return hipGetLastError();
}

hipError_t fronts_clean(double* d_T, int64_t n, FrontsCheck* chk, hipStream_t st) {
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(kPassBlocks, (2 * n + 255) / 256));
    hipLaunchKernelGGL(cap_clean_kernel, dim3(grid), dim3(256), 0, st, d_T, n, chk);
    return hipGetLastError();
}

size_t bidir_join_work_bytes(int64_t n) { return layout(nullptr, n).total; }

// the join's pop ranks per front (after bidir_join on d_work): UINT_MAX for cells not ranked
void bidir_join_ranks(const void* d_work, int64_t n, const unsigned** rg, const unsigned** rs) {
    const JoinLayout L = layout(const_cast<void*>(d_work), n);
    *rg = L.rg;
    *rs = L.rs;
}

// the packed join of two rank arrays (join_min_kernel) into *d_best (set to ~0 first by the caller)
hipError_t bidir_join_min(const unsigned* d_rg, const unsigned* d_rs, int64_t n, unsigned long long* d_best,
                          hipStream_t st) {
    const unsigned jgrid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(kPassBlocks, (n + 255) / 256));
    hipLaunchKernelGGL(join_min_kernel, dim3(jgrid), dim3(256), 0, st, d_rg, d_rs, n, d_best);
    return hipGetLastError();
}

// the band relaxation's band cells and sweeps per front (after bidir_partial with a cost)
hipError_t bidir_band_stats(const void* d_work, int64_t n, unsigned out[4], hipStream_t st) {
    const JoinLayout L = layout(const_cast<void*>(d_work), n);
    hipError_t e = hipMemcpyAsync(out, L.sel->nb, 2 * sizeof(unsigned), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMemcpyAsync(out + 2, L.sel->sweeps, 2 * sizeof(unsigned), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    return e;
}

}  // namespace eik
