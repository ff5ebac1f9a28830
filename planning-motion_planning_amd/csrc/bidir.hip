// bidir.hip -- nodeJoin of biComputeTmap (FastMarching.py:114-162) from two full fields.
//
// The reference advances a goal front and a start front one pop each per iteration and stops
// at iteration k when the goal front's k-th pop g_k is already closed by the start front
// (rankS(g_k) <= k, :150-152) or the start front's k-th pop s_k is closed by the goal front
// (rankG(s_k) <= k, :153-155).  A front pops nodes in increasing T, so with
//     rankG(n) = position of n in ascending TG,  rankS(n) = position in ascending TS
// the stopping iteration is k* = min_n max(rankG(n), rankS(n)), and the join is g_{k*} when it
// qualifies (the G test runs first), else s_{k*}.  Ranks come from two device radix sorts of
// the fields' bit patterns (non-negative IEEE doubles sort as unsigned integers); ties of
// exactly equal T are ranked by node index (the reference breaks them LIFO by insertion time,
// which a field does not record -- SURVEY.md §7 "join approximated").
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "eik_common.hpp"

namespace eik {

__global__ void iota_keys_kernel(const double* __restrict__ T, int64_t n, unsigned long long* __restrict__ keys,
                                 unsigned* __restrict__ idx) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    keys[i] = (unsigned long long)__double_as_longlong(T[i]);
    idx[i] = (unsigned)i;
}

// rank[sorted_idx[k]] = k for finite entries, UINT_MAX for unreached (never popped) ones
__global__ void scatter_rank_kernel(const unsigned long long* __restrict__ skeys, const unsigned* __restrict__ sidx,
                                    int64_t n, unsigned* __restrict__ rank) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const bool fin = skeys[k] < 0x7FF0000000000000ull;
    rank[sidx[k]] = fin ? (unsigned)k : 0xFFFFFFFFu;
}

// packed = (2*max(rG,rS) + (rG == max ? 0 : 1)) << 29 | node ; the min identifies the join.
// Grid-stride over the cells, a wave then a workgroup (LDS) minimum, ONE atomicMin per workgroup:
// one atomic per wave on the single result word serialised ~260k device-scope atomics for a
// 4096^2 raster (2.98 ms, tools/rover_probe.py under rocprofv3).
constexpr int kJoinBlocks = 1024;
__global__ __launch_bounds__(256) void join_min_kernel(const unsigned* __restrict__ rg, const unsigned* __restrict__ rs,
                                                       int64_t n, unsigned long long* __restrict__ best) {
    __shared__ unsigned long long wmin[4];
    unsigned long long v = ~0ull;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const unsigned a = rg[i], b = rs[i];
        if (a != 0xFFFFFFFFu && b != 0xFFFFFFFFu) {
            const unsigned long long m = a > b ? a : b;
            const unsigned long long c = ((2ull * m + (a == m ? 0ull : 1ull)) << 29) | (unsigned long long)i;
            v = c < v ? c : v;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(v, off, 64);
        v = o < v ? o : v;
    }
    if ((threadIdx.x & 63) == 0) wmin[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long m = wmin[0];
        for (int w = 1; w < 4; ++w) m = wmin[w] < m ? wmin[w] : m;
        if (m != ~0ull) atomicMin(best, m);
    }
}

struct JoinScratch {
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
};

// d_TG/d_TS: n doubles; d_work must hold 2n u64 + 4n u32 (+ cub scratch appended by caller).
hipError_t bidir_join(const double* d_TG, const double* d_TS, int64_t n, void* d_work, size_t work_bytes,
                      unsigned long long* d_best, hipStream_t st) {
    if (n >= (1ll << 29)) return hipErrorInvalidValue;
    char* p = static_cast<char*>(d_work);
    auto* k_in = reinterpret_cast<unsigned long long*>(p);
    auto* k_out = k_in + n;
    auto* i_in = reinterpret_cast<unsigned*>(k_out + n);
    auto* i_out = i_in + n;
    auto* rg = i_out + n;
    auto* rs = rg + n;
    char* cub_tmp = reinterpret_cast<char*>(rs + n);
    const size_t used = (size_t)(cub_tmp - p);
    size_t cub_bytes = 0;
    hipError_t e1 = hipcub::DeviceRadixSort::SortPairs(nullptr, cub_bytes, k_in, k_out, i_in, i_out, (int)n, 0, 64, st);
    if (e1 != hipSuccess) return e1;
    if (used + cub_bytes > work_bytes) return hipErrorOutOfMemory;
    const unsigned grid = (unsigned)((n + 255) / 256);
    for (int f = 0; f < 2; ++f) {
        hipLaunchKernelGGL(iota_keys_kernel, dim3(grid), dim3(256), 0, st, f == 0 ? d_TG : d_TS, n, k_in, i_in);
        hipError_t e = hipcub::DeviceRadixSort::SortPairs(cub_tmp, cub_bytes, k_in, k_out, i_in, i_out, (int)n, 0, 64, st);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(scatter_rank_kernel, dim3(grid), dim3(256), 0, st, k_out, i_out, n, f == 0 ? rg : rs);
    }
    hipError_t e0 = hipMemsetAsync(d_best, 0xFF, sizeof(unsigned long long), st);
    if (e0 != hipSuccess) return e0;
    const unsigned jgrid = (unsigned)std::min<int64_t>(kJoinBlocks, (n + 255) / 256);
    hipLaunchKernelGGL(join_min_kernel, dim3(jgrid), dim3(256), 0, st, rg, rs, n, d_best);
    return hipGetLastError();
}

// biComputeTmap returns the PARTIAL fields of the two fronts at the meeting iteration k
// (FastMarching.py:141-162): front f has popped its source and the next k nodes, i.e. the cells of
// rank <= k in its field (rank 0 = the source).  Those keep their final values; a cell of the
// narrow band (finite, not popped, a popped 4-neighbour) keeps its value too -- the reference's
// tentative band value is >= the final value, equal when its last update saw final neighbours,
// and the paths descended from nodeJoin (:1225-1226) then match the reference's
// (tests/test_gpu_path.py); every other cell is +inf, as the reference leaves it.  In place: a
// cell's own value changes only to +inf, its neighbours' closedness comes from the ranks.
__global__ void bidir_partial_kernel(double* __restrict__ T, const unsigned* __restrict__ rank, int64_t H, int64_t W,
                                     const unsigned long long* __restrict__ best) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long b = *best;
    if (i >= H * W || b == ~0ull) return;  // fronts never met: the reference raises, fields unused
    const unsigned k = (unsigned)(b >> 30);
    if (rank[i] <= k) return;
    const int64_t y = i / W, x = i - y * W;
    const bool band = (x > 0 && rank[i - 1] <= k) || (x + 1 < W && rank[i + 1] <= k) ||
                      (y > 0 && rank[i - W] <= k) || (y + 1 < H && rank[i + W] <= k);
    if (!band) T[i] = Real<double>::inf();
}

hipError_t bidir_partial(double* d_TG, double* d_TS, int64_t H, int64_t W, const void* d_work,
                         const unsigned long long* d_best, hipStream_t st) {
    const int64_t n = H * W;
    const char* p = static_cast<const char*>(d_work);
    const unsigned* rg = reinterpret_cast<const unsigned*>(p + (size_t)n * (2 * 8 + 2 * 4));
    const unsigned* rs = rg + n;
    const unsigned grid = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(bidir_partial_kernel, dim3(grid), dim3(256), 0, st, d_TG, rg, H, W, d_best);
    hipLaunchKernelGGL(bidir_partial_kernel, dim3(grid), dim3(256), 0, st, d_TS, rs, H, W, d_best);
    return hipGetLastError();
}

size_t bidir_join_work_bytes(int64_t n) {
    size_t cub_bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, cub_bytes, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                       (unsigned*)nullptr, (unsigned*)nullptr, (int)n, 0, 64, (hipStream_t)0);
    return (size_t)n * (2 * 8 + 4 * 4) + cub_bytes + 256;
}

}  // namespace eik
