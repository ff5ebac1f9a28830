// fim2d.hip -- block Fast Iterative Method for the 2D Eikonal cost-to-go (gfx950 / CDNA4).
//
// Replaces the reference's sequential Fast Marching wavefront (FastMarching.py:44-162: a
// Python narrow band kept sorted with bisect) by a tile-parallel FIM whose fixed point is the
// same discrete Godunov solution (the reference FMM equals the
// Jacobi fixed point to 1e-13):
//
//  * the raster is cut into 64x64 tiles; an ACTIVE LIST of tiles is kept on the device;
//  * one workgroup (4 x wave64) per active tile stages cost + T (+1-cell halo) in LDS and runs
//    ONE round of four concurrent quadrant sweeps (one per wave).  Each sweep is Gauss-Seidel
//    along skewed anti-diagonals (lane l = column, step s = row s-l), so the upstream x value
//    comes from lane l-1 through a DPP wave shift and the upstream y value from the lane's own
//    previous step: one round propagates any characteristic in that quadrant across the tile;
//  * updates are monotone min-updates (T = min(T, godunov(...))) merged with ds_min, so the
//    racing waves and the stale halos of concurrently processed tiles are all benign;
//  * a tile whose values changed re-enqueues itself; a tile whose boundary row/column changed
//    enqueues that neighbour (dedup by a per-tile mark, appended with one atomic per tile);
//  * the host runs outer iterations (one launch each) until the list is empty.
//
// The same kernel serves B independent maps (tile id = map * tiles_per_map + tile) and a
// subdomain of a domain-decomposed raster (ghost strips N/S/W/E read in place of the
// out-of-range neighbours; edge-row changes are flagged for the halo exchange).
#include "eik_common.hpp"
#include "eik_kernels.hpp"

namespace eik {

template <typename R>
__device__ __forceinline__ R load_T(const Fim2dArgs& a, const R* __restrict__ T, int64_t gy, int64_t gx) {
    constexpr R INF = Real<R>::inf();
    if (gy >= 0 && gy < a.H && gx >= 0 && gx < a.W) return T[gy * a.W + gx];
    if (gy == -1 && gx >= 0 && gx < a.W) return a.ghost[0] ? static_cast<const R*>(a.ghost[0])[gx] : INF;
    if (gy == a.H && gx >= 0 && gx < a.W) return a.ghost[1] ? static_cast<const R*>(a.ghost[1])[gx] : INF;
    if (gx == -1 && gy >= 0 && gy < a.H) return a.ghost[2] ? static_cast<const R*>(a.ghost[2])[gy] : INF;
    if (gx == a.W && gy >= 0 && gy < a.H) return a.ghost[3] ? static_cast<const R*>(a.ghost[3])[gy] : INF;
    return INF;
}

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

// One quadrant sweep of the staged tile.  DX/DY = +-1: direction of propagation.
// Lane l owns column x; at step s it updates row r = s - l (skewed Gauss-Seidel), so its
// upstream x neighbour is lane l-1's previous result (DPP) and its upstream y neighbour its own.
// Branch- and select-free: r is clamped to [-1, 64]; rows -1 and 64 are the halo rows, whose
// cost is +inf in Cs (same 66-stride layout as Ts), so a lane outside the tile computes +inf or
// NaN and its ds_min / min / `<` are no-ops.  Every LDS access of a step shares one address.
template <typename R, int DX, int DY>
__device__ __forceinline__ bool sweep_quadrant(R* __restrict__ Ts, const R* __restrict__ Cs, int lane, R keep) {
    const int x = DX > 0 ? lane : kTile - 1 - lane;
    const int col = x + 1;
    bool changed = false;

    auto addr = [&](int s) {
        int r = s - lane;
        r = r < -1 ? -1 : (r > kTile ? kTile : r);
        const int lr = DY > 0 ? r + 1 : kTile - r;  // LDS row 0..65
        return lr * kLds + col;
    };
    // the upstream halo row value is the lane's "previous row" result before it starts
    R cur = Ts[(DY > 0 ? 0 : kLds - 1) * kLds + col];
    int o = addr(0);
    R p_old = Ts[o], p_dnx = Ts[o + DX], p_dny = Ts[o + DY * kLds], p_upx = Ts[o - DX], p_c = Cs[o];
#pragma clang loop unroll_count(2)
    for (int s = 0; s < 2 * kTile; ++s) {
        const R old = p_old, dnx = p_dnx, dny = p_dny, uxh = p_upx, c = p_c;
        const int oc = o;
        o = addr(s + 1);  // next step's loads issue before this step's ds_min (no intra-wave RAW)
        p_old = Ts[o];
        p_dnx = Ts[o + DX];
        p_dny = Ts[o + DY * kLds];
        p_upx = Ts[o - DX];
        p_c = Cs[o];
        const R upx = wave_shr1(cur, uxh);  // lane 0: halo column
        const R a = umin(upx, dnx);
        const R b = umin(cur, dny);
        const R w = godunov2_step(a, b, c);
        lds_min(&Ts[oc], w);
        changed |= w < old * keep;
        cur = umin(w, old);  // NaN (both-inf case) sorts above every value: keeps old
    }
    return changed;
}

template <typename R>
__global__ __launch_bounds__(kThreads) void fim2d_sweep_kernel(Fim2dArgs a) {
    constexpr R INF = Real<R>::inf();
    // Ts: tile + halo ring, plus one guard row above and below (the clamped r = -1 / 64 steps
    // read one row beyond the halo: in-bounds, +inf, and masked by the +inf halo cost anyway)
    __shared__ R Tbuf[(kLds + 2) * kLds];
    __shared__ R Cs[kLds * kLds];  // same layout as Ts; halo ring = +inf
    R* const Ts = Tbuf + kLds;
    __shared__ unsigned s_round, s_flags;
    __shared__ unsigned s_key[5];  // min new value: self, N, S, W, E (f32 bits)
    __shared__ int s_defer;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < kLds) {
        Tbuf[tid] = INF;
        Tbuf[(kLds + 1) * kLds + tid] = INF;
    }
    const int cur = a.iter % 3, nxt = (a.iter + 1) % 3, rst = (a.iter + 2) % 3;
    const int cnt = a.counts[cur];
    if (blockIdx.x == 0 && tid == 0) {
        a.counts[rst] = 0;
        a.minkey[rst] = 0x7f800000u;
    }
    const unsigned stamp = a.iter + 2;  // "enqueued for iteration iter+1"
    const float thr = __uint_as_float(a.minkey[cur]) + a.delta;  // ordering window of this launch
    const R keep = (R)a.keep;

    for (int it = blockIdx.x; it < cnt; it += gridDim.x) {
        const int tile = a.lists[(int64_t)cur * a.capacity + it];
        if (a.delta < INF) {  // ordered mode: defer tiles whose entering T is beyond the window
            if (tid == 0) {
                const float k = __uint_as_float(atomicOr(&a.key[tile], 0u));
                s_defer = k > thr;
                if (k > thr) enqueue(a, tile, nxt, stamp, k);
                else atomicExch(&a.key[tile], 0x7f800000u);  // entering values count afresh
            }
            __syncthreads();
            const bool defer = s_defer;
            __syncthreads();
            if (defer) continue;  // uniform across the workgroup
        }
        const int map = tile / a.tiles_per_map;
        const int rem = tile - map * a.tiles_per_map;
        const int ty = rem / a.ntx, tx = rem - (rem / a.ntx) * a.ntx;
        const R* __restrict__ cost = static_cast<const R*>(a.cost) + (int64_t)map * a.H * a.W;
        R* __restrict__ T = static_cast<R*>(a.T) + (int64_t)map * a.H * a.W;
        const int64_t y0 = (int64_t)ty * kTile, x0 = (int64_t)tx * kTile;
        const bool full = (y0 + kTile <= a.H) && (x0 + kTile <= a.W) && ((a.W & 3) == 0);

        if (tid == 0) {
            s_round = 0;
            s_flags = 0;
        }
        if (tid < 5) s_key[tid] = 0x7f800000u;
        // ---- stage the tile: 16 cells per thread (4 rows x 4 consecutive columns)
        R told[16];
        const int cx = (tid & 15) * 4;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int ry = (tid >> 4) + 16 * k;
            const int64_t gy = y0 + ry;
            if (full) {
                if constexpr (sizeof(R) == 4) {
                    const float4 t4 = *reinterpret_cast<const float4*>(&T[gy * a.W + x0 + cx]);
                    const float4 c4 = *reinterpret_cast<const float4*>(&cost[gy * a.W + x0 + cx]);
                    told[4 * k + 0] = t4.x; told[4 * k + 1] = t4.y; told[4 * k + 2] = t4.z; told[4 * k + 3] = t4.w;
                    R* cr = &Cs[(ry + 1) * kLds + cx + 1];
                    cr[0] = c4.x; cr[1] = c4.y; cr[2] = c4.z; cr[3] = c4.w;
                } else {
                    const double2 t0 = *reinterpret_cast<const double2*>(&T[gy * a.W + x0 + cx]);
                    const double2 t1 = *reinterpret_cast<const double2*>(&T[gy * a.W + x0 + cx + 2]);
                    const double2 c0 = *reinterpret_cast<const double2*>(&cost[gy * a.W + x0 + cx]);
                    const double2 c1 = *reinterpret_cast<const double2*>(&cost[gy * a.W + x0 + cx + 2]);
                    told[4 * k + 0] = t0.x; told[4 * k + 1] = t0.y; told[4 * k + 2] = t1.x; told[4 * k + 3] = t1.y;
                    R* cr = &Cs[(ry + 1) * kLds + cx + 1];
                    cr[0] = c0.x; cr[1] = c0.y; cr[2] = c1.x; cr[3] = c1.y;
                }
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int64_t gx = x0 + cx + e;
                    const bool in = gy < a.H && gx < a.W;
                    told[4 * k + e] = load_T<R>(a, T, gy, gx);  // ghost cells land in padding
                    Cs[(ry + 1) * kLds + cx + e + 1] = in ? cost[gy * a.W + gx] : INF;
                }
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) Ts[(ry + 1) * kLds + cx + e + 1] = told[4 * k + e];
        }
        // halo ring: wave 0 north row, 1 south row, 2 west column, 3 east column
        {
            R v;
            if (wave == 0)      v = load_T<R>(a, T, y0 - 1, x0 + lane);
            else if (wave == 1) v = load_T<R>(a, T, y0 + kTile, x0 + lane);
            else if (wave == 2) v = load_T<R>(a, T, y0 + lane, x0 - 1);
            else                v = load_T<R>(a, T, y0 + lane, x0 + kTile);
            int h;
            if (wave == 0)      h = 0 * kLds + lane + 1;
            else if (wave == 1) h = (kLds - 1) * kLds + lane + 1;
            else if (wave == 2) h = (lane + 1) * kLds + 0;
            else                h = (lane + 1) * kLds + kLds - 1;
            Ts[h] = v;
            Cs[h] = INF;
            if (lane < 4) Cs[(lane >> 1) * (kLds - 1) * kLds + (lane & 1) * (kLds - 1)] = INF;  // corners
        }
        __syncthreads();

        // ---- sweep rounds (4 quadrant directions concurrently, one per wave)
        bool last_changed = false;
        for (int round = 0;; ++round) {
            bool ch;
            if (wave == 0)      ch = sweep_quadrant<R, +1, +1>(Ts, Cs, lane, keep);
            else if (wave == 1) ch = sweep_quadrant<R, -1, +1>(Ts, Cs, lane, keep);
            else if (wave == 2) ch = sweep_quadrant<R, +1, -1>(Ts, Cs, lane, keep);
            else                ch = sweep_quadrant<R, -1, -1>(Ts, Cs, lane, keep);
            if (__any(ch) && lane == 0) atomicOr(&s_round, 1u << (round & 31));
            __syncthreads();
            last_changed = (s_round >> (round & 31)) & 1u;
            if (!last_changed || round + 1 >= a.max_rounds) break;
        }

        // ---- write back changed cells, collect side flags and the smallest entering values
        unsigned fl = 0;
        R kmin_self = INF, kmin[4] = {INF, INF, INF, INF};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int ry = (tid >> 4) + 16 * k;
            const int64_t gy = y0 + ry;
            R nv[4];
            bool any = false;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                nv[e] = Ts[(ry + 1) * kLds + cx + e + 1];
                const bool chg = nv[e] < told[4 * k + e];
                any |= chg;
                if (nv[e] < told[4 * k + e] * keep) {
                    kmin_self = umin(kmin_self, nv[e]);
                    // A neighbour can only improve if this edge value undercuts the neighbour's
                    // adjacent cell (the halo value, stale => larger => conservative).
                    const int lx = cx + e + 1, ly = ry + 1;
#ifdef EIK_NO_FILTER
                    if (ry == 0) fl |= 1u;
                    if (ry == kTile - 1) fl |= 2u;
                    if (cx + e == 0) fl |= 4u;
                    if (cx + e == kTile - 1) fl |= 8u;
#else
                    if (ry == 0 && nv[e] < Ts[lx]) { fl |= 1u; kmin[0] = umin(kmin[0], nv[e]); }
                    if (ry == kTile - 1 && nv[e] < Ts[(kLds - 1) * kLds + lx]) { fl |= 2u; kmin[1] = umin(kmin[1], nv[e]); }
                    if (cx + e == 0 && nv[e] < Ts[ly * kLds]) { fl |= 4u; kmin[2] = umin(kmin[2], nv[e]); }
                    if (cx + e == kTile - 1 && nv[e] < Ts[ly * kLds + kLds - 1]) { fl |= 8u; kmin[3] = umin(kmin[3], nv[e]); }
#endif
                    const int64_t gx = x0 + cx + e;                     // subdomain edges (DD)
                    if (gy == a.H - 1 && ry != kTile - 1) fl |= 32u;
                    if (gx == a.W - 1 && cx + e != kTile - 1) fl |= 64u;
                }
            }
            if (any) {
                if (full) {
                    if constexpr (sizeof(R) == 4) {
                        *reinterpret_cast<float4*>(&T[gy * a.W + x0 + cx]) = make_float4(nv[0], nv[1], nv[2], nv[3]);
                    } else {
                        *reinterpret_cast<double2*>(&T[gy * a.W + x0 + cx]) = make_double2(nv[0], nv[1]);
                        *reinterpret_cast<double2*>(&T[gy * a.W + x0 + cx + 2]) = make_double2(nv[2], nv[3]);
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int64_t gx = x0 + cx + e;
                        if (gy < a.H && gx < a.W && nv[e] < told[4 * k + e]) T[gy * a.W + gx] = nv[e];
                    }
                }
            }
        }
        if (fl) atomicOr(&s_flags, fl);
        if (kmin_self < INF) atomicMin(&s_key[0], __float_as_uint((float)kmin_self));
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (kmin[q] < INF) atomicMin(&s_key[q + 1], __float_as_uint((float)kmin[q]));
        __syncthreads();
        if (tid < 5) {  // up to 5 enqueues, one per lane, so their atomics overlap
            const unsigned f = s_flags;
            const int base = map * a.tiles_per_map;
            const float kk = __uint_as_float(s_key[tid]);
            if (tid == 0 && last_changed) enqueue(a, tile, nxt, stamp, kk);
            if (tid == 1 && (f & 1u) && ty > 0) enqueue(a, base + rem - a.ntx, nxt, stamp, kk);
            if (tid == 2 && (f & 2u) && ty + 1 < a.nty) enqueue(a, base + rem + a.ntx, nxt, stamp, kk);
            if (tid == 3 && (f & 4u) && tx > 0) enqueue(a, base + rem - 1, nxt, stamp, kk);
            if (tid == 4 && (f & 8u) && tx + 1 < a.ntx) enqueue(a, base + rem + 1, nxt, stamp, kk);
            if (tid == 0 && a.edge_dirty) {  // subdomain edges (domain decomposition)
                unsigned e = 0;
                if ((f & 1u) && ty == 0) e |= 1u;
                if (((f & 2u) || (f & 32u)) && ty + 1 == a.nty) e |= 2u;
                if ((f & 4u) && tx == 0) e |= 4u;
                if (((f & 8u) || (f & 64u)) && tx + 1 == a.ntx) e |= 8u;
                if (e) atomicOr(a.edge_dirty, e);
            }
            if (tid == 0 && a.visits) atomicAdd(a.visits, 1ull);
        }
        __syncthreads();  // LDS reuse by the next tile of this workgroup
    }
}

// T = inf everywhere; T[goal] = 0; marks cleared.  Goals: one per map (gx < 0: none).
template <typename R>
__global__ void fim2d_init_kernel(R* __restrict__ T, int64_t n, unsigned* __restrict__ mark, int64_t ntiles,
                                  unsigned* __restrict__ key, unsigned* __restrict__ minkey) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) T[i] = Real<R>::inf();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ntiles; i += stride) {
        mark[i] = 0;
        key[i] = 0x7f800000u;
    }
    if (blockIdx.x == 0 && threadIdx.x < 3) minkey[threadIdx.x] = threadIdx.x == 0 ? 0u : 0x7f800000u;
}

template <typename R>
__global__ void fim2d_seed_kernel(Fim2dArgs a, const int64_t* __restrict__ goals, int nmaps) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m == 0) {
        a.counts[1] = 0;
        a.counts[2] = 0;
    }
    if (m >= nmaps) return;
    const int64_t gx = goals[2 * m], gy = goals[2 * m + 1];
    if (gx < 0 || gy < 0 || gx >= a.W || gy >= a.H) return;
    static_cast<R*>(a.T)[(int64_t)m * a.H * a.W + gy * a.W + gx] = R(0);
    const int tile = m * a.tiles_per_map + (int)(gy / kTile) * a.ntx + (int)(gx / kTile);
    a.mark[tile] = 1;  // enqueued for iteration 0
    a.key[tile] = 0u;  // T = 0 enters at the goal
    const int pos = atomicAdd(&a.counts[0], 1);
    a.lists[pos] = tile;
}

// Domain decomposition: ghost = min(ghost, recv) and enqueue (for iteration `iter`) every edge
// tile next to a ghost cell that decreased.  side: 0 N, 1 S, 2 W, 3 E.
template <typename R>
__global__ void fim2d_merge_ghost_kernel(Fim2dArgs a, int side, const R* __restrict__ recv, int64_t len) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= len) return;
    R* g = static_cast<R*>(const_cast<void*>(a.ghost[side]));
    const R v = recv[i];
    if (v < g[i]) {
        g[i] = v;
        int ty, tx;
        if (side < 2) {
            tx = (int)(i / kTile);
            ty = side == 0 ? 0 : a.nty - 1;
        } else {
            ty = (int)(i / kTile);
            tx = side == 2 ? 0 : a.ntx - 1;
        }
        enqueue(a, ty * a.ntx + tx, a.iter % 3, a.iter + 1, (float)v);
    }
}

// Copy this subdomain's edge rows/columns of T into contiguous send strips.
template <typename R>
__global__ void fim2d_pack_edges_kernel(Fim2dArgs a, R* __restrict__ n, R* __restrict__ s, R* __restrict__ w,
                                        R* __restrict__ e) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const R* T = static_cast<const R*>(a.T);
    if (i < a.W) {
        if (n) n[i] = T[i];
        if (s) s[i] = T[(a.H - 1) * a.W + i];
    }
    if (i < a.H) {
        if (w) w[i] = T[i * a.W];
        if (e) e[i] = T[i * a.W + a.W - 1];
    }
}

// ------------------------------------------------------------------------- host launchers
template <typename R>
static hipError_t launch_sweep(const Fim2dArgs& a, int grid, hipStream_t st) {
    hipLaunchKernelGGL(fim2d_sweep_kernel<R>, dim3(grid), dim3(kThreads), 0, st, a);
    return hipGetLastError();
}

hipError_t fim2d_sweep(const Fim2dArgs& a, bool f64, int grid, hipStream_t st) {
    return f64 ? launch_sweep<double>(a, grid, st) : launch_sweep<float>(a, grid, st);
}

hipError_t fim2d_init(const Fim2dArgs& a, bool f64, int nmaps, const int64_t* d_goals, hipStream_t st) {
    const int64_t n = (int64_t)nmaps * a.H * a.W;
    const int64_t ntiles = (int64_t)nmaps * a.tiles_per_map;
    const int grid = (int)std::min<int64_t>(4096, (n + 255) / 256);
    hipError_t e0 = hipMemsetAsync(a.counts, 0, sizeof(int) * 4, st);
    if (e0 != hipSuccess) return e0;
    if (f64) {
        hipLaunchKernelGGL(fim2d_init_kernel<double>, dim3(grid), dim3(256), 0, st, static_cast<double*>(a.T), n,
                           a.mark, ntiles, a.key, a.minkey);
        hipLaunchKernelGGL(fim2d_seed_kernel<double>, dim3((nmaps + 255) / 256), dim3(256), 0, st, a, d_goals, nmaps);
    } else {
        hipLaunchKernelGGL(fim2d_init_kernel<float>, dim3(grid), dim3(256), 0, st, static_cast<float*>(a.T), n,
                           a.mark, ntiles, a.key, a.minkey);
        hipLaunchKernelGGL(fim2d_seed_kernel<float>, dim3((nmaps + 255) / 256), dim3(256), 0, st, a, d_goals, nmaps);
    }
    return hipGetLastError();
}

hipError_t fim2d_merge_ghost(const Fim2dArgs& a, bool f64, int side, const void* recv, int64_t len, hipStream_t st) {
    const int grid = (int)((len + 255) / 256);
    if (f64)
        hipLaunchKernelGGL(fim2d_merge_ghost_kernel<double>, dim3(grid), dim3(256), 0, st, a, side,
                           static_cast<const double*>(recv), len);
    else
        hipLaunchKernelGGL(fim2d_merge_ghost_kernel<float>, dim3(grid), dim3(256), 0, st, a, side,
                           static_cast<const float*>(recv), len);
    return hipGetLastError();
}

hipError_t fim2d_pack_edges(const Fim2dArgs& a, bool f64, void* n, void* s, void* w, void* e, hipStream_t st) {
    const int64_t len = a.H > a.W ? a.H : a.W;
    const int grid = (int)((len + 255) / 256);
    if (f64)
        hipLaunchKernelGGL(fim2d_pack_edges_kernel<double>, dim3(grid), dim3(256), 0, st, a, (double*)n, (double*)s,
                           (double*)w, (double*)e);
    else
        hipLaunchKernelGGL(fim2d_pack_edges_kernel<float>, dim3(grid), dim3(256), 0, st, a, (float*)n, (float*)s,
                           (float*)w, (float*)e);
    return hipGetLastError();
}

}  // namespace eik
