// fim3d.hip -- block FIM for the 3D (x, y, z) Eikonal of FastMarching3D.py on gfx950.
//
// Reference: FastMarching3D.py:19-145 (updateNode with the 6-neighbour "drop the largest"
// n-D Godunov solve, :59-75; sorted-list narrow band; computeTmap driver).  Layout follows the
// reference: cost[y][x][z] row-major (z fastest), nodes (x, y, z).
//
// Tiles are TX x TY x TZ boxes of <= 1024 cells chosen per volume (16x16xL for the planner's
// thin layered volumes, 8x16x8 for cubes).  A 256-thread workgroup stages the box + a 1-cell
// halo in LDS and relaxes it in place (every thread owns up to 4 cells; chaotic relaxation is
// monotone, so it converges to the same fixed point) until a pass changes nothing or the pass
// budget runs out, then writes back and activates the face neighbours whose halo its new face
// values undercut -- the same active-list / mark machinery as fim2d.hip.
#include "fim_engine.hpp"

namespace eik {

// FastMarching3D.py:59-75: try all three axes, drop the largest while the n-axis solution does
// not exceed it (C^2 > sum (Tmax - Ti)^2 is the reference's acceptance test).
template <typename R>
__device__ __forceinline__ R godunov3(R a, R b, R c, R C) {
    // sort ascending
    R t;
    if (a > b) { t = a; a = b; b = t; }
    if (b > c) { t = b; b = c; c = t; }
    if (a > b) { t = a; a = b; b = t; }
    // Solutions written relative to the smallest neighbour (b' = b - a, c' = c - a):
    // (S + sqrt(nC^2 + S^2 - nQ)) / n of the reference equals a + (S' + sqrt(nC^2 - (nQ' - S'^2)))/n
    // with nQ' - S'^2 = 2(b'^2 + c'^2 - b'c') for n = 3 -- no cancellation of the large T values
    // (the reference's form loses ~1e-4 relative in fp32 at T ~ 300).
    const R C2 = C * C;
    const R bp = b - a, cp = c - a;
    if (c != Real<R>::inf() && C2 > cp * cp + (c - b) * (c - b)) {
        return a + (bp + cp + __builtin_sqrt(R(3) * C2 - R(2) * (bp * bp + cp * cp - bp * cp))) / R(3);
    }
    if (b != Real<R>::inf() && C2 > bp * bp) {
        return a + (bp + __builtin_sqrt(R(2) * C2 - bp * bp)) / R(2);
    }
    return a + C;
}

// (solve3_ref, the reference's FastMarching3D.py:59-75 in its own arithmetic: eik_common.hpp)

// the solver's local update: the reference's arithmetic in fp64, the cancellation-free form in fp32
template <typename R>
__device__ __forceinline__ R local3(R a, R b, R c, R C) {
    if constexpr (sizeof(R) == 8) return solve3_ref(a, b, c, C);
    else return godunov3<R>(a, b, c, C);
}

__device__ __forceinline__ void enqueue3(const Fim3dArgs& a, int tile, int list, unsigned stamp) {
    if (atomicMax(&a.mark[tile], stamp) < stamp) {
        const int pos = atomicAdd(&a.counts[list], 1);
        a.lists[(int64_t)list * a.capacity + pos] = tile;
    }
}

#ifndef EIK_FIM3D_ALT
#define EIK_FIM3D_ALT 0
#endif
constexpr int kMaxCells3 = 1024;
constexpr int kMaxHalo3 = 18 * 18 * 10;  // (TX+2)(TY+2)(TZ+2) bound for the tile shapes used

// LDS of one 3D tile visit
template <typename R>
struct TileLds3 {
    R Ts[kMaxHalo3];
    R Cs[kMaxCells3];
    unsigned flags;   // bits 0..5: face x-, x+, y-, y+, z-, z+ neighbour can improve; 128: the
                      // last relaxation pass changed the tile (pass cap reached: revisit)
    int changed[3];   // triple-buffered by pass: reset two barriers after the last read
    int tile;
    int passes;       // relaxation passes of the last visit (stats)
};

// The early-exit bound (see Fim3dArgs::stop_off): T[start] only decreases, so a stale read only
// prunes less; every cell whose final value is <= the final bound is still reached exactly (its
// upstream cells have smaller values), and nothing above it is kept by the early exit.
template <typename R, bool COH>
__device__ __forceinline__ R early_bound(const Fim3dArgs& a) {
    if (a.stop_off < 0) return Real<R>::inf();
    const R* T = static_cast<const R*>(a.T);
    const R ts = COH ? ld_agent(T + a.stop_off) : T[a.stop_off];
    return (ts + *static_cast<const R*>(a.stop_slack)) * R(1.000001);
}

// Stage one TX x TY x TZ tile + 1-cell halo in LDS, relax it in place (every thread owns up to 4
// cells; chaotic relaxation is monotone, so it converges to the same fixed point) until a pass
// changes nothing or a.max_passes ran, write the lowered cells back and leave the face flags in
// L.flags.  COH (persistent driver): T is read with sc1 loads and written with sc1 stores, every
// storing wave drains before the closing barrier (fim2d.hip's memory-model recipe), so the
// caller's activations publish the new faces.  Ends with a workgroup barrier.
template <typename R, bool COH>
__device__ __forceinline__ void process_tile3(const Fim3dArgs& a, int tile, TileLds3<R>& L, R bound) {
    constexpr R INF = Real<R>::inf();
    const int tid = threadIdx.x;
    const int TX = a.tx, TY = a.ty, TZ = a.tz;
    const int HX = TX + 2, HY = TY + 2, HZ = TZ + 2;  // halo box, index ((y*HX)+x)*HZ+z
    const int ncell = TX * TY * TZ;
    const int vol = tile / a.tpv, rem = tile - vol * a.tpv;  // batch: volume, tile in volume
    const int bz = rem % a.ntz, bxy = rem / a.ntz, bx = bxy % a.ntx, by = bxy / a.ntx;
    const int64_t x0 = (int64_t)bx * TX, y0 = (int64_t)by * TY, z0 = (int64_t)bz * TZ;
    const int64_t voff = (int64_t)vol * a.H * a.W * a.L;
    const R* __restrict__ cost = static_cast<const R*>(a.cost) + voff;
    const TMem<R, COH> T(static_cast<R*>(a.T) + voff, a.H * a.W * a.L);
    if (tid == 0) {
        L.flags = 0;
        L.changed[0] = 0;
        L.changed[1] = 0;
        L.changed[2] = 0;
    }
    // stage the halo box (cells outside the volume read +inf)
    const int nh = HX * HY * HZ;
    for (int i = tid; i < nh; i += 256) {
        const int hz = i % HZ, hxy = i / HZ, hx = hxy % HX, hy = hxy / HX;
        const int64_t gz = z0 + hz - 1, gx = x0 + hx - 1, gy = y0 + hy - 1;
        const bool in = gz >= 0 && gz < a.L && gx >= 0 && gx < a.W && gy >= 0 && gy < a.H;
        const R v = T.ld(in ? (gy * a.W + gx) * a.L + gz : 0);
        L.Ts[i] = in ? v : INF;
    }
    R told[4], cst[4];
    int hidx[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int c = tid + 256 * k;
        hidx[k] = -1;
        cst[k] = INF;
        if (c < ncell) {
            const int cz = c % TZ, cxy = c / TZ, cx = cxy % TX, cy = cxy / TX;
            hidx[k] = ((cy + 1) * HX + (cx + 1)) * HZ + (cz + 1);
            const int64_t gz = z0 + cz, gx = x0 + cx, gy = y0 + cy;
            const bool in = gz < a.L && gx < a.W && gy < a.H;
            cst[k] = in ? cost[(gy * a.W + gx) * a.L + gz] : INF;
            L.Cs[c] = cst[k];
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) told[k] = hidx[k] >= 0 ? L.Ts[hidx[k]] : INF;

    // in-place relaxation passes.  A thread's cells k = 0..3 lie kTY/4 rows apart in y (c = tid +
    // 256 k) and are relaxed in order, so a pass is Gauss-Seidel along y in steps of a quarter tile;
    // EIK_FIM3D_ALT: the order alternates (+y on even passes, -y on odd ones) -- measured and OFF:
    // end-effector full field 1.27 -> 1.55 ms, more passes per visit (profiles/r03o_fim3d_persistent_ab.log)
    bool last = false;
    const int sx = HZ, sy = HX * HZ;
    int pass = 0;
    for (; pass < a.max_passes; ++pass) {
        const int slot = pass % 3;
        bool ch = false;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const int k = (EIK_FIM3D_ALT && (pass & 1)) ? 3 - kk : kk;
            if (hidx[k] < 0) continue;
            const int h = hidx[k];
            const R v = L.Ts[h];
            const R tx_ = fmin(L.Ts[h - sx], L.Ts[h + sx]);
            const R ty_ = fmin(L.Ts[h - sy], L.Ts[h + sy]);
            const R tz_ = fmin(L.Ts[h - 1], L.Ts[h + 1]);
            const R nv = cst[k] == INF ? INF : local3<R>(tx_, ty_, tz_, cst[k]);
            if (nv < v && nv <= bound) {
                L.Ts[h] = nv;  // owner-only write; concurrent readers see old or new (both bounds)
                ch = true;
            }
        }
        if (ch) L.changed[slot] = 1;
        if (tid == 0) L.changed[(pass + 1) % 3] = 0;  // read at pass-2, all past barrier pass-1
        __syncthreads();
        last = L.changed[slot] != 0;
        if (!last) break;
    }
    if (tid == 0) L.passes = pass + (last ? 0 : 1);

    // write back and collect face flags (bit f: face f's neighbour can improve)
    unsigned fl = last ? 128u : 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (hidx[k] < 0) continue;
        const int h = hidx[k];
        const R nv = L.Ts[h];
        if (!(nv < told[k])) continue;
        const int c = tid + 256 * k;
        const int cz = c % TZ, cxy = c / TZ, cx = cxy % TX, cy = cxy / TX;
        const int64_t gz = z0 + cz, gx = x0 + cx, gy = y0 + cy;
        if (gz < a.L && gx < a.W && gy < a.H) T.st((gy * a.W + gx) * a.L + gz, nv);
        if (cx == 0 && nv < L.Ts[h - sx]) fl |= 1u;
        if (cx == TX - 1 && nv < L.Ts[h + sx]) fl |= 2u;
        if (cy == 0 && nv < L.Ts[h - sy]) fl |= 4u;
        if (cy == TY - 1 && nv < L.Ts[h + sy]) fl |= 8u;
        if (cz == 0 && nv < L.Ts[h - 1]) fl |= 16u;
        if (cz == TZ - 1 && nv < L.Ts[h + 1]) fl |= 32u;
    }
    if (fl) atomicOr(&L.flags, fl);
    if constexpr (COH) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
    __syncthreads();
}

// The face neighbour of `tile` across face f (0..5: x-, x+, y-, y+, z-, z+), or -1 at the volume's end.
__device__ __forceinline__ int face_neighbour3(const Fim3dArgs& a, int tile, int f) {
    const int vol = tile / a.tpv, rem = tile - vol * a.tpv;
    const int bz = rem % a.ntz, bxy = rem / a.ntz, bx = bxy % a.ntx, by = bxy / a.ntx;
    switch (f) {
        case 0: return bx > 0 ? tile - a.ntz : -1;
        case 1: return bx + 1 < a.ntx ? tile + a.ntz : -1;
        case 2: return by > 0 ? tile - a.ntx * a.ntz : -1;
        case 3: return by + 1 < a.nty ? tile + a.ntx * a.ntz : -1;
        case 4: return bz > 0 ? tile - 1 : -1;
        default: return bz + 1 < a.ntz ? tile + 1 : -1;
    }
}

// LIST driver: one launch per outer iteration over the active list.
template <typename R>
__global__ __launch_bounds__(256) void fim3d_sweep_kernel(Fim3dArgs a) {
    __shared__ TileLds3<R> L;
    const int tid = threadIdx.x;
    const int cur = a.iter % 3, nxt = (a.iter + 1) % 3, rst = (a.iter + 2) % 3;
    const int cnt = a.counts[cur];
    if (blockIdx.x == 0 && tid == 0) a.counts[rst] = 0;
    const unsigned stamp = a.iter + 2;
    const R bound = early_bound<R, false>(a);
    for (int it = blockIdx.x; it < cnt; it += gridDim.x) {
        const int tile = a.lists[(int64_t)cur * a.capacity + it];
        process_tile3<R, false>(a, tile, L, bound);
        if (tid < 6) {
            const unsigned f = L.flags;
            const int nb = face_neighbour3(a, tile, tid);
            if (((f >> tid) & 1u) && nb >= 0) enqueue3(a, nb, nxt, stamp);
        }
        if (tid == 64) {
            if (L.flags & 128u) enqueue3(a, tile, nxt, stamp);
            if (a.visits) atomicAdd(a.visits, 1ull);
        }
        __syncthreads();
    }
}

// PERSISTENT driver (cf. fim2dl_persist_kernel): one launch per solve; workgroups take tiles from
// the device FIFO of fim_engine.hpp (q carries its queue words; q.visits[0] counts visits, a.visits
// the relaxation passes) and a
// visit's face activations queue the neighbours into the running launch.  A tile whose last pass
// still changed it (pass cap) re-queues itself through its state word, as a busy tile activated by
// a neighbour does; the solve ends when no tile is pending or busy.
template <typename R>
__global__ __launch_bounds__(256) void fim3d_persist_kernel(Fim3dArgs a, Fim2dArgs q) {
    __shared__ TileLds3<R> L;
    int tile = -1;
    unsigned nvis = 0;
    for (;;) {
        if (threadIdx.x < 64) {
            if (tile >= 0) {
                const unsigned f = L.flags;
                if (threadIdx.x < 6) {
                    const int nb = face_neighbour3(a, tile, threadIdx.x);
                    if (((f >> threadIdx.x) & 1u) && nb >= 0) qpush(q, nb, kSelf);
                }
                if (threadIdx.x == 6 && (f & 128u)) atomicOr(&q.qstate[tile], kPending | kSelf);
                // relaxation passes (stats) in the 3D args' counter: q.visits[1] is part of the budget
                if (threadIdx.x == 7 && a.visits) atomicAdd(a.visits, (unsigned long long)L.passes);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
                if (threadIdx.x == 0) {
                    qfinish(q, tile);
                    if (++nvis == 64u) {  // visit cap (negative costs never converge)
                        charge_visits(q, 64ull);
                        nvis = 0;
                    }
                }
            }
        } else if (threadIdx.x == 64) {
            unsigned trig = 0;
            L.tile = qgrab(q, trig);
        }
        __syncthreads();
        tile = __builtin_amdgcn_readfirstlane(L.tile);
        if (tile < 0) break;
        process_tile3<R, true>(a, tile, L, early_bound<R, true>(a));
    }
    if (threadIdx.x == 0 && nvis) atomicAdd(q.visits, (unsigned long long)nvis);
}

template <typename R>
__global__ void fim3d_init_kernel(R* __restrict__ T, int64_t n, unsigned* __restrict__ mark, int64_t ntiles) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) T[i] = Real<R>::inf();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ntiles; i += stride) mark[i] = 0;
}

template <typename R>
__global__ void fim3d_seed_kernel(Fim3dArgs a, const int64_t* __restrict__ goals, int B) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b == 0) {
        a.counts[1] = 0;
        a.counts[2] = 0;
        a.counts[0] = B;
    }
    if (b >= B) return;
    const int64_t gx = goals[3 * b], gy = goals[3 * b + 1], gz = goals[3 * b + 2];
    static_cast<R*>(a.T)[(int64_t)b * a.H * a.W * a.L + (gy * a.W + gx) * a.L + gz] = R(0);
    const int tile = b * a.tpv + ((int)(gy / a.ty) * a.ntx + (int)(gx / a.tx)) * a.ntz + (int)(gz / a.tz);
    a.mark[tile] = 1;
    a.lists[b] = tile;
}

hipError_t fim3d_init(const Fim3dArgs& a, bool f64, const int64_t* d_goals, int B, hipStream_t st) {
    const int64_t n = (int64_t)B * a.H * a.W * a.L;
    const int grid = (int)std::min<int64_t>(4096, (n + 255) / 256);
    const int sg = (B + 255) / 256;
    if (f64) {
        hipLaunchKernelGGL(fim3d_init_kernel<double>, dim3(grid), dim3(256), 0, st, static_cast<double*>(a.T), n,
                           a.mark, (int64_t)a.capacity);
        hipLaunchKernelGGL(fim3d_seed_kernel<double>, dim3(sg), dim3(256), 0, st, a, d_goals, B);
    } else {
        hipLaunchKernelGGL(fim3d_init_kernel<float>, dim3(grid), dim3(256), 0, st, static_cast<float*>(a.T), n,
                           a.mark, (int64_t)a.capacity);
        hipLaunchKernelGGL(fim3d_seed_kernel<float>, dim3(sg), dim3(256), 0, st, a, d_goals, B);
    }
    return hipGetLastError();
}

hipError_t fim3d_sweep(const Fim3dArgs& a, bool f64, int grid, hipStream_t st) {
    if (f64)
        hipLaunchKernelGGL(fim3d_sweep_kernel<double>, dim3(grid), dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL(fim3d_sweep_kernel<float>, dim3(grid), dim3(256), 0, st, a);
    return hipGetLastError();
}

// persistent driver: T = inf, queue state and slots cleared (the host zeroes the control words)
template <typename R>
__global__ void fim3d_pinit_kernel(R* __restrict__ T, int64_t n, unsigned* __restrict__ qstate, int64_t ntiles,
                                   unsigned* __restrict__ qslot, int64_t nslots) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) T[i] = Real<R>::inf();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ntiles; i += stride) qstate[i] = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += stride) qslot[i] = 0;
}

// T[goal of volume b] = 0 and its tile queued
template <typename R>
__global__ void fim3d_pseed_kernel(Fim3dArgs a, Fim2dArgs q, const int64_t* __restrict__ goals, int B) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int64_t gx = goals[3 * b], gy = goals[3 * b + 1], gz = goals[3 * b + 2];
    static_cast<R*>(a.T)[(int64_t)b * a.H * a.W * a.L + (gy * a.W + gx) * a.L + gz] = R(0);
    __threadfence();
    qpush(q, b * a.tpv + ((int)(gy / a.ty) * a.ntx + (int)(gx / a.tx)) * a.ntz + (int)(gz / a.tz), kSelf);
}

hipError_t fim3d_persist_init(const Fim3dArgs& a, const Fim2dArgs& q, bool f64, const int64_t* d_goals, int B,
                              hipStream_t st) {
    const int64_t n = (int64_t)B * a.H * a.W * a.L;
    const int64_t nslots = (int64_t)q.qmask + 1;
    const int grid = (int)std::min<int64_t>(4096, (std::max<int64_t>(n, nslots) + 255) / 256);
    hipError_t e = hipMemsetAsync(q.qhead, 0, kQueueCtlBytes, st);  // head tail active error
    if (e != hipSuccess) return e;
    const int sg = (B + 255) / 256;
    if (f64) {
        hipLaunchKernelGGL(fim3d_pinit_kernel<double>, dim3(grid), dim3(256), 0, st, static_cast<double*>(a.T), n,
                           q.qstate, (int64_t)a.capacity, q.qslot, nslots);
        hipLaunchKernelGGL(fim3d_pseed_kernel<double>, dim3(sg), dim3(256), 0, st, a, q, d_goals, B);
    } else {
        hipLaunchKernelGGL(fim3d_pinit_kernel<float>, dim3(grid), dim3(256), 0, st, static_cast<float*>(a.T), n,
                           q.qstate, (int64_t)a.capacity, q.qslot, nslots);
        hipLaunchKernelGGL(fim3d_pseed_kernel<float>, dim3(sg), dim3(256), 0, st, a, q, d_goals, B);
    }
    return hipGetLastError();
}

hipError_t fim3d_persist(const Fim3dArgs& a, const Fim2dArgs& q, bool f64, int grid, hipStream_t st) {
    if (f64)
        hipLaunchKernelGGL(fim3d_persist_kernel<double>, dim3(grid), dim3(256), 0, st, a, q);
    else
        hipLaunchKernelGGL(fim3d_persist_kernel<float>, dim3(grid), dim3(256), 0, st, a, q);
    return hipGetLastError();
}

int fim3d_persist_resident(bool f64, int cus) {
    int per_cu = 0;
    const hipError_t e = f64 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fim3d_persist_kernel<double>, 256, 0)
                             : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fim3d_persist_kernel<float>, 256, 0);
    if (e != hipSuccess || per_cu < 1) per_cu = 1;
    return per_cu * cus;
}

// FastMarching3D.computeTmap's early exit (:137-142: the loop breaks right after popping
// `start`) restated on a converged full field Tf.  The reference pops in nondecreasing T, so the
// closed set is {T < T[start]} plus `start` itself; closed cells keep their final values.  Ties:
// the reference pops equal T in LIFO insertion order, which a field does not record; cells exactly
// tied with `start` are taken as not yet popped (the fp64 solver computes in the reference's
// arithmetic, solve3_ref, so ties of the reference are ties here).  Every other finite-cost cell
// with a closed 6-neighbour is in the narrow band and keeps its value too: the reference's
// tentative band value (:77-95) is >= the final value, equal when its last update saw final
// neighbours, and depends on the sequential update order beyond that; the path the planner
// descends from `start` (:1639) is the reference's on every fixture (tests/golden/fm3d_early.npz).
// The rest is +inf, as the reference leaves it (np.gradient at :200 sees those cells).
// ts_off: -1 = no early exit (start == goal, outside the volume: the reference never pops it).
template <typename R>
__global__ __launch_bounds__(256) void fim3d_early_kernel(const R* __restrict__ cost, const R* __restrict__ Tf,
                                                          R* __restrict__ Te, int64_t H, int64_t W, int64_t L,
                                                          int64_t ts_off) {
    constexpr R INF = Real<R>::inf();
    const R ts = ts_off >= 0 ? Tf[ts_off] : INF;  // +inf: no early exit
    const int64_t n = H * W * L;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const R v = Tf[i];
        if (v < ts || i == ts_off) {
            Te[i] = v;
            continue;
        }
        if (!(cost[i] < INF)) {
            Te[i] = INF;
            continue;
        }
        const int64_t z = i % L, xy = i / L, x = xy % W, y = xy / W;
        auto closed = [&](bool in, int64_t j) { return in && (Tf[j] < ts || j == ts_off); };
        const bool band = closed(x > 0, i - L) || closed(x + 1 < W, i + L) || closed(y > 0, i - W * L) ||
                          closed(y + 1 < H, i + W * L) || closed(z > 0, i - 1) || closed(z + 1 < L, i + 1);
        Te[i] = band ? v : INF;
    }
}

hipError_t fim3d_early(const void* cost, const void* Tf, void* Te, int64_t H, int64_t W, int64_t L, int64_t ts_off,
                       bool f64, hipStream_t st) {
    const int64_t n = H * W * L;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(8192, (n + 255) / 256));
    if (f64)
        hipLaunchKernelGGL(fim3d_early_kernel<double>, dim3(grid), dim3(256), 0, st, static_cast<const double*>(cost),
                           static_cast<const double*>(Tf), static_cast<double*>(Te), H, W, L, ts_off);
    else
        hipLaunchKernelGGL(fim3d_early_kernel<float>, dim3(grid), dim3(256), 0, st, static_cast<const float*>(cost),
                           static_cast<const float*>(Tf), static_cast<float*>(Te), H, W, L, ts_off);
    return hipGetLastError();
}

template <typename R>
__global__ __launch_bounds__(256) void max_finite_kernel(const R* __restrict__ c, int64_t n, R* __restrict__ out) {
    R m = R(0);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const R v = c[i];
        if (v < Real<R>::inf() && v > m) m = v;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const R o = __shfl_xor(m, off, 64);
        m = o > m ? o : m;
    }
    // non-negative IEEE values order as unsigned integers of their bits
    if ((threadIdx.x & 63) == 0) {
        if constexpr (sizeof(R) == 8)
            atomicMax(reinterpret_cast<unsigned long long*>(out), (unsigned long long)__double_as_longlong(m));
        else
            atomicMax(reinterpret_cast<unsigned*>(out), __float_as_uint(m));
    }
}

hipError_t max_finite(const void* cost, int64_t n, bool f64, void* d_max, hipStream_t st) {
    hipError_t e = hipMemsetAsync(d_max, 0, 8, st);
    if (e != hipSuccess) return e;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (n + 255) / 256));
    if (f64)
        hipLaunchKernelGGL(max_finite_kernel<double>, dim3(grid), dim3(256), 0, st, static_cast<const double*>(cost),
                           n, static_cast<double*>(d_max));
    else
        hipLaunchKernelGGL(max_finite_kernel<float>, dim3(grid), dim3(256), 0, st, static_cast<const float*>(cost), n,
                           static_cast<float*>(d_max));
    return hipGetLastError();
}

// tile shape for a volume with L layers: <= 1024 cells, halo box <= 18 x 18 x 10
void fim3d_tile_shape(int64_t L, int* tx, int* ty, int* tz) {
    if (L <= 4) {
        *tz = (int)L;
        *tx = 16;
        *ty = 16;
    } else if (L <= 8) {
        *tz = (int)L;
        *tx = 16;
        *ty = 8;
    } else {
        *tz = 8;
        *tx = 16;
        *ty = 8;
    }
}

}  // namespace eik
