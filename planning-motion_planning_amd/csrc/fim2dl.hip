// fim2dl.hip -- layered block FIM: the Eikonal of FastMarching3D.py on volumes with few layers
// (gfx950 / CDNA4).
//
// The rover's coupled (x, y, locomotion-mode) costmaps (BASELINE configs[4]) are 3D volumes
// cost[y][x][z] (FastMarching3D.py layout, z fastest) whose z extent is a handful of layers.
// The generic 3D solver (fim3d.hip) relaxes small boxes Jacobi-style; here the volume is treated
// as a 2D raster of cells that carry NL <= 4 layers, solved by the same tile-queue engine as the
// 2D solver (fim_engine.hpp, persistent FIFO driver, in-place revisits, activation-direction
// sweeps -- fim2d.hip):
//
//  * a 64 x 64 tile keeps, per cell, its NL layers in one float4 LDS slot (T and cost; unused
//    slots +inf), so one ds_read_b128 fetches every layer of a neighbour;
//  * each of the four waves runs one quadrant sweep (skewed anti-diagonals, DPP upstream-x, as
//    in fim2d.hip); at each step a lane updates its cell in ALL layers -- NL independent
//    Godunov chains that hide each other's latency.  The z neighbours of a layer are the
//    cell's other layers as read at that step (Jacobi in z within a step, Gauss-Seidel in x/y);
//  * the local solve is the reference's n-D Godunov "drop the largest" rule
//    (FastMarching3D.py:59-75) over the axis minima (x, y, z), in the form of fim3d.hip's
//    godunov3 (solutions relative to the smallest neighbour), made select-only.
// Layers outside [z0, z0 + NL) are not solved and read as +inf: a volume whose first and last
// layers are all-impassable (the reference pads z with inf, Coupled_motion_planner.py:355-356)
// is solved on its inner layers only (the host checks the padding).  Parity with the CPU FMM
// is the same fixed-point argument as 2D (the reference FM3D equals
// the 3D Godunov fixed point to 3.5e-12).
#include "fim_engine.hpp"

namespace eik {

constexpr int kMaxLayers = 4;  // float4 per cell in LDS

struct TileLdsL {
    float4 Tbuf[(kLds + 2 * kGuard) * kLds];  // tile + halo ring (66 x 66 at offset kGuard * kLds), guard rows
                                              // above and below (fim2d.hip's sweep_quadrant)
    float4 Cbuf[(kLds + 2 * kGuard) * kLds];  // costs in the same layout; halo ring and guard rows = +inf
    unsigned flags;
    unsigned key[5];
    int tile;
    unsigned dirs;
};
// A sweep's 4-step group spans rows [-(kAhead - 1), kLds - 1 + kAhead - 1]: every row it reads (T
// and cost alike) is inside the guard rows of both arrays, and a guard row's +inf cost keeps its T
// at +inf (the Godunov update of an infinite cost never lowers a cell).
static_assert(kGuard >= kAhead - 1, "guard rows must cover a group's overshoot");
static_assert(offsetof(TileLdsL, Cbuf) == sizeof(float4) * (kLds + 2 * kGuard) * kLds, "Cbuf must follow Tbuf");
static_assert(sizeof(TileLdsL) <= 160 * 1024, "one layered tile per CU (160 KB LDS)");

__device__ __forceinline__ float f4get(const float4& v, int z) { return z == 0 ? v.x : z == 1 ? v.y : z == 2 ? v.z : v.w; }

// n-D Godunov of FastMarching3D.py:59-75 on the axis minima a, b, c (non-negative or +inf, never
// NaN): sorted s0 <= s1 <= s2, the 3-axis solution when C^2 > (s2-s0)^2 + (s2-s1)^2, else the
// 2-axis one when C^2 > (s1-s0)^2, else s0 + C.  The 1- and 2-axis cases share one form with
// d = min(s1 - s0, C) (as godunov2_fast); the 3-axis case is selected.  A NaN from inf - inf
// fails every comparison / sorts above +inf in the unsigned min, so +inf inputs give +inf.
// EIK_G3_ONE_SQRT (default on): the case is selected BEFORE the square root, so each layer-update
// takes one v_sqrt_f32 (a quarter-rate transcendental) instead of two -- the layered sweep is VALU-bound
// at its one wave per SIMD (~100 VALU per 3-layer step).
#ifndef EIK_G3_ONE_SQRT
#define EIK_G3_ONE_SQRT 1
#endif
// Sorted triple of non-negative floats / +inf / NaN on their bit patterns: one v_min3_u32, one
// v_med3_u32, one v_max3_u32 (the compiler's min/max network took ~9 instructions).
__device__ __forceinline__ void sort3u(float a, float b, float c, float& s0, float& s1, float& s2) {
    unsigned r0, r1, r2;
    asm("v_min3_u32 %0, %1, %2, %3" : "=v"(r0) : "v"(__float_as_uint(a)), "v"(__float_as_uint(b)), "v"(__float_as_uint(c)));
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r1) : "v"(__float_as_uint(a)), "v"(__float_as_uint(b)), "v"(__float_as_uint(c)));
    asm("v_max3_u32 %0, %1, %2, %3" : "=v"(r2) : "v"(__float_as_uint(a)), "v"(__float_as_uint(b)), "v"(__float_as_uint(c)));
    s0 = __uint_as_float(r0);
    s1 = __uint_as_float(r1);
    s2 = __uint_as_float(r2);
}
#ifndef EIK_G3_SORT3
#define EIK_G3_SORT3 1
#endif
__device__ __forceinline__ float godunov3_fast(float a, float b, float c, float C) {
#if EIK_G3_SORT3
    float s0, s1, s2;
    sort3u(a, b, c, s0, s1, s2);
#else
    const float lo = umin(a, b), hi = umax(a, b);
    const float mid = umin(hi, c), s2 = umax(hi, c);
    const float s0 = umin(lo, mid), s1 = umax(lo, mid);
#endif
    const float C2 = C * C;
    const float bp = s1 - s0, cp = s2 - s0, cb = s2 - s1;
    const float d = umin(bp, C);
#if EIK_G3_ONE_SQRT
    const float cb2 = cb * cb;
    const bool three = C2 > __builtin_fmaf(cp, cp, cb2);  // NaN (an +inf axis) -> false
    // 2 axes: 2C^2 - d^2; 3 axes: 3C^2 - 2(bp^2 + cp^2 - bp cp), and bp^2 - bp cp + cp^2 = cb^2 + bp cp
    const float q12 = __builtin_fmaf(-d, d, C2) + C2;
    const float q3 = __builtin_fmaf(-2.f, __builtin_fmaf(bp, cp, cb2), 3.f * C2);
    const float num = three ? bp + cp : d;
    const float k = three ? 1.f / 3.f : 0.5f;
    return __builtin_fmaf(num + __builtin_amdgcn_sqrtf(three ? q3 : q12), k, s0);
#else
    const float t12 = __builtin_fmaf(0.5f, d + __builtin_amdgcn_sqrtf(__builtin_fmaf(-d, d, C2) + C2), s0);
    const float q3 = 3.f * C2 - 2.f * (bp * bp + cp * cp - bp * cp);
    const float t3 = __builtin_fmaf(bp + cp + __builtin_amdgcn_sqrtf(q3), 1.f / 3.f, s0);
    return C2 > cp * cp + cb * cb ? t3 : t12;
#endif
}

// One quadrant sweep over all NL layers (cf. sweep_quadrant in fim2d.hip; same skew, clamp and
// read-ahead, float4 cells, and the same upstream-only x/y neighbours: the four concurrent sweeps
// cover every x/y neighbour pair and the n-D update is monotone, so the fixed point is the one of
// reading both neighbours per axis -- 3 float4 LDS reads per step instead of 5).
template <int NL, int DX, int DY>
__device__ __forceinline__ void sweep_layered(float4* __restrict__ Ts, int lane) {
    constexpr float INF = __builtin_inff();
    constexpr int S = (int)sizeof(float4);
    constexpr int kRow = kLds * S;
    constexpr int kCsB = (kLds + 2 * kGuard) * kLds * S;  // Cs - Ts in bytes (Cbuf - Tbuf)
    constexpr int D = kAhead;
    char* const base = reinterpret_cast<char*>(Ts);
    auto ld = [&](int off) { return *reinterpret_cast<const float4*>(base + off); };
    const int col = (DX > 0 ? lane : kTile - 1 - lane) + 1;
    // the LDS row is clamped once per group of D steps (its lowest row into [-(D - 1), 65]) and the
    // group's steps are immediate offsets from it, as in fim2d.hip's sweep_quadrant
    const int lo_b = -(D - 1) * kRow + col * S, hi_b = (kLds - 1) * kRow + col * S;
    int raw = DY > 0 ? (1 - lane) * kRow + col * S : (kTile - (D - 1) + lane) * kRow + col * S;
    auto off = [](int u) { return (DY > 0 ? u : D - 1 - u) * kRow; };
    auto clampb = [&](int x) {
        int r;
        asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(lo_b), "v"(hi_b));
        return r;
    };
    const float4 h = ld((DY > 0 ? 0 : kLds - 1) * kRow + col * S);
    float cur[NL];
#pragma unroll
    for (int z = 0; z < NL; ++z) cur[z] = f4get(h, z);
    float4 q_old[D], q_upx[D], q_c[D];
    int gb = clampb(raw);  // lowest row of the group being fetched
    raw += DY * D * kRow;
    auto fetch = [&](int u) {
        const int o = gb + off(u);
        q_old[u] = ld(o);
        q_upx[u] = ld(o - DX * S);
        q_c[u] = ld(o + kCsB);
    };
#pragma unroll
    for (int u = 0; u < D; ++u) fetch(u);
    for (int s = 0; s < 2 * kTile; s += D) {
        const int gcur = gb;
        gb = clampb(raw);
        raw += DY * D * kRow;
#pragma unroll
        for (int u = 0; u < D; ++u) {
            float* const cell = reinterpret_cast<float*>(base + gcur + off(u));
#pragma unroll
            for (int z = 0; z < NL; ++z) {
                const float old = f4get(q_old[u], z);
                // lanes 1..: lane l-1's fresh value, or the (possibly lower) LDS one; lane 0: halo column
                const float ux = umin(wave_shr1_umin_id(cur[z]), f4get(q_upx[u], z));
                const float tz = umin(z > 0 ? f4get(q_old[u], z - 1) : INF, z + 1 < NL ? f4get(q_old[u], z + 1) : INF);
                const float w = godunov3_fast(ux, cur[z], tz, f4get(q_c[u], z));
                lds_min(cell + z, w);
                cur[z] = umin(w, old);
            }
            fetch(u);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

// Stage, sweep and write back one layered tile (cf. process_tile in fim2d.hip).  Thread t owns
// cells t + 256 j (j < 16): row (t >> 6) + 4 j, column t & 63 -- a wave reads whole tile rows,
// i.e. 64 * ls contiguous floats per layer load.  Leaves L.flags (bits 0..3: neighbour N/S/W/E
// can improve; 128: some cell decreased by more than the tolerance).
template <int NL, bool COH>
__device__ __forceinline__ void process_tile_layered(const Fim2dArgs& a, int tile, TileLdsL& L, float keep) {
    constexpr float INF = __builtin_inff();
    const float4 INF4 = make_float4(INF, INF, INF, INF);
    float4* const Ts = L.Tbuf + kGuard * kLds;
    float4* const Cs = L.Cbuf + kGuard * kLds;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int map = tile / a.tiles_per_map;
    const int rem = tile - map * a.tiles_per_map;
    const int ty = rem / a.ntx, tx = rem - (rem / a.ntx) * a.ntx;
    const int64_t ls = a.ls, plane = a.H * a.W * ls;
    const float* __restrict__ cost = static_cast<const float*>(a.cost) + map * plane;
    const TMem<float, COH> T(static_cast<float*>(a.T) + map * plane, plane);
    const int64_t y0 = (int64_t)ty * kTile, x0 = (int64_t)tx * kTile;

    if (tid == 0) L.flags = 0;
    if (tid < 5) L.key[tid] = 0x7f800000u;
    // halo ring: wave 0 north row, 1 south row, 2 west column, 3 east column (out of range: +inf)
    int h;
    int64_t hy, hx;
    if (wave == 0)      { h = 0 * kLds + lane + 1;          hy = y0 - 1;      hx = x0 + lane; }
    else if (wave == 1) { h = (kLds - 1) * kLds + lane + 1; hy = y0 + kTile;  hx = x0 + lane; }
    else if (wave == 2) { h = (lane + 1) * kLds + 0;        hy = y0 + lane;   hx = x0 - 1; }
    else                { h = (lane + 1) * kLds + kLds - 1; hy = y0 + lane;   hx = x0 + kTile; }
    const bool hin = hy >= 0 && hy < a.H && hx >= 0 && hx < a.W;
    const int64_t hgi = hin ? (hy * a.W + hx) * ls + a.z0 : 0;
    auto load_halo = [&]() {  // unconditional loads (an in-range index), then the +inf select
        float v[4] = {INF, INF, INF, INF};
#pragma unroll
        for (int z = 0; z < NL; ++z) v[z] = T.ld(hgi + z);
#pragma unroll
        for (int z = 0; z < NL; ++z) v[z] = hin ? v[z] : INF;
        return make_float4(v[0], v[1], v[2], v[3]);
    };
    // ---- stage: every global load of the visit (T, cost, halo) is issued before the first LDS
    // store and each path stores its own values (as fim2d.hip's process_tile; interleaved, the
    // staging took one memory round trip per row, 16 in all)
    float told[16][NL];
    auto store_tile = [&](const float (&cc)[16][NL], float4 hv) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int ry = wave + 4 * j;
            float t4[4] = {INF, INF, INF, INF}, c4[4] = {INF, INF, INF, INF};
#pragma unroll
            for (int z = 0; z < NL; ++z) {
                t4[z] = told[j][z];
                c4[z] = cc[j][z];
            }
            Ts[(ry + 1) * kLds + lane + 1] = make_float4(t4[0], t4[1], t4[2], t4[3]);
            Cs[(ry + 1) * kLds + lane + 1] = make_float4(c4[0], c4[1], c4[2], c4[3]);
        }
        Ts[h] = hv;
    };
    if (y0 + kTile <= a.H && x0 + kTile <= a.W) {  // full tile: no per-cell range test
        float cc[16][NL];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int64_t gi = ((y0 + wave + 4 * j) * a.W + x0 + lane) * ls + a.z0;
#pragma unroll
            for (int z = 0; z < NL; ++z) {
                told[j][z] = T.ld(gi + z);
                cc[j][z] = cost[gi + z];
            }
        }
        store_tile(cc, load_halo());
    } else {
        float cc[16][NL];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int64_t gy = y0 + wave + 4 * j, gx = x0 + lane;
            const bool in = gy < a.H && gx < a.W;
            const int64_t gi = in ? (gy * a.W + gx) * ls + a.z0 : 0;
#pragma unroll
            for (int z = 0; z < NL; ++z) {
                const float t = T.ld(gi + z), c = cost[gi + z];
                told[j][z] = in ? t : INF;
                cc[j][z] = in ? c : INF;
            }
        }
        store_tile(cc, load_halo());
    }
    Cs[h] = INF4;
    if (lane < 4) {
        const int corner = (lane >> 1) * (kLds - 1) * kLds + (lane & 1) * (kLds - 1);
        Cs[corner] = INF4;
        Ts[corner] = INF4;
    }
    __syncthreads();

    const int kPasses = COH ? a.max_passes : 1;
    unsigned dirs = L.dirs;  // this pass's sweeps (register: see fim2d.hip process_tile)
    for (int pass = 0;; ++pass) {
        if ((dirs >> wave) & 1u) {
            if (wave == 0)      sweep_layered<NL, +1, +1>(Ts, lane);
            else if (wave == 1) sweep_layered<NL, -1, +1>(Ts, lane);
            else if (wave == 2) sweep_layered<NL, +1, -1>(Ts, lane);
            else                sweep_layered<NL, -1, -1>(Ts, lane);
        }
        __syncthreads();
        // ---- write back changed cells, collect side flags
        unsigned fl = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int ry = wave + 4 * j;
            const int64_t gy = y0 + ry, gx = x0 + lane;
            const bool in = gy < a.H && gx < a.W;
            const int64_t gi = (gy * a.W + gx) * ls + a.z0;
            const float4 nv4 = Ts[(ry + 1) * kLds + lane + 1];
#pragma unroll
            for (int z = 0; z < NL; ++z) {
                const float nv = f4get(nv4, z);
                if (in && nv < told[j][z]) T.st(gi + z, nv);
                if (nv < told[j][z] * keep) {
                    fl |= 128u;
                    // a neighbour can improve only if this edge value undercuts its adjacent cell
                    if (ry == 0 && nv < f4get(Ts[lane + 1], z)) fl |= 1u;
                    if (ry == kTile - 1 && nv < f4get(Ts[(kLds - 1) * kLds + lane + 1], z)) fl |= 2u;
                    if (lane == 0 && nv < f4get(Ts[(ry + 1) * kLds], z)) fl |= 4u;
                    if (lane == kTile - 1 && nv < f4get(Ts[(ry + 1) * kLds + kLds - 1], z)) fl |= 8u;
                }
                told[j][z] = nv;  // what memory holds now
            }
        }
        if (fl) atomicOr(&L.flags, fl);
        if constexpr (COH) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
        __syncthreads();
        const unsigned f = L.flags;  // uniform
        if (!(f & 128u) || pass + 1 >= kPasses) break;
        // the halo reload is issued first and the budget charge goes to wave 1, so wave 0's
        // activation atomics are the only round trips the next pass waits for
        const float4 hv = load_halo();
        if (tid == 64) charge_inplace_pass(a);  // in-place passes: stats and the visit budget
        activate_neighbours(a, tile, f, L.key, 0, 0u);  // lanes 0..4 (T already drained)
        dirs = 0xFu;  // a self revisit: every direction
        Ts[h] = hv;
        __syncthreads();  // every wave has read L.flags and its halo side is in
        if (tid == 0) L.flags = 0;
    }
}

// Persistent driver (cf. fim2d_persist_kernel): one launch per solve, device FIFO of tiles.
template <int NL>
__global__ __launch_bounds__(kThreads) void fim2dl_persist_kernel(Fim2dArgs a) {
    __shared__ TileLdsL L;
    constexpr float INF = __builtin_inff();
    for (int i = threadIdx.x; i < kGuard * kLds; i += kThreads) {  // guard rows: read by sweeps, never lowered
        L.Tbuf[i] = make_float4(INF, INF, INF, INF);
        L.Tbuf[(kLds + kGuard) * kLds + i] = make_float4(INF, INF, INF, INF);
        L.Cbuf[i] = make_float4(INF, INF, INF, INF);
        L.Cbuf[(kLds + kGuard) * kLds + i] = make_float4(INF, INF, INF, INF);
    }
    const float keep = a.keep;
    int tile = -1;
    unsigned nvis = 0;
    for (;;) {
        if (threadIdx.x < 64) {
            if (tile >= 0) {
                const unsigned f = L.flags;
                activate_neighbours(a, tile, f, L.key, 0, 0u);
                if (threadIdx.x == 0 && (f & 128u)) atomicOr(&a.qstate[tile], kPending | kSelf);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (threadIdx.x == 0) {
                    qfinish(a, tile);
                    if (++nvis == 64u) {  // visit cap (negative costs never converge)
                        charge_visits(a, 64ull);
                        nvis = 0;
                    }
                }
            }
        } else if (threadIdx.x == 64) {
            unsigned trig = 0;
            const int t = qgrab(a, trig);
            L.tile = t;
            L.dirs = sweep_dirs(trig);
        }
        __syncthreads();
        tile = __builtin_amdgcn_readfirstlane(L.tile);
        if (tile < 0) break;
        process_tile_layered<NL, true>(a, tile, L, keep);
    }
    if (threadIdx.x == 0 && nvis) atomicAdd(a.visits, (unsigned long long)nvis);
}

__global__ void fim2dl_init_kernel(float* __restrict__ T, int64_t n, unsigned* __restrict__ qstate, int64_t ntiles,
                                   unsigned* __restrict__ qslot, int64_t nslots) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) T[i] = __builtin_inff();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ntiles; i += stride) qstate[i] = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += stride) qslot[i] = 0;
}

// T[goal] = 0 (gz: absolute layer index) and the goal's tile queued
__global__ void fim2dl_seed_kernel(Fim2dArgs a, int64_t gx, int64_t gy, int64_t gz) {
    static_cast<float*>(a.T)[(gy * a.W + gx) * a.ls + gz] = 0.f;
    qpush(a, (int)(gy / kTile) * a.ntx + (int)(gx / kTile), kSelf);
}

__global__ void fim2dl_rewind_kernel(Fim2dArgs a) { *a.qhead = *a.qtail; }

// flag |= 1 if layer z of the [HW][L] volume holds a finite cost
__global__ void layer_finite_kernel(const float* __restrict__ cost, int64_t hw, int64_t L, int64_t z, int* flag) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    bool any = false;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < hw; i += stride)
        any |= cost[i * L + z] != __builtin_inff();
    if (__any(any) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

// ------------------------------------------------------------------------- host launchers
hipError_t fim2dl_init(const Fim2dArgs& a, int64_t gx, int64_t gy, int64_t gz, hipStream_t st) {
    const int64_t n = a.H * a.W * a.ls;
    const int64_t nslots = (int64_t)a.qmask + 1;
    const int grid = (int)std::min<int64_t>(4096, (n + 255) / 256);
    hipError_t e = hipMemsetAsync(a.qhead, 0, kQueueCtlBytes, st);  // head tail active error
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(fim2dl_init_kernel, dim3(grid), dim3(256), 0, st, static_cast<float*>(a.T), n, a.qstate,
                       (int64_t)a.tiles_per_map, a.qslot, nslots);
    hipLaunchKernelGGL(fim2dl_seed_kernel, dim3(1), dim3(1), 0, st, a, gx, gy, gz);
    return hipGetLastError();
}

template <int NL>
static int resident_of(int cus) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fim2dl_persist_kernel<NL>, kThreads, 0) != hipSuccess ||
        per_cu < 1)
        per_cu = 1;
    return per_cu * cus;
}

int fim2dl_persist_resident(int nl, int cus) {
    switch (nl) {
        case 1: return resident_of<1>(cus);
        case 2: return resident_of<2>(cus);
        case 3: return resident_of<3>(cus);
        default: return resident_of<4>(cus);
    }
}

hipError_t fim2dl_persist(const Fim2dArgs& a, int nl, int grid, hipStream_t st) {
    switch (nl) {
        case 1: hipLaunchKernelGGL(fim2dl_persist_kernel<1>, dim3(grid), dim3(kThreads), 0, st, a); break;
        case 2: hipLaunchKernelGGL(fim2dl_persist_kernel<2>, dim3(grid), dim3(kThreads), 0, st, a); break;
        case 3: hipLaunchKernelGGL(fim2dl_persist_kernel<3>, dim3(grid), dim3(kThreads), 0, st, a); break;
        case 4: hipLaunchKernelGGL(fim2dl_persist_kernel<4>, dim3(grid), dim3(kThreads), 0, st, a); break;
        default: return hipErrorInvalidValue;
    }
    hipLaunchKernelGGL(fim2dl_rewind_kernel, dim3(1), dim3(1), 0, st, a);
    return hipGetLastError();
}

hipError_t layer_finite(const float* cost, int64_t hw, int64_t L, int64_t z, int* d_flag, hipStream_t st) {
    const int grid = (int)std::min<int64_t>(2048, (hw + 255) / 256);
    hipLaunchKernelGGL(layer_finite_kernel, dim3(grid), dim3(256), 0, st, cost, hw, L, z, d_flag);
    return hipGetLastError();
}

}  // namespace eik
