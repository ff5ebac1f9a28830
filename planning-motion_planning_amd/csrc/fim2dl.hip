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
//  * a 64 x 64 tile (fp32; fp64: 40 rows x 64 columns, see kRowsOf) keeps, per cell, its NL layers
//    in one LDS slot (T and cost arrays; fp32 a float4, unused slots +inf, so one ds_read_b128
//    fetches every layer of a neighbour; fp64 three doubles);
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

constexpr int kMaxLayers = 4;  // float4 per cell in LDS (fp32); 3 doubles per cell (fp64)

// A cell's layers in LDS: fp32 one float4 (one ds_read_b128 fetches every layer; unused slots
// +inf), fp64 three doubles (NL <= 3: the 155 KB tile of 40 rows below fits the 160 KB LDS).
template <typename R> struct LCell;
template <> struct LCell<float> {
    float4 v;
    __device__ __forceinline__ float get(int z) const { return z == 0 ? v.x : z == 1 ? v.y : z == 2 ? v.z : v.w; }
    static __device__ __forceinline__ LCell make(const float (&x)[4]) { return LCell{make_float4(x[0], x[1], x[2], x[3])}; }
};
template <> struct LCell<double> {
    double v[3];
    __device__ __forceinline__ double get(int z) const { return v[z]; }
    static __device__ __forceinline__ LCell make(const double (&x)[4]) { return LCell{{x[0], x[1], x[2]}}; }
};
// tile rows: 64 (fp32, 156 KB of LDS) or EIK_L64_ROWS (fp64; 40 rows: (40 + 2 + 8 guard) x 66 cells x
// 48 B = 155 KB, the most that fits 160 KB with a step count divisible by the read-ahead depth);
// always 64 columns (one lane each)
#ifndef EIK_L64_ROWS
#define EIK_L64_ROWS 40
#endif
// EIK_L32_ROWS: the fp32 tile's rows (64; round 6 probed 24 / 32 for a second workgroup per CU --
// DESIGN.md §3.3)
#ifndef EIK_L32_ROWS
#define EIK_L32_ROWS 64
#endif
template <typename R> constexpr int kRowsOf = sizeof(R) == 4 ? EIK_L32_ROWS : EIK_L64_ROWS;
// EIK_LSPLIT (round 6, verdict r05 item 5): more than one wave per SIMD for the layered sweep.  The
// tile (one per CU: 156 KB of LDS fp32, 155 KB fp64) is swept by 4 x G waves: wave w runs quadrant
// direction w & 3 on the layer group g = w >> 2 (kLZ0: {0, 1} and {2} for 3 layers in 2 groups).  A layer's chain
// only ever reads its own register state and the other layers through LDS (the z neighbours are the
// read-ahead LDS values, Jacobi in z within a step -- sweep_layered), so the layers partition across
// waves with no new synchronisation: each SIMD interleaves G dependent chains instead of one wave's NL
// chains.  Waves 4.. only sweep (staging, write-back, halo and queue roles stay on waves 0..3) and pass
// the same workgroup barriers.  G = min(NL, EIK_LSPLIT_F32 / _F64); 1 = the one-wave-per-SIMD kernel.
// Measured on C5 (4096^2 x 3, same box, 2 alternations, profiles/r06s7/): G = 1 / 2 / 3 gives fp64 3.70-3.73 /
// 4.34-4.37 / 4.45 and fp32 6.23-6.27 / 7.60-7.66 / 7.09-7.18 Gcells/s (fp32 at G = 3: 168 VGPRs and three
// waves per SIMD cost more than the third chain gives), so fp64 runs three groups and fp32 two.
#ifndef EIK_LSPLIT_F32
#define EIK_LSPLIT_F32 2
#endif
#ifndef EIK_LSPLIT_F64
#define EIK_LSPLIT_F64 3
#endif
template <typename R, int NL>
constexpr int kLGroups = (sizeof(R) == 4 ? EIK_LSPLIT_F32 : EIK_LSPLIT_F64) < NL ? (sizeof(R) == 4 ? EIK_LSPLIT_F32 : EIK_LSPLIT_F64) : NL;
template <typename R, int NL> constexpr int kLThreads = kLGroups<R, NL> * kThreads;
// first layer of group g: the groups' sizes rounded up from the first (3 layers in 2 groups: {0, 1}, {2} --
// the main waves take the larger share: 6.3 -> 7.2 Gcells/s on C5 fp32, against 6.7 for {0}, {1, 2})
#ifndef EIK_LSPLIT_CEIL
#define EIK_LSPLIT_CEIL 1
#endif
// EIK_LSPLIT_ROWS: the sweep-only waves share the staging and write-back rows (1, default) or only sweep (0)
#ifndef EIK_LSPLIT_ROWS
#define EIK_LSPLIT_ROWS 1
#endif
template <int NL, int G> constexpr int kLZ0(int g) { return EIK_LSPLIT_CEIL ? (g * NL + G - 1) / G : g * NL / G; }

// EIK_FRESH_SKIP_L: a full tile's first visit stages only the cost -- its T layers are still the init
// kernel's +inf (the seed kernel queues the goal's tile as visited), as fim2d.hip's kFreshSkip
#ifndef EIK_FRESH_SKIP_L
#define EIK_FRESH_SKIP_L 1
#endif
constexpr bool kFreshSkipL = EIK_FRESH_SKIP_L;

template <typename R, int TH>
struct TileLdsL {
    LCell<R> Tbuf[(TH + 2 + 2 * kGuard) * kLds];  // tile + halo ring ((TH+2) x 66 at offset kGuard * kLds), guard
                                                  // rows above and below (fim2d.hip's sweep_quadrant)
    LCell<R> Cbuf[(TH + 2 + 2 * kGuard) * kLds];  // costs in the same layout; halo ring and guard rows = +inf
    unsigned flags;
    unsigned key[5];
    int tile;
    unsigned dirs;
    unsigned fresh;  // the tile's first visit (kFreshSkipL)
};
// A sweep's 4-step group spans rows [-(kAhead - 1), TH + 1 + kAhead - 1]: every row it reads (T
// and cost alike) is inside the guard rows of both arrays, and a guard row's +inf cost keeps its T
// at +inf (the Godunov update of an infinite cost never lowers a cell).
static_assert(kGuard >= kAhead - 1, "guard rows must cover a group's overshoot");
using TileLdsL32 = TileLdsL<float, kTile>;
using TileLdsL64 = TileLdsL<double, EIK_L64_ROWS>;
static_assert(offsetof(TileLdsL32, Cbuf) == sizeof(float4) * (kTile + 2 + 2 * kGuard) * kLds, "Cbuf must follow Tbuf");
static_assert(offsetof(TileLdsL64, Cbuf) == 24 * (EIK_L64_ROWS + 2 + 2 * kGuard) * kLds, "Cbuf must follow Tbuf");
static_assert(EIK_L64_ROWS % 4 == 0 && EIK_L64_ROWS <= kTile, "fp64 tile rows: whole rows per thread, <= 64");
static_assert(sizeof(TileLdsL<float, kTile>) <= 160 * 1024, "one layered fp32 tile per CU (160 KB LDS)");
static_assert(sizeof(TileLdsL64) <= 160 * 1024, "one layered fp64 tile per CU (160 KB LDS)");

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
// fp64 (the reference's precision): the same select-before-one-square-root form.  The minima are
// IEEE minNum / maxNum (v_min_f64 / v_max_f64: a NaN operand yields the other; the inputs are
// never NaN), the square root is the range-free two-Newton sequence of the 2D fp64 step
// (eik_common.hpp godunov2_chain, EIK_CHAIN 3): q >= C^2 in both cases (3 axes: C^2 > cp^2 + cb^2
// gives q3 > C^2) and the staged costs are >= 2^-500, so q >= 2^-1000; C = +inf gives NaN (no update).
__device__ __forceinline__ double fmax_nn(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double godunov3_fast(double a, double b, double c, double C) {
    const double lo = fmin_nn(a, b), hi = fmax_nn(a, b);
    const double s0 = fmin_nn(lo, c), s2 = fmax_nn(hi, c), s1 = fmin_nn(hi, fmax_nn(lo, c));
    const double C2 = C * C;
    const double bp = s1 - s0, cp = s2 - s0, cb = s2 - s1;
    const double d = fmin_nn(bp, C);  // NaN bp (all +inf) -> C
    const double cb2 = cb * cb;
    const bool three = C2 > __builtin_fma(cp, cp, cb2);
    const double q12 = __builtin_fma(-d, d, C2) + C2;
    const double q3 = __builtin_fma(-2.0, __builtin_fma(bp, cp, cb2), 3.0 * C2);
    const double num = three ? bp + cp : d;
    const double k = three ? 1.0 / 3.0 : 0.5;
    const double q = three ? q3 : q12;
    const double y = __builtin_amdgcn_rsq(q);
    const double g = q * y, h = 0.5 * y;
    const double s1n = __builtin_fma(__builtin_fma(-g, g, q), h, g);
    const double r = __builtin_fma(__builtin_fma(-s1n, s1n, q), h, s1n);
    return __builtin_fma(num + r, k, s0);
}

// Lane l-1's fresh value for lanes 1.. (DPP wave shift), lane 0's from LDS (the halo column).
// fp32: the prefetched LDS value of the same cell is a valid, possibly lower, bound too -- one
// v_min_u32_dpp takes both; fp64: the DPP value alone (as fim2d.hip's fp64 sweep).
__device__ __forceinline__ float upstream_x(float cur, float lds) { return umin(wave_shr1_umin_id(cur), lds); }
__device__ __forceinline__ double upstream_x(double cur, double lds) { return wave_shr1(cur, lds); }
__device__ __forceinline__ float min_nn(float a, float b) { return umin(a, b); }
__device__ __forceinline__ double min_nn(double a, double b) { return fmin_nn(a, b); }

// One quadrant sweep over all NL layers (cf. sweep_quadrant in fim2d.hip; same skew, clamp and
// read-ahead, one LDS cell per neighbour, and the same upstream-only x/y neighbours: the four
// concurrent sweeps cover every x/y neighbour pair and the n-D update is monotone, so the fixed
// point is the one of reading both neighbours per axis -- 3 cell reads per step instead of 5).
// TH tile rows: TH + 64 skewed steps.
// EIK_SWEEP_UNROLL_L: groups of kAhead steps per loop iteration (one back-branch each; fim2d.hip's
// EIK_SWEEP_UNROLL).  1 -> 2: C5 fp64 1.85-1.92 -> 1.98-2.00, fp32 4.67 -> 4.76-4.85 Gcells/s; 4 in
// between (profiles/r05p_layered_unroll_ab.log)
#ifndef EIK_SWEEP_UNROLL_L
#define EIK_SWEEP_UNROLL_L 2
#endif
#define EIK_STRL_(x) #x
#define EIK_UNROLL_L_(n) _Pragma(EIK_STRL_(unroll n))
#define EIK_UNROLL_L(n) EIK_UNROLL_L_(n)
template <typename R, int TH, int NL, int DX, int DY, int Z0 = 0, int Z1 = NL>
__device__ __forceinline__ void sweep_layered(LCell<R>* __restrict__ Ts, int lane) {
    constexpr R INF = Real<R>::inf();
    constexpr int S = (int)sizeof(LCell<R>);
    constexpr int kRow = kLds * S;
    constexpr int kCsB = (TH + 2 + 2 * kGuard) * kLds * S;  // Cs - Ts in bytes (Cbuf - Tbuf)
    constexpr int D = kAhead;
    static_assert((TH + kTile) % D == 0, "pipeline depth must divide the step count");
    char* const base = reinterpret_cast<char*>(Ts);
    auto ld = [&](int off) { return *reinterpret_cast<const LCell<R>*>(base + off); };
    const int col = (DX > 0 ? lane : kTile - 1 - lane) + 1;
    // the LDS row is clamped once per group of D steps (its lowest row into [-(D - 1), TH + 1]) and
    // the group's steps are immediate offsets from it, as in fim2d.hip's sweep_quadrant
    const int lo_b = -(D - 1) * kRow + col * S, hi_b = (TH + 1) * kRow + col * S;
    int raw = DY > 0 ? (1 - lane) * kRow + col * S : (TH - (D - 1) + lane) * kRow + col * S;
    auto off = [](int u) { return (DY > 0 ? u : D - 1 - u) * kRow; };
    auto clampb = [&](int x) {
        int r;
        asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(lo_b), "v"(hi_b));
        return r;
    };
    const LCell<R> h = ld((DY > 0 ? 0 : TH + 1) * kRow + col * S);
    R cur[NL];  // (layers outside [Z0, Z1) are another wave's: unused here)
#pragma unroll
    for (int z = Z0; z < Z1; ++z) cur[z] = h.get(z);
    LCell<R> q_old[D], q_upx[D], q_c[D];
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
    EIK_UNROLL_L(EIK_SWEEP_UNROLL_L)
    for (int s = 0; s < TH + kTile; s += D) {
        const int gcur = gb;
        gb = clampb(raw);
        raw += DY * D * kRow;
#pragma unroll
        for (int u = 0; u < D; ++u) {
            R* const cell = reinterpret_cast<R*>(base + gcur + off(u));
#pragma unroll
            for (int z = Z0; z < Z1; ++z) {
                const R old = q_old[u].get(z);
                const R ux = upstream_x(cur[z], q_upx[u].get(z));
                // layer neighbours; an end layer has one (the minima are inline asm, which the
                // compiler cannot fold against the +inf of a missing neighbour)
                R tz;
                if constexpr (NL == 1) tz = INF;
                else if (z == 0) tz = q_old[u].get(1);
                else if (z + 1 == NL) tz = q_old[u].get(z - 1);
                else tz = min_nn(q_old[u].get(z - 1), q_old[u].get(z + 1));
                const R w = godunov3_fast(ux, cur[z], tz, q_c[u].get(z));
                lds_min(cell + z, w);
                cur[z] = min_nn(w, old);  // NaN w (no update) keeps old
            }
            fetch(u);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

// (EIK_SPLIT_WB_L, round 4: fim2d.hip's split-role boundary -- two waves storing the write-back
// without waiting, two reloading the halo, activations after the drain from the next sweep --
// measured and removed: C5 fp64 1.96-2.01 -> 1.81-1.87, fp32 4.73-4.83 -> 4.19-4.35 Gcells/s,
// profiles/r04e_layered_split_ab.log.)

// EIK_ACT_SPLIT_L: the split activations of fim2d.hip's in-place passes (EIK_ACT_SPLIT) for the
// layered solver.  Off: no gain on C5 (fp64 2.01-2.07 -> 2.00-2.03, fp32 4.80-4.85 -> 4.69-4.82
// Gcells/s, profiles/r03zz2_layered_act_split_ab.log), unlike the 2D sweep (C2 -3.5 / -6 %).
#ifndef EIK_ACT_SPLIT_L
#define EIK_ACT_SPLIT_L 0
#endif

// Stage, sweep and write back one layered tile (cf. process_tile in fim2d.hip).  Thread t owns
// cells t + 64 RW j (j < TH / RW): row (t >> 6) + RW j, column t & 63 -- a wave reads whole tile rows,
// i.e. 64 * ls contiguous values per layer load.  Leaves L.flags (bits 0..3: neighbour N/S/W/E
// can improve; 128: some cell decreased by more than the tolerance).
template <typename R, int NL, bool COH>
__device__ __forceinline__ void process_tile_layered(const Fim2dArgs& a, int tile, TileLdsL<R, kRowsOf<R>>& L,
                                                     float keep) {
    constexpr int TH = kRowsOf<R>;
    // staging and write-back rows: wave r of the RW row waves owns rows r, r + RW, ... (EIK_LSPLIT: the
    // sweep-only waves share them when the rows divide -- half the told[] registers and half the rows per
    // thread at a pass boundary)
    constexpr int G = kLGroups<R, NL>;
    constexpr int RW = EIK_LSPLIT_ROWS ? 4 * G : 4;
    constexpr int NJ = (TH + RW - 1) / RW;  // cells per thread (the last one only on the first TH % RW row waves)
    constexpr R INF = Real<R>::inf();
    const R INFS[4] = {INF, INF, INF, INF};
    const LCell<R> INFC = LCell<R>::make(INFS);
    LCell<R>* const Ts = L.Tbuf + kGuard * kLds;
    LCell<R>* const Cs = L.Cbuf + kGuard * kLds;
    const int tid = threadIdx.x, lane = tid & 63;
    // waves 0..3: halo ring and queue roles, the first layer group's sweeps; waves 4.. (EIK_LSPLIT): the other
    // groups' sweeps; the RW row waves: staging and write-back
    const int wave = (tid >> 6) & 3;
    const bool main = tid < kThreads;
    const int rw = tid >> 6;
    const bool stager = rw < RW;
    auto rowok = [&](int j) { return TH % RW == 0 || rw + RW * j < TH; };  // wave-uniform
    const int map = tile / a.tiles_per_map;
    const int rem = tile - map * a.tiles_per_map;
    const int ty = rem / a.ntx, tx = rem - (rem / a.ntx) * a.ntx;
    // value (y, x, solved layer z) at (y * W + x) * ls + z0 + z * lzs: the [y][x][L] volume (ls = L,
    // lzs = 1) or its layer-planar copy (ls = 1, z0 = 0, lzs = H * W; solve_layered)
    const int64_t ls = a.ls, lzs = a.lzs, plane = a.H * a.W * (lzs > 1 ? NL : ls);
    const R* __restrict__ cost = static_cast<const R*>(a.cost) + map * plane;
    const int64_t y0 = (int64_t)ty * TH, x0 = (int64_t)tx * kTile;
    // T through one buffer resource per solved layer, based at the tile's first halo row: T[i + z *
    // lzs] is Tz[z] at i - b0, and a resource's 32-bit offsets span the TH + 2 rows of one layer the
    // visit touches, whatever the volume's size.  (One resource over the whole T capped the layered
    // solver at 4 GiB: a 16384^2 x 5 fp32 volume went to fim3d.hip at 0.3 Gcells/s,
    // tools/layered_scale_probe.py.)  Indices of out-of-range cells (0, selected away) wrap to
    // offsets past the range: the buffer returns 0 for them.
    const int64_t b0 = (y0 > 0 ? (y0 - 1) * a.W : 0) * ls + a.z0;
    const int64_t span = (TH + 2) * a.W * ls;
    TMem<R, COH> Tz[NL];
#pragma unroll
    for (int z = 0; z < NL; ++z) Tz[z] = TMem<R, COH>(static_cast<R*>(a.T) + map * plane + b0 + z * lzs, span);

    if (tid == 0) L.flags = 0;
    if (tid < 5) L.key[tid] = 0x7f800000u;
    // halo ring: wave 0 north row, 1 south row, 2 west column, 3 east column (out of range: +inf;
    // lanes >= TH of the column waves have none)
    int h;
    int64_t hy, hx;
    if (wave == 0)      { h = 0 * kLds + lane + 1;          hy = y0 - 1;      hx = x0 + lane; }
    else if (wave == 1) { h = (TH + 1) * kLds + lane + 1;   hy = y0 + TH;     hx = x0 + lane; }
    else if (wave == 2) { h = (lane + 1) * kLds + 0;        hy = y0 + lane;   hx = x0 - 1; }
    else                { h = (lane + 1) * kLds + kLds - 1; hy = y0 + lane;   hx = x0 + kTile; }
    const bool hcell = main && (wave < 2 || lane < TH);
    const bool hin = hcell && hy >= 0 && hy < a.H && hx >= 0 && hx < a.W;
    const int64_t hgi = hin ? (hy * a.W + hx) * ls + a.z0 : 0;
    // domain decomposition: the halo cell just outside the block comes from the side's ghost strip, nl
    // values per edge cell ([i][z], as fim2dl_pack_edges_kernel writes them); agent-scope loads -- a
    // live launch's halo agent lowers the ghosts while the block solves (a cut tile's ghost row /
    // column inside the tile is read at staging only: the agent's activation of a busy tile re-queues
    // it, and the next visit stages the new value)
    const R* hg = nullptr;
    int64_t hgo = 0;
    if (hcell && !hin) {
        const R* const* G = reinterpret_cast<const R* const*>(a.ghost);
        if (wave == 0 && hy == -1 && hx < a.W)         { hg = G[0]; hgo = hx * NL; }
        else if (wave == 1 && hy == a.H && hx < a.W)   { hg = G[1]; hgo = hx * NL; }
        else if (wave == 2 && hx == -1 && hy < a.H)    { hg = G[2]; hgo = hy * NL; }
        else if (wave == 3 && hx == a.W && hy < a.H)   { hg = G[3]; hgo = hy * NL; }
    }
    auto load_halo = [&]() {  // unconditional loads (an in-range index), then the +inf select
        R v[4] = {INF, INF, INF, INF};
#pragma unroll
        for (int z = 0; z < NL; ++z) v[z] = Tz[z].ld(hgi - b0);
#pragma unroll
        for (int z = 0; z < NL; ++z) v[z] = hin ? v[z] : (hg ? (COH ? ld_agent(hg + hgo + z) : hg[hgo + z]) : INF);
        return LCell<R>::make(v);
    };
    // ---- stage: every global load of the visit (T, cost, halo) is issued before the first LDS
    // store and each path stores its own values (as fim2d.hip's process_tile; interleaved, the
    // staging took one memory round trip per row, 16 in all)
    R told[NJ][NL];
    auto store_tile = [&](const R (&cc)[NJ][NL], LCell<R> hv) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            if (!rowok(j)) continue;
            const int ry = rw + RW * j;
            R t4[4] = {INF, INF, INF, INF}, c4[4] = {INF, INF, INF, INF};
#pragma unroll
            for (int z = 0; z < NL; ++z) {
                t4[z] = told[j][z];
                c4[z] = cc[j][z];
            }
            Ts[(ry + 1) * kLds + lane + 1] = LCell<R>::make(t4);
            Cs[(ry + 1) * kLds + lane + 1] = LCell<R>::make(c4);
        }
        if (hcell) Ts[h] = hv;
    };
    // fp64: costs as the sweep keeps them (>= 2^-500: the range-free square root, fim2d.hip stage_cost)
    auto scost = [](R c) -> R {
        if constexpr (sizeof(R) == 8) return (c >= R(0) && c < 0x1p-500) ? R(0x1p-500) : c;  // NaN stays NaN
        else return c;
    };
    if (!stager) {
        // (EIK_LSPLIT: the sweep-only waves stage nothing unless they own rows)
    } else if (COH && kFreshSkipL && y0 + TH <= a.H && x0 + kTile <= a.W && __builtin_amdgcn_readfirstlane(L.fresh)) {
        R cc[NJ][NL];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            if (!rowok(j)) continue;
            const int64_t gi = ((y0 + rw + RW * j) * a.W + x0 + lane) * ls + a.z0;
#pragma unroll
            for (int z = 0; z < NL; ++z) {
                told[j][z] = INF;
                cc[j][z] = scost(cost[gi + z * lzs]);
            }
        }
        store_tile(cc, load_halo());
        if (tid == 0) atomicAdd(a.visits + 2, 1ull);  // eik_stats::fresh_visits
    } else if (y0 + TH <= a.H && x0 + kTile <= a.W) {  // full tile: no per-cell range test
        R cc[NJ][NL];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            if (!rowok(j)) continue;
            const int64_t gi = ((y0 + rw + RW * j) * a.W + x0 + lane) * ls + a.z0;
#pragma unroll
            for (int z = 0; z < NL; ++z) {
                told[j][z] = Tz[z].ld(gi - b0);
                cc[j][z] = scost(cost[gi + z * lzs]);
            }
        }
        store_tile(cc, load_halo());
    } else {
        R cc[NJ][NL];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            if (!rowok(j)) continue;
            const int64_t gy = y0 + rw + RW * j, gx = x0 + lane;
            const bool in = gy < a.H && gx < a.W;
            const int64_t gi = in ? (gy * a.W + gx) * ls + a.z0 : 0;
            // a block's south / east ghost cells inside a tile cut by the block's end: the ghost's
            // value with an infinite cost (a halo cell, never updated)
            const R* const* G = reinterpret_cast<const R* const*>(a.ghost);
            const R* gc = (gy == a.H && gx < a.W) ? G[1] : (gx == a.W && gy < a.H) ? G[3] : nullptr;
            const int64_t go = (gy == a.H ? gx : gy) * NL;
#pragma unroll
            for (int z = 0; z < NL; ++z) {
                const R t = Tz[z].ld(gi - b0), c = cost[gi + z * lzs];
                told[j][z] = in ? t : (gc ? (COH ? ld_agent(gc + go + z) : gc[go + z]) : INF);
                cc[j][z] = in ? scost(c) : INF;
            }
        }
        store_tile(cc, load_halo());
    }
    if (hcell) Cs[h] = INFC;
    if (main && lane < 4) {
        const int corner = (lane >> 1) * (TH + 1) * kLds + (lane & 1) * (kLds - 1);
        Cs[corner] = INFC;
        Ts[corner] = INFC;
    }
    __syncthreads();

    const int kPasses = COH ? a.max_passes : 1;
    unsigned dirs = L.dirs;  // this pass's sweeps (register: see fim2d.hip process_tile)
    int act_tile = -1;       // EIK_ACT_SPLIT_L: this lane's activation issued at the last pass boundary
    unsigned act_old = 0u, act_kold = 0x7f800000u;
    float act_k = 0.f;  // priority mode: the activation's key and the neighbour's key before it
    for (int pass = 0;; ++pass) {
        if (EIK_ACT_SPLIT_L && act_tile >= 0) {  // wave 0 lanes 1..4, as its sweep starts (fim2d.hip)
            qpush_complete(a, act_tile, act_old, act_k, act_kold);
            act_tile = -1;
        }
        if ((dirs >> wave) & 1u) {
            const int grp = tid >> 8;  // wave-uniform
            auto run = [&](auto gc) {
                constexpr int g = decltype(gc)::value, Z0 = kLZ0<NL, G>(g), Z1 = kLZ0<NL, G>(g + 1);
                if (wave == 0)      sweep_layered<R, TH, NL, +1, +1, Z0, Z1>(Ts, lane);
                else if (wave == 1) sweep_layered<R, TH, NL, -1, +1, Z0, Z1>(Ts, lane);
                else if (wave == 2) sweep_layered<R, TH, NL, +1, -1, Z0, Z1>(Ts, lane);
                else                sweep_layered<R, TH, NL, -1, -1, Z0, Z1>(Ts, lane);
            };
            if (grp == 0) run(std::integral_constant<int, 0>{});
            else if constexpr (G > 1) {
                if (grp == 1) run(std::integral_constant<int, 1>{});
                else if constexpr (G > 2) {
                    if (grp == 2) run(std::integral_constant<int, 2>{});
                    else if constexpr (G > 3) run(std::integral_constant<int, 3>{});
                }
            }
        }
        __syncthreads();
        // ---- write back changed cells, collect side flags (priority bands: and the entering keys,
        // the smallest improved value per side and overall, as fim2d.hip's write-back)
        unsigned fl = 0;
        R kmin_self = INF, kmin[4] = {INF, INF, INF, INF};
        if (stager) {  // (EIK_LSPLIT: only the row waves store)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            if (!rowok(j)) continue;
            const int ry = rw + RW * j;
            const int64_t gy = y0 + ry, gx = x0 + lane;
            const bool in = gy < a.H && gx < a.W;
            const int64_t gi = (gy * a.W + gx) * ls + a.z0;
            const LCell<R> nv4 = Ts[(ry + 1) * kLds + lane + 1];
#pragma unroll
            for (int z = 0; z < NL; ++z) {
                const R nv = nv4.get(z);
                if (in && nv < told[j][z]) Tz[z].st(gi - b0, nv);
                if (nv < told[j][z] * R(keep)) {
                    fl |= 128u;
                    kmin_self = min_nn(kmin_self, nv);
                    // a neighbour can improve only if this edge value undercuts its adjacent cell
                    if (ry == 0 && nv < Ts[lane + 1].get(z)) { fl |= 1u; kmin[0] = min_nn(kmin[0], nv); }
                    if (ry == TH - 1 && nv < Ts[(TH + 1) * kLds + lane + 1].get(z)) { fl |= 2u; kmin[1] = min_nn(kmin[1], nv); }
                    if (lane == 0 && nv < Ts[(ry + 1) * kLds].get(z)) { fl |= 4u; kmin[2] = min_nn(kmin[2], nv); }
                    if (lane == kTile - 1 && nv < Ts[(ry + 1) * kLds + kLds - 1].get(z)) { fl |= 8u; kmin[3] = min_nn(kmin[3], nv); }
                }
                told[j][z] = nv;  // what memory holds now
            }
        }
        }
        if (fl) atomicOr(&L.flags, fl);
        if (a.bctl) {  // priority bands: the entering keys (f32 bits: T >= 0)
            if (kmin_self < INF) atomicMin(&L.key[0], __float_as_uint((float)kmin_self));
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (kmin[q] < INF) atomicMin(&L.key[q + 1], __float_as_uint((float)kmin[q]));
        }
        if constexpr (COH) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
        __syncthreads();
        const unsigned f = L.flags;  // uniform
        if (!(f & 128u) || pass + 1 >= kPasses) break;
        // the halo reload is issued first and the budget charge goes to wave 1, so wave 0's
        // activation atomics are the only round trips the next pass waits for
        const LCell<R> hv = hcell ? load_halo() : INFC;
        if (tid == 64) charge_inplace_pass(a);  // in-place passes: stats and the visit budget
        if constexpr (COH && EIK_ACT_SPLIT_L)
            act_tile = activate_neighbours_issue(a, tile, f, act_old, L.key, act_k, act_kold);  // queued as the next pass starts
        else
            activate_neighbours(a, tile, f, L.key, 0, 0u);  // lanes 0..4 (T already drained)
        dirs = 0xFu;  // a self revisit: every direction
        if (hcell) Ts[h] = hv;
        __syncthreads();  // every wave has read L.flags and its halo side is in
        if (tid == 0) L.flags = 0;
    }
}

// Live DD halo agent of the layered solver (a block of a few-layer volume, SURVEY §8(e) C5: split in
// x-y, layers together; fim_engine.hpp live_agent_loop serves the mailbox): PACK stores this block's
// edges, NL values per edge cell ([i][z], fim2dl_pack_edges_kernel's layout), into the neighbours'
// receive strips; MERGE min-merges the received strips into the ghosts and queues the edge tile of
// every cell that dropped in any layer (FIFO blocks: a tile already pending costs one atomic).
template <typename R, int NL>
__device__ __forceinline__ void live_agent_layered(const Fim2dArgs& a, unsigned* sh) {
    constexpr int TH = kRowsOf<R>;
    const int tid = threadIdx.x;
    const R* T = static_cast<const R*>(a.T);
    auto at = [&](int64_t y, int64_t x, int z) { return ld_agent(T + (y * a.W + x) * a.ls + a.z0 + z * a.lzs); };
    auto pack = [&](unsigned par, bool) {
        R* tg[4];
        for (int k = 0; k < 4; ++k) tg[k] = static_cast<R*>(a.live->send[par][k]);
        for (int64_t i = tid; i < a.W; i += blockDim.x)
#pragma unroll
            for (int z = 0; z < NL; ++z) {
                if (tg[0]) st_scoped(tg[0] + i * NL + z, at(0, i, z), __HIP_MEMORY_SCOPE_SYSTEM);
                if (tg[1]) st_scoped(tg[1] + i * NL + z, at(a.H - 1, i, z), __HIP_MEMORY_SCOPE_SYSTEM);
            }
        for (int64_t i = tid; i < a.H; i += blockDim.x)
#pragma unroll
            for (int z = 0; z < NL; ++z) {
                if (tg[2]) st_scoped(tg[2] + i * NL + z, at(i, 0, z), __HIP_MEMORY_SCOPE_SYSTEM);
                if (tg[3]) st_scoped(tg[3] + i * NL + z, at(i, a.W - 1, z), __HIP_MEMORY_SCOPE_SYSTEM);
            }
    };
    auto merge = [&](unsigned par, unsigned* count) {
        for (int side = 0; side < 4; ++side) {
            const R* rv = static_cast<const R*>(a.live->recv[par][side]);
            R* g = static_cast<R*>(const_cast<void*>(a.ghost[side]));
            if (!rv || !g) continue;
            const int64_t len = side < 2 ? a.W : a.H;
            for (int64_t i = tid; i < len; i += blockDim.x) {
                bool dropped = false;
                float k = __builtin_inff();
#pragma unroll
                for (int z = 0; z < NL; ++z) {
                    const R v = ld_system(rv + i * NL + z);
                    if (v < ld_agent(g + i * NL + z)) {
                        st_scoped(g + i * NL + z, v, __HIP_MEMORY_SCOPE_AGENT);
                        dropped = true;
                        k = fminf(k, (float)v);
                    }
                }
                if (!dropped) continue;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // the ghost before the activation
                atomicAdd(count, 1u);
                const int ty = side < 2 ? (side == 0 ? 0 : a.nty - 1) : (int)(i / TH);
                const int tx = side < 2 ? (int)(i / kTile) : (side == 2 ? 0 : a.ntx - 1);
                qpush(a, ty * a.ntx + tx, kFromN << side, k);
            }
        }
    };
    live_agent_loop(a, sh, pack, merge);
}

// Persistent driver (cf. fim2d_persist_kernel): one launch per solve, device FIFO of tiles.  A live
// launch (a.live: a decomposition block on dd.solve_live) keeps workgroup 0 as its halo agent.
template <typename R, int NL>
__global__ __launch_bounds__((kLThreads<R, NL>)) void fim2dl_persist_kernel(Fim2dArgs a) {
    constexpr int TH = kRowsOf<R>;
    __shared__ TileLdsL<R, TH> L;
    if (a.live && blockIdx.x == 0) {
        __shared__ unsigned sh[4];
        live_agent_layered<R, NL>(a, sh);
        return;
    }
    constexpr R INF = Real<R>::inf();
    const R INFS[4] = {INF, INF, INF, INF};
    for (int i = threadIdx.x; i < kGuard * kLds; i += kLThreads<R, NL>) {  // guard rows: read by sweeps, never lowered
        L.Tbuf[i] = LCell<R>::make(INFS);
        L.Tbuf[(TH + 2 + kGuard) * kLds + i] = LCell<R>::make(INFS);
        L.Cbuf[i] = LCell<R>::make(INFS);
        L.Cbuf[(TH + 2 + kGuard) * kLds + i] = LCell<R>::make(INFS);
    }
    const float keep = a.keep;
    int tile = -1;
    unsigned nvis = 0;
    for (;;) {
        if (threadIdx.x < 64) {
            if (tile >= 0) {
                const unsigned f = L.flags;
                activate_neighbours(a, tile, f, L.key, 0, 0u);
                if (threadIdx.x == 0 && (f & 128u)) {
                    if (a.bctl) atomicMin(&a.key[tile], 0u);  // priority mode: a self re-queue goes first
                    atomicOr(&a.qstate[tile], kPending | kSelf);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (threadIdx.x == 0) {
                    qfinish(a, tile);
                    if (++nvis == 64u) {  // visit cap (negative costs never converge)
                        charge_visits(a, 64ull);
                        nvis = 0;
                    }
                }
            }
        } else if (threadIdx.x < 128 && (a.bctl || threadIdx.x == 64)) {
            // wave 1 takes the next tile (priority bands: the whole wave; else lane 64)
            unsigned trig = 0;
            const int t = a.bctl ? qgrab_prio(a, trig) : qgrab(a, trig);
            if (threadIdx.x == 64) {
                L.tile = t;
                L.dirs = sweep_dirs(trig);
                L.fresh = !(trig & kVisited);
            }
        }
        __syncthreads();
        tile = __builtin_amdgcn_readfirstlane(L.tile);
        if (tile < 0) break;
        process_tile_layered<R, NL, true>(a, tile, L, keep);
    }
    if (threadIdx.x == 0 && nvis) atomicAdd(a.visits, (unsigned long long)nvis);
}

template <typename R>
__global__ void fim2dl_init_kernel(R* __restrict__ T, int64_t n, unsigned* __restrict__ qstate, int64_t ntiles,
                                   unsigned* __restrict__ qslot, int64_t nslots) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) T[i] = Real<R>::inf();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ntiles; i += stride) qstate[i] = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += stride) qslot[i] = 0;
}

// T[goal] = 0 (gz: absolute layer index) and the goal's tile (th rows) queued
template <typename R>
__global__ void fim2dl_seed_kernel(Fim2dArgs a, int64_t gx, int64_t gy, int64_t gz, int th) {
    static_cast<R*>(a.T)[(gy * a.W + gx) * a.ls + a.z0 + gz * a.lzs] = R(0);  // gz: the solved layer's index
    __threadfence();
    qpush(a, (int)(gy / th) * a.ntx + (int)(gx / kTile), kSelf | kVisited);  // T not all +inf
}


// flag |= 1 if layer z of the [HW][L] volume holds a finite cost
template <typename R>
__global__ void layer_finite_kernel(const R* __restrict__ cost, int64_t hw, int64_t L, int64_t z, int* flag) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    bool any = false;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < hw; i += stride)
        any |= cost[i * L + z] != Real<R>::inf();
    if (__any(any) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

// Layer-planar working copies (EIK_LAYER_PLANAR, solve_layered): the planner's volumes are
// [y][x][L] with z fastest and +inf padding layers, so a tile row's stores of its nl solved layers
// touch every line of the cells' L values (the fp32 C5 kernel wrote 1.69x its algorithmic bytes,
// profiles/pmc_traffic_c5.json).  The solve runs on copies [nl][H][W] instead (every tile-row load
// and store one contiguous run per layer), the cost copied in and the field copied out once.
template <typename R>
__global__ void layer_planar_in_kernel(const R* __restrict__ vol, int64_t hw, int64_t L, int z0, int nl,
                                       R* __restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < hw; c += stride)
        for (int z = 0; z < nl; ++z) out[z * hw + c] = vol[c * L + z0 + z];
}
// the whole cell: the solved layers from the copy, +inf elsewhere (the padding's field) -- the
// volume's lines are written whole
template <typename R>
__global__ void layer_planar_out_kernel(const R* __restrict__ pl, int64_t hw, int64_t L, int z0, int nl,
                                        R* __restrict__ vol) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < hw * L; i += stride) {
        const int64_t c = i / L;
        const int z = (int)(i - c * L) - z0;
        vol[i] = (z >= 0 && z < nl) ? pl[z * hw + c] : Real<R>::inf();
    }
}
hipError_t layer_planar(const void* src, void* dst, bool f64, int64_t hw, int64_t L, int z0, int nl, bool in,
                        hipStream_t st) {
    const int grid = (int)std::min<int64_t>(8192, (hw * (in ? 1 : L) + 255) / 256);
    if (f64) {
        if (in)
            hipLaunchKernelGGL(layer_planar_in_kernel<double>, dim3(grid), dim3(256), 0, st,
                               static_cast<const double*>(src), hw, L, z0, nl, static_cast<double*>(dst));
        else
            hipLaunchKernelGGL(layer_planar_out_kernel<double>, dim3(grid), dim3(256), 0, st,
                               static_cast<const double*>(src), hw, L, z0, nl, static_cast<double*>(dst));
    } else {
        if (in)
            hipLaunchKernelGGL(layer_planar_in_kernel<float>, dim3(grid), dim3(256), 0, st,
                               static_cast<const float*>(src), hw, L, z0, nl, static_cast<float*>(dst));
        else
            hipLaunchKernelGGL(layer_planar_out_kernel<float>, dim3(grid), dim3(256), 0, st,
                               static_cast<const float*>(src), hw, L, z0, nl, static_cast<float*>(dst));
    }
    return hipGetLastError();
}

// Domain decomposition of a layered volume ("C5: split x-y only, layers stay
// together"): a rank's edge rows / columns, nl values per edge cell ([i][z]), into send strips ...
template <typename R>
__global__ void fim2dl_pack_edges_kernel(Fim2dArgs a, int nl, R* __restrict__ n, R* __restrict__ s,
                                         R* __restrict__ w, R* __restrict__ e) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const R* T = static_cast<const R*>(a.T);
    auto at = [&](int64_t y, int64_t x, int z) { return T[(y * a.W + x) * a.ls + a.z0 + z * a.lzs]; };
    for (int z = 0; z < nl; ++z) {
        if (i < a.W) {
            if (n) n[i * nl + z] = at(0, i, z);
            if (s) s[i * nl + z] = at(a.H - 1, i, z);
        }
        if (i < a.H) {
            if (w) w[i * nl + z] = at(i, 0, z);
            if (e) e[i * nl + z] = at(i, a.W - 1, z);
        }
    }
}
// ... and the received strips min-merged into the ghosts; an edge cell whose ghost dropped in any
// layer queues its tile (th: tile rows) for the next launch
template <typename R>
__global__ void fim2dl_merge_ghost_kernel(Fim2dArgs a, int nl, int th, int side, const R* __restrict__ recv,
                                          int64_t len) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= len) return;
    R* g = static_cast<R*>(const_cast<void*>(a.ghost[side]));
    bool dropped = false;
    for (int z = 0; z < nl; ++z) {
        const R v = recv[i * nl + z];
        if (v < g[i * nl + z]) {
            g[i * nl + z] = v;
            dropped = true;
        }
    }
    if (!dropped) return;
    const int ty = side < 2 ? (side == 0 ? 0 : a.nty - 1) : (int)(i / th);
    const int tx = side < 2 ? (int)(i / kTile) : (side == 2 ? 0 : a.ntx - 1);
    qpush(a, ty * a.ntx + tx, kFromN << side);
}

hipError_t fim2dl_pack_edges(const Fim2dArgs& a, int nl, bool f64, void* n, void* s, void* w, void* e, hipStream_t st) {
    const int64_t len = a.H > a.W ? a.H : a.W;
    const int grid = (int)((len + 255) / 256);
    if (f64)
        hipLaunchKernelGGL(fim2dl_pack_edges_kernel<double>, dim3(grid), dim3(256), 0, st, a, nl, (double*)n,
                           (double*)s, (double*)w, (double*)e);
    else
        hipLaunchKernelGGL(fim2dl_pack_edges_kernel<float>, dim3(grid), dim3(256), 0, st, a, nl, (float*)n, (float*)s,
                           (float*)w, (float*)e);
    return hipGetLastError();
}

hipError_t fim2dl_merge_ghost(const Fim2dArgs& a, int nl, bool f64, int side, const void* recv, hipStream_t st) {
    const int64_t len = side < 2 ? a.W : a.H;
    const int grid = (int)((len + 255) / 256);
    if (f64)
        hipLaunchKernelGGL(fim2dl_merge_ghost_kernel<double>, dim3(grid), dim3(256), 0, st, a, nl, kRowsOf<double>,
                           side, static_cast<const double*>(recv), len);
    else
        hipLaunchKernelGGL(fim2dl_merge_ghost_kernel<float>, dim3(grid), dim3(256), 0, st, a, nl, kRowsOf<float>, side,
                           static_cast<const float*>(recv), len);
    return hipGetLastError();
}

// ------------------------------------------------------------------------- host launchers
int fim2dl_rows(bool f64) { return f64 ? kRowsOf<double> : kRowsOf<float>; }

// gz: the goal's layer among the solved ones (0 .. nl-1); n: T's elements to set to +inf
hipError_t fim2dl_init(const Fim2dArgs& a, bool f64, int64_t gx, int64_t gy, int64_t gz, int64_t n, hipStream_t st) {
    const int64_t nslots = (int64_t)a.qmask + 1;
    const int grid = (int)std::min<int64_t>(4096, (std::max(n, nslots) + 255) / 256);
    hipError_t e = hipMemsetAsync(a.qhead, 0, kQueueCtlBytes, st);  // head tail active error
    if (e != hipSuccess) return e;
    // (gx < 0: no goal in this block -- a domain-decomposed volume's other ranks)
    if (f64) {
        hipLaunchKernelGGL(fim2dl_init_kernel<double>, dim3(grid), dim3(256), 0, st, static_cast<double*>(a.T), n,
                           a.qstate, (int64_t)a.tiles_per_map, a.qslot, nslots);
        if (gx >= 0)
            hipLaunchKernelGGL(fim2dl_seed_kernel<double>, dim3(1), dim3(1), 0, st, a, gx, gy, gz, kRowsOf<double>);
    } else {
        hipLaunchKernelGGL(fim2dl_init_kernel<float>, dim3(grid), dim3(256), 0, st, static_cast<float*>(a.T), n,
                           a.qstate, (int64_t)a.tiles_per_map, a.qslot, nslots);
        if (gx >= 0)
            hipLaunchKernelGGL(fim2dl_seed_kernel<float>, dim3(1), dim3(1), 0, st, a, gx, gy, gz, kRowsOf<float>);
    }
    return hipGetLastError();
}

template <typename R, int NL>
static int resident_of(int cus) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fim2dl_persist_kernel<R, NL>, kLThreads<R, NL>, 0) != hipSuccess ||
        per_cu < 1)
        per_cu = 1;
    return per_cu * cus;
}

int fim2dl_persist_resident(int nl, bool f64, int cus) {
    if (f64) {
        switch (nl) {
            case 1: return resident_of<double, 1>(cus);
            case 2: return resident_of<double, 2>(cus);
            default: return resident_of<double, 3>(cus);
        }
    }
    switch (nl) {
        case 1: return resident_of<float, 1>(cus);
        case 2: return resident_of<float, 2>(cus);
        case 3: return resident_of<float, 3>(cus);
        default: return resident_of<float, 4>(cus);
    }
}

hipError_t fim2dl_persist(const Fim2dArgs& a, int nl, bool f64, int grid, hipStream_t st) {
    if (f64) {
        switch (nl) {
            case 1: hipLaunchKernelGGL((fim2dl_persist_kernel<double, 1>), dim3(grid), dim3(kLThreads<double, 1>), 0, st, a); break;
            case 2: hipLaunchKernelGGL((fim2dl_persist_kernel<double, 2>), dim3(grid), dim3(kLThreads<double, 2>), 0, st, a); break;
            case 3: hipLaunchKernelGGL((fim2dl_persist_kernel<double, 3>), dim3(grid), dim3(kLThreads<double, 3>), 0, st, a); break;
            default: return hipErrorInvalidValue;
        }
    } else {
        switch (nl) {
            case 1: hipLaunchKernelGGL((fim2dl_persist_kernel<float, 1>), dim3(grid), dim3(kLThreads<float, 1>), 0, st, a); break;
            case 2: hipLaunchKernelGGL((fim2dl_persist_kernel<float, 2>), dim3(grid), dim3(kLThreads<float, 2>), 0, st, a); break;
            case 3: hipLaunchKernelGGL((fim2dl_persist_kernel<float, 3>), dim3(grid), dim3(kLThreads<float, 3>), 0, st, a); break;
            case 4: hipLaunchKernelGGL((fim2dl_persist_kernel<float, 4>), dim3(grid), dim3(kLThreads<float, 4>), 0, st, a); break;
            default: return hipErrorInvalidValue;
        }
    }
    // the queue rewind of fim2d.hip (with bands: FIFO leftovers of the last dispatch dropped, bits cleared)
    return fim2d_qrewind(a, st);
}

hipError_t layer_finite(const void* cost, bool f64, int64_t hw, int64_t L, int64_t z, int* d_flag, hipStream_t st) {
    const int grid = (int)std::min<int64_t>(2048, (hw + 255) / 256);
    if (f64)
        hipLaunchKernelGGL(layer_finite_kernel<double>, dim3(grid), dim3(256), 0, st, static_cast<const double*>(cost), hw,
                           L, z, d_flag);
    else
        hipLaunchKernelGGL(layer_finite_kernel<float>, dim3(grid), dim3(256), 0, st, static_cast<const float*>(cost), hw,
                           L, z, d_flag);
    return hipGetLastError();
}

}  // namespace eik
