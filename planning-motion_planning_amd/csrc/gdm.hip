// gdm.hip -- gradient-descent path extraction (getPathGDM, FastMarching.py:164-236) and the
// inf-aware normalised gradient (computeGradient, FastMarching.py:242-300) on gfx950.
//
// The path is inherently sequential (<= round(15000/tau) dependent steps), so it runs as ONE
// small kernel: a single wave whose lane 0 walks the field.  Per step the reference builds the
// normalised gradient in a 6x6 window (allocating four full-size arrays, :255-258) but only ever
// reads it at the four bilinear corners; the kernel evaluates the gradient at exactly those
// four corners (bit-identical control flow, see oracle/eikonal_oracle.c grad_at/orc_gdm2d).
//
// Arithmetic is IEEE fp64 with contraction disabled.  The one deliberate difference: the
// reference squares numpy scalars with `x**2`, which goes through glibc pow() and is not
// always correctly rounded; the device uses the exact product x*x (<= 1 ulp per square,
// tolerance stated in tests/test_gpu_path.py).
#include "eik_common.hpp"
#include "eik_kernels.hpp"

#pragma clang fp contract(off)

namespace eik {

template <typename R>
__device__ __forceinline__ double tv(const R* __restrict__ T, int64_t W, int64_t j, int64_t i) {
    return (double)T[j * W + i];
}

// computeGradient body at one (j, i), FastMarching.py:262-297
template <typename R>
__device__ void grad_at(const R* __restrict__ T, int64_t m, int64_t n, int64_t j, int64_t i, double& gnx, double& gny) {
    double gy, gx;
    if (j == 0)
        gy = tv(T, n, 1, i) - tv(T, n, 0, i);
    else if (j == m - 1)
        gy = tv(T, n, j, i) - tv(T, n, j - 1, i);
    else if (__builtin_isinf(tv(T, n, j + 1, i)))
        gy = __builtin_isinf(tv(T, n, j - 1, i)) ? 0.0 : tv(T, n, j, i) - tv(T, n, j - 1, i);
    else
        gy = __builtin_isinf(tv(T, n, j - 1, i)) ? tv(T, n, j + 1, i) - tv(T, n, j, i)
                                                 : (tv(T, n, j + 1, i) - tv(T, n, j - 1, i)) / 2;
    if (i == 0)
        gx = tv(T, n, j, 1) - tv(T, n, j, 0);
    else if (i == n - 1)
        gx = tv(T, n, j, i) - tv(T, n, j, i - 1);
    else if (__builtin_isinf(tv(T, n, j, i + 1)))
        gx = __builtin_isinf(tv(T, n, j, i - 1)) ? 0.0 : tv(T, n, j, i) - tv(T, n, j, i - 1);
    else
        gx = __builtin_isinf(tv(T, n, j, i - 1)) ? tv(T, n, j, i + 1) - tv(T, n, j, i)
                                                 : (tv(T, n, j, i + 1) - tv(T, n, j, i - 1)) / 2;
    const double den = __builtin_sqrt(gx * gx + gy * gy);
    gnx = gx / den;
    gny = gy / den;
}

// interpolatePoint FastMarching.py:305-338 on a 2x2 patch g[jj][ii]
__device__ __forceinline__ double interp2_patch(double a, double b, const double (&g)[2][2]) {
    const double a00 = g[0][0];
    const double a10 = g[0][1] - g[0][0];
    const double a01 = g[1][0] - g[0][0];
    const double a11 = g[1][1] + g[0][0] - g[0][1] - g[1][0];
    if (a == 0) return b == 0 ? a00 : a00 + a01 * b;
    return b == 0 ? a00 + a10 * a : a00 + a10 * a + a01 * b + a11 * a * b;
}

// interp2_patch with the four cases of :327-336 evaluated and selected (no divergent branches on
// the walker's critical path; same operations in the same order as each case)
__device__ __forceinline__ double interp2_sel(double a, double b, double g00, double g01, double g10, double g11) {
    const double a00 = g00;
    const double a10 = g01 - g00;
    const double a01 = g10 - g00;
    const double a11 = g11 + g00 - g01 - g10;
    const double ra = a00 + a10 * a;            // b == 0
    const double rb = a00 + a01 * b;            // a == 0
    const double rf = ra + a01 * b + a11 * a * b;
    // bitwise selects: the compiler turns the ?: form into branches on the walker's chain
    const long long za = -(long long)(a == 0), zb = -(long long)(b == 0);
    const long long r0 = (__double_as_longlong(rb) & ~zb) | (__double_as_longlong(a00) & zb);   // a == 0
    const long long r1 = (__double_as_longlong(rf) & ~zb) | (__double_as_longlong(ra) & zb);    // a != 0
    return __longlong_as_double((r1 & ~za) | (r0 & za));
}

__device__ __forceinline__ double norm2(double a, double b) { return __builtin_sqrt(a * a + b * b); }

// Correctly rounded f64 square root and division exactly as the compiler lowers them for gfx950,
// minus the range handling: the same operations in the same order, so the same bits wherever
// that handling is the identity.  sqrt: the input scaling (x < 2^-767) and its undo are
// identities for x >= 2^-767 (and the compiler's final select, which keeps +-0 and +inf, is one
// for finite x > 0, so it is left out: the walker never takes x = 0 or +inf here).  n / d: v_div_scale_f64 leaves
// both operands as they are and v_div_fmas_f64 is a plain fma when d is normal in
// [2^-900, 2^100], n is 0 or normal with |n| >= 2^-900 and |n| <= |d|; v_div_fixup_f64 then only
// forces the sign of the quotient to sign(n) ^ sign(d), which it already has -- except a zero
// quotient of n = -0, which comes out +0 here (only ever squared or subtracted later: same path
// bits).  The walker takes these on its fast path and leaves it for the exact forms outside
// that domain (walk_odd).
__device__ __forceinline__ double sqrt_core(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = y * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    return __builtin_fma(d, h, g);
}
// sqrt_core that also hands out its refined half reciprocal hh ~ 1 / (2 sqrt(x)) (one
// Goldschmidt update of v_rsq_f64's estimate: ~2^-44 relative or better).  Same bits as sqrt_core.
__device__ __forceinline__ double sqrt_core_h(double x, double& hh) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = y * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    hh = h;
    double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    return __builtin_fma(d, h, g);
}
// sqrt_core_h with ONE residual correction after the Goldschmidt update instead of two: g is
// within ~2^-43 of sqrt(x) there, so g + (x - g^2) h is within ~2^-86 and the final fma rounds it
// as the correctly rounded root unless sqrt(x) lies that close to a rounding midpoint (~2^-33 of
// roots; an exact midpoint is impossible).  Checked bit for bit against sqrt by
// walker_math_selftest_kernel (counts[5]) on the walker's domain x in [2^-767, 2^200].  Two
// dependent operations shorter: the lane-pair walker's chain (LOOP 4) holds two of them per step.
__device__ __forceinline__ double sqrt_c1_h(double x, double& hh) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = y * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    hh = h;
    const double d = __builtin_fma(-g, g, x);
    return __builtin_fma(d, h, g);
}
// n / d for d = sqrt_core_h(x, h), from the reciprocal 2h the square root already holds: q0 =
// n * 2h is formed while the root is still being refined, and ONE residual correction (e = n -
// d q0 by fma, q0 + e 2h by fma) leaves two dependent operations after d instead of div_core's
// eight.  The exact sum q0 + e 2h is within ~2^-86 (relative) of n / d, so the final fma rounds it
// as the correctly rounded quotient unless n / d lies that close to a rounding midpoint (~2^-33
// of quotients): checked bit for bit against n / d by walker_math_selftest_kernel (counts[4]) on
// the walker's domain (d = sqrt(x), x in [2^-767, 2^200], |n| <= d, n = 0 or |n| >= 2^-900).
__device__ __forceinline__ double div_rs(double n, double d, double h) {
    const double r = h + h;  // exact
    const double q0 = n * r;
    const double e = __builtin_fma(-d, q0, n);
    return __builtin_fma(e, r, q0);
}
__device__ __forceinline__ double div_core(double n, double d) {
    double r = __builtin_amdgcn_rcp(d);
    double e = __builtin_fma(-d, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-d, r, 1.0);
    r = __builtin_fma(r, e, r);
    const double q = n * r;
    e = __builtin_fma(-d, q, n);
    return __builtin_fma(e, r, q);
}
// interpolatePoint's general case (:336) for every (a, b): where a == 0 or b == 0 it equals the
// special cases of :327-334 bit for bit (the skipped terms are exact zeros added to a nonzero
// sum; only the sign of a zero result can differ) as long as the four corners are finite; a NaN
// corner makes |g|^2 NaN, and walk_odd sends the step to the exact form.
__device__ __forceinline__ double interp2_general(double a, double b, double g00, double g01, double g10, double g11) {
    const double a10 = g01 - g00, a01 = g10 - g00, a11 = g11 + g00 - g01 - g10;
    return g00 + a10 * a + a01 * b + a11 * a * b;
}
// The step's operands leave the domain of sqrt_core / div_core: |g|^2 outside [2^-767, 2^200]
// or not finite, or an interpolated component that is nonzero but below 2^-900 in magnitude.
// (With |g|^2 >= 2^-767 every divisor is >= 2^-383; with |g|^2 <= 2^200 both divisors, |g| and
// sqrt(dx_n^2 + dy^2) <= |g| + 1, stay <= 2^100, the range div_core's argument and the self-test
// cover; in the |g| >= 0.01 branch dx_n^2 + dy^2 >= 5e-5.)
__device__ __forceinline__ bool walk_odd(double dx, double dy, double s1) {
    const double lo = 0x1p-767, big = 0x1p200, tiny = 0x1p-900;
    return !(s1 >= lo && s1 <= big) | ((dx != 0.0) & (__builtin_fabs(dx) < tiny)) |
           ((dy != 0.0) & (__builtin_fabs(dy) < tiny));
}

// DPP quad_perm moves of a double, the 2D walker's lane-pair form: Q = 0xB1 [1, 0, 3, 2] the
// partner lane's value (lane ^ 1), 0xA0 [0, 0, 2, 2] the even lane's, 0xF5 [1, 1, 3, 3] the odd one's
template <int Q>
__device__ __forceinline__ double quad_perm_f64(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)b, Q, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(b >> 32), Q, 0xf, 0xf, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double pair_swap(double v) { return quad_perm_f64<0xB1>(v); }

__device__ __forceinline__ double readlane_f64(double v, int l) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

enum { kGdmDone = 0, kGdmFallback = 1, kGdmError = 2 };
#ifndef EIK_P3PROBE
#define EIK_P3PROBE(k) ((void)0)  // 3D walker phase timing hooks (tools/path3_prof.hip)
#define EIK_P3DECL ((void)0)
#define EIK_P3FLUSH ((void)0)
#endif
#ifndef EIK_P3RUN
#define EIK_P3RUN 1  // the 3D walker's integer-descent run loop (gdm3d_kernel)
#endif
#ifndef EIK_P2PROBE
#define EIK_P2PROBE(k) ((void)0)  // 2D walker phase timing hooks (tools/path2_prof.hip)
#define EIK_P2DECL ((void)0)
#define EIK_P2FLUSH ((void)0)
#endif

// Path kernel layout: ONE workgroup of 16 waves.  Wave 0 is the walker: it runs the reference
// loop (:173-232) step by step, reading the inf-aware normalised gradient (Gnx, Gny) of the four
// bilinear corners from an LDS window of 64 x 64 nodes.  Waves 1..15 are builders: they compute
// the gradient of a window (computeGradient's body, :262-297, at every node of the window) from
// T in HBM into one of two LDS buffers.  When the walker comes within kPrefetch nodes of an
// inner window edge it requests the window centred on itself into the idle buffer and keeps
// walking; when it leaves the current window it switches (waiting only if the build is still
// running, or if it turned away from the prefetched window).  The gradient at a node depends on
// T only, so precomputing it is exactly the reference's per-step computeGradient evaluated
// earlier: the path is bit-identical to the single-lane form.
constexpr int kPW = 64;                          // window side (nodes), one builder lane per column
constexpr int kPathThreads = 1024;               // 16 waves: walker + 15 builders
// (Round 4, measured and removed: EIK_PATH_SIMD0_FREE -- the waves sharing the walker's SIMD (4, 8,
// 12) did not build, so builds never took the walker's issue slots.  Walk 2.512-2.532 ms against
// 2.513-2.527 ms, 0.406-0.410 us/step both (profiles/r04g_walker_simd0_ab.log): the walker's step
// is its own dependent f64 chain, not issue-bound.)
constexpr int kBuilders = kPathThreads / 64 - 1;
constexpr int kRowsPerBuilder = (kPW + kBuilders - 1) / kBuilders;
constexpr int kPrefetch = 16;                    // nodes from an inner edge that trigger a prefetch
constexpr unsigned long long kPathSpin = 200000000ull;  // 2 s of s_memrealtime (100 MHz): never hang

struct PathLds {
    double2 g[2][kPW][kPW];  // (Gnx, Gny) per node, 2 x 64 KiB
    long long req_x0, req_y0;
    int req_seq;             // walker -> builders: request number (-1: quit)
    int req_b;               // target buffer of the request
    int done;                // builders -> walker: finished builds x kBuilders
};

// Builder wave `w` fills rows w, w + kBuilders, ... of window buffer b (origin x0, y0).  Every T
// load of a wave is issued before any is used (5 neighbours x kRowsPerBuilder rows per lane), so
// a build costs about one HBM/L2 round trip plus the arithmetic.
template <typename R>
__device__ void build_window(PathLds& s, const R* __restrict__ T, int64_t H, int64_t W, int b, int64_t x0,
                             int64_t y0, int w) {
    const int lane = threadIdx.x & 63;
    const int64_t i = x0 + lane;
    const bool col_ok = i < W;
    const int64_t ic = col_ok ? i : W - 1;
    const int64_t iw = ic > 0 ? ic - 1 : 0, ie = ic + 1 < W ? ic + 1 : W - 1;
    double c[kRowsPerBuilder], nn[kRowsPerBuilder], ss[kRowsPerBuilder], ww[kRowsPerBuilder], ee[kRowsPerBuilder];
#pragma unroll
    for (int k = 0; k < kRowsPerBuilder; ++k) {
        const int r = w + k * kBuilders;
        int64_t j = y0 + r;
        j = (r < kPW && j < H) ? j : H - 1;
        const int64_t jn = j > 0 ? j - 1 : 0, js = j + 1 < H ? j + 1 : H - 1;
        c[k] = (double)T[j * W + ic];
        nn[k] = (double)T[jn * W + ic];
        ss[k] = (double)T[js * W + ic];
        ww[k] = (double)T[j * W + iw];
        ee[k] = (double)T[j * W + ie];
    }
#pragma unroll
    for (int k = 0; k < kRowsPerBuilder; ++k) {
        const int r = w + k * kBuilders;
        const int64_t j = y0 + r;
        if (r >= kPW || j >= H || !col_ok) continue;
        double gy, gx;  // FastMarching.py:262-294 with the five loaded values
        if (j == 0)
            gy = ss[k] - c[k];
        else if (j == H - 1)
            gy = c[k] - nn[k];
        else if (__builtin_isinf(ss[k]))
            gy = __builtin_isinf(nn[k]) ? 0.0 : c[k] - nn[k];
        else
            gy = __builtin_isinf(nn[k]) ? ss[k] - c[k] : (ss[k] - nn[k]) / 2;
        if (i == 0)
            gx = ee[k] - c[k];
        else if (i == W - 1)
            gx = c[k] - ww[k];
        else if (__builtin_isinf(ee[k]))
            gx = __builtin_isinf(ww[k]) ? 0.0 : c[k] - ww[k];
        else
            gx = __builtin_isinf(ww[k]) ? ee[k] - c[k] : (ee[k] - ww[k]) / 2;
        const double den = __builtin_sqrt(gx * gx + gy * gy);  // :296-297
        s.g[b][r][lane] = make_double2(gx / den, gy / den);
    }
}

template <typename R>
__device__ void path_builder(PathLds& s, const R* __restrict__ T, int64_t H, int64_t W) {
    const int wv = (int)(threadIdx.x >> 6);
    const int w = wv - 1;  // builder index 0 .. kBuilders - 1
    int seen = 0;
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        const int q = __hip_atomic_load(&s.req_seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (q < 0) return;
        if (q == seen) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > kPathSpin) return;  // walker gone: give up
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        seen = q;
        build_window<R>(s, T, H, W, s.req_b, s.req_x0, s.req_y0, w);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(&s.done, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        t0 = __builtin_amdgcn_s_memrealtime();
    }
}

template <typename R, int LOOP>
__global__ __launch_bounds__(kPathThreads) void gdm2d_kernel(Gdm2dArgs a) {
    __shared__ PathLds s;
    const R* __restrict__ T = static_cast<const R*>(a.T);
    const int64_t H = a.H, W = a.W;
    if (threadIdx.x == 0) {
        s.req_seq = 0;
        s.done = 0;
    }
    __syncthreads();
    if (threadIdx.x >= 64) {
        path_builder<R>(s, T, H, W);
        return;
    }
    // ---- walker (wave 0; every lane runs the same uniform loop, lane 0 stores)
    EIK_P2DECL;
    const bool lead = threadIdx.x == 0;
    double* out = a.out;
    int status = kGdmDone;
    double px = a.ix, py = a.iy;  // gamma[-1], kept in registers
    if (lead) {
        out[0] = px;
        out[1] = py;
    }
    int64_t n = 1;
    const double tau = a.tau;
    // window origins of the two buffers (scalars, not an indexed array: no private->LDS promotion)
    int64_t wx0 = -((int64_t)1 << 40), wx1 = wx0, wy0 = wx0, wy1 = wx0;
    int cur = 0, seq = 0;
    bool pending = false;
    const int64_t xmax = W > kPW ? W - kPW : 0, ymax = H > kPW ? H - kPW : 0;
    auto issue = [&](int b, int64_t i, int64_t j) {  // build the window centred on (i, j) into b
        int64_t x0 = i - kPW / 2, y0 = j - kPW / 2;
        x0 = x0 > xmax ? xmax : x0 < 0 ? 0 : x0;
        y0 = y0 > ymax ? ymax : y0 < 0 ? 0 : y0;
        if (b) { wx1 = x0; wy1 = y0; } else { wx0 = x0; wy0 = y0; }
        s.req_x0 = x0;
        s.req_y0 = y0;
        s.req_b = b;
        __hip_atomic_store(&s.req_seq, ++seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    auto wait_built = [&]() -> bool {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(&s.done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < seq * kBuilders) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > kPathSpin) return false;
            __builtin_amdgcn_s_sleep(1);
        }
        return true;
    };
    auto inside = [&](int b, int64_t i, int64_t j) {
        const int64_t x0 = b ? wx1 : wx0, y0 = b ? wy1 : wy0;
        return i >= x0 && j >= y0 && i + 1 < x0 + kPW && j + 1 < y0 + kPW;
    };
    // Fast path: while lo_x <= i <= hi_x and lo_y <= j <= hi_y nothing has to happen this step
    // (the corners lie in the current window and, unless a build is pending, not within
    // kPrefetch of an inner edge) -- four int32 compares on the step's dependency chain instead
    // of the window bookkeeping, which runs only when the bounds are crossed.
    int lo_x = 1, hi_x = 0, lo_y = 1, hi_y = 0;  // empty: the first step takes the slow path
    int cx0i = 0, cy0i = 0;                     // current window origin
    auto set_bounds = [&]() {
        const int64_t x0 = cur ? wx1 : wx0, y0 = cur ? wy1 : wy0;
        cx0i = (int)x0;
        cy0i = (int)y0;
        lo_x = cx0i + (!pending && x0 > 0 ? kPrefetch : 0);
        hi_x = cx0i + kPW - 2 - (!pending && x0 < xmax ? kPrefetch : 0);
        lo_y = cy0i + (!pending && y0 > 0 ? kPrefetch : 0);
        hi_y = cy0i + kPW - 2 - (!pending && y0 < ymax ? kPrefetch : 0);
        hi_x = hi_x < (int)W - 2 ? hi_x : (int)W - 2;  // inside the bounds implies i + 1 < W, j + 1 < H
        hi_y = hi_y < (int)H - 2 ? hi_y : (int)H - 2;
    };
    // Window bookkeeping of a step whose cell (i, j) left the fast bounds: errors (NaN point, out
    // of range) set status and return false; else the corners are in window `cur` afterwards.
    auto slow_step = [&](uint32_t i, uint32_t j) -> bool {
        if (__builtin_isnan(px) || __builtin_isnan(py)) { status = kGdmError; return false; }
        if (i + 1 >= (uint64_t)W || j + 1 >= (uint64_t)H) { status = kGdmError; return false; }
        if (!inside(cur, i, j)) {  // the 2 x 2 interpolation corners left the window
            const int nb = seq == 0 ? 0 : 1 - cur;
            bool have = false;
            if (pending) {
                pending = false;
                if (!wait_built()) { status = kGdmError; return false; }
                have = inside(nb, i, j);
            }
            if (!have) {
                issue(nb, i, j);
                if (!wait_built()) { status = kGdmError; return false; }
            }
            cur = nb;
        }
        const int64_t cx0 = cur ? wx1 : wx0, cy0 = cur ? wy1 : wy0;
        if (!pending && ((i - cx0 < kPrefetch && cx0 > 0) || (cx0 + kPW - 2 - i < kPrefetch && cx0 < xmax) ||
                         (j - cy0 < kPrefetch && cy0 > 0) || (cy0 + kPW - 2 - j < kPrefetch && cy0 < ymax))) {
            issue(1 - cur, i, j);
            pending = true;
        }
        set_bounds();
        return true;
    };
    // NaN fallback (:178-218) as the reference behaves under numpy 2: the neighbour probe
    // `np.uint32(nearN + [0,-1])` raises OverflowError, caught at :217.  Lane 0 edits the path.
    auto nan_fallback = [&]() {
        if (lead) {
            int64_t nx = (int64_t)__builtin_rint(px), ny = (int64_t)__builtin_rint(py);
            bool empty = false, oob = false;
            for (;;) {
                const int64_t qx = nx < 0 ? nx + W : nx, qy = ny < 0 ? ny + H : ny;
                if (qx < 0 || qy < 0 || qx >= W || qy >= H) { oob = true; break; }
                if (!__builtin_isinf(tv(T, W, qy, qx))) break;
                --n;
                if (n == 0) { empty = true; break; }
                nx = (int64_t)__builtin_rint(out[2 * (n - 1)]);
                ny = (int64_t)__builtin_rint(out[2 * (n - 1) + 1]);
            }
            if (!empty && !oob) {
                while (n > 0 && norm2(out[2 * (n - 1)] - (double)nx, out[2 * (n - 1) + 1] - (double)ny) < 1) --n;
                if (n < a.cap) {
                    out[2 * n] = (double)nx;
                    out[2 * n + 1] = (double)ny;
                    ++n;
                }
            }
        }
        status = kGdmFallback;
    };
    // One step's arithmetic from the four corners (g00, g01, g10, g11) of cell (i, j):
    // :175-176 interpolation, :220-229 normalisation, :230 step.
    struct StepOut {
        double dx, dy, sx, sy;
    };
    auto step_math = [&](const double2& g00, const double2& g01, const double2& g10, const double2& g11, double fa,
                         double fb) -> StepOut {
        StepOut o;
        o.dx = interp2_sel(fa, fb, g00.x, g01.x, g10.x, g11.x);  // :175
        o.dy = interp2_sel(fa, fb, g00.y, g01.y, g10.y, g11.y);  // :176
        // |(dx, dy)| is the same value in the test (:220) and both normalisations (:221-227)
        const double nrm = __builtin_sqrt(o.dx * o.dx + o.dy * o.dy);
        const double dxn = o.dx / nrm;  // both branches
        // :220-224 (|g| < 0.01: unit step) or :225-229 (dy normalised with the normalised dx)
        const double dyn = nrm < 0.01 ? o.dy / nrm : o.dy / __builtin_sqrt(dxn * dxn + o.dy * o.dy);
        o.sx = px - tau * dxn;
        o.sy = py - tau * dyn;
        return o;
    };
    // step_math with interp2_general, sqrt_core and div_core (same bits where walk_odd is false,
    // set in `odd`)
    auto step_math_core = [&](const double2& g00, const double2& g01, const double2& g10, const double2& g11, double fa,
                              double fb, bool& odd) -> StepOut {
        StepOut o;
        o.dx = interp2_general(fa, fb, g00.x, g01.x, g10.x, g11.x);
        o.dy = interp2_general(fa, fb, g00.y, g01.y, g10.y, g11.y);
        const double s1 = o.dx * o.dx + o.dy * o.dy;
        const double nrm = sqrt_core(s1);
        const double dxn = div_core(o.dx, nrm);
        // both divisors computed, selected bitwise (a ?: here becomes a branch on the chain)
        const double r2 = sqrt_core(dxn * dxn + o.dy * o.dy);
        const long long small = -(long long)(nrm < 0.01);
        const double den = __longlong_as_double((__double_as_longlong(nrm) & small) | (__double_as_longlong(r2) & ~small));
        const double dyn = div_core(o.dy, den);
        o.sx = px - tau * dxn;
        o.sy = py - tau * dyn;
        odd = walk_odd(o.dx, o.dy, s1);
        return o;
    };
    // step_math_core with the divisions taken from the square roots' reciprocals (div_rs): the
    // step's dependent f64 chain 45 -> 33 operations (LOOP 3)
    auto step_math_rs = [&](const double2& g00, const double2& g01, const double2& g10, const double2& g11, double fa,
                            double fb, bool& odd) -> StepOut {
        StepOut o;
        o.dx = interp2_general(fa, fb, g00.x, g01.x, g10.x, g11.x);
        o.dy = interp2_general(fa, fb, g00.y, g01.y, g10.y, g11.y);
        const double s1 = o.dx * o.dx + o.dy * o.dy;
        double h1, h2;
        const double nrm = sqrt_core_h(s1, h1);
        const double dxn = div_rs(o.dx, nrm, h1);
        const double r2 = sqrt_core_h(dxn * dxn + o.dy * o.dy, h2);
        const long long small = -(long long)(nrm < 0.01);
        const double den = __longlong_as_double((__double_as_longlong(nrm) & small) | (__double_as_longlong(r2) & ~small));
        const double hd = __longlong_as_double((__double_as_longlong(h1) & small) | (__double_as_longlong(h2) & ~small));
        const double dyn = div_rs(o.dy, den, hd);
        o.sx = px - tau * dxn;
        o.sy = py - tau * dyn;
        odd = walk_odd(o.dx, o.dy, s1);
        return o;
    };
    // the point budget folded into the step count: point n = k + 1 is stored at step k (:173)
    const long kmax = a.steps < a.cap - 1 ? a.steps : a.cap - 1;
    long k = 0;
    if constexpr (LOOP >= 1) {
        // One exit per step: the step is computed before its special cases are known (window
        // bookkeeping due, NaN gradient, stop radius, point budget), and a single uniform branch
        // leaves the tight loop when any of them holds; the handler below then takes the same
        // decisions as the reference-structured loop (the `else` branch) for that step.  The
        // many uniform branches of that loop, each behind a VALU compare, cost more per step than
        // the arithmetic they skip.  The LDS address of a step whose cell is outside the fast
        // bounds is clamped into the window buffers (its values are discarded).
        constexpr unsigned kWinBytes = sizeof(s.g[0]);
        // LOOP 4, the lane-pair form: even lanes carry the x component of every per-component
        // quantity (coordinate, fraction, interpolated gradient, quotient), odd lanes the y one,
        // so each f64 instruction of the step does the work of both components; the few sums and
        // hand-overs across the pair are DPP moves (pair_swap).  Every lane computes the same
        // operations on the same operands as form 3 does for its component -- sums of the two
        // components (dx dx + dy dy, ex ex + ey ey) are commutative, so both lanes of a pair hold
        // the same bits -- and the exit conditions are wave-uniform votes.
        const bool yl = (threadIdx.x & 1) != 0;
        const double dmax = __builtin_fabs(tau) * 1.4142135623730951 * (1.0 + 0x1p-20) + 0x1p-20;
        double* const outl = out + (threadIdx.x & 1);
        for (; k < kmax;) {
            uint32_t i, j;
            bool in, odd = false;
            StepOut o;
            double fa, fb;
            if constexpr (LOOP == 4) {
                double p = yl ? py : px, d = 0.0, pn = 0.0;
                // this lane's fast bounds (x or y) as a half-open f64 range: lo <= p < hi + 1 (NaN
                // fails it; p in (-1, 0) goes to the handler, which is exact anyway)
                const double loc = yl ? lo_y : lo_x, hic = (yl ? hi_y : hi_x) + 1;
                // Steps this loop may take without the stop test: none of them can come within 1.5
                // of the goal (:231) -- a step moves each coordinate by at most |tau| (|dxn|, |dyn|
                // <= 1), so k steps move at most k |tau| sqrt(2) (with slack for rounding) -- and
                // within the point budget.  The step after them leaves to the handler, which tests.
                const double ex0 = px - a.ex, ey0 = py - a.ey;
                const double room = (__builtin_sqrt(ex0 * ex0 + ey0 * ey0) * (1.0 - 0x1p-30) - 1.5) / dmax;
                long kl = kmax - 1 - k;
                const long safe = room >= 1.0 ? (room < 2e9 ? (long)room : 2000000000L) : 0L;  // NaN: 0
                kl = kl < safe ? kl : safe;
                const int left = (int)kl;
                // the corners' LDS address in vector registers: each lane scales its own cell
                // index (x: 16 B per column, y: kPW x 16 B per row) and adds its partner's (DPP)
                const unsigned sc = yl ? kPW * (unsigned)sizeof(double2) : (unsigned)sizeof(double2);
                const unsigned c0 = (unsigned)(yl ? cy0i : cx0i) * sc;
                const char* const base = reinterpret_cast<const char*>(s.g[cur]) + (yl ? sizeof(double) : 0);
                int kk = 0;
                // One conditional branch per step: the point is stored and the state advanced before
                // the exit test (the stores are in range -- n < cap -- and a step the handler below
                // redoes stores its point at the same index), and the exit undoes the advance.
                double pp = p;
                bool leave;
                do {
                    // (one v_cvt_u32_f64 on p, the corner as (double)u beside it: no difference,
                    // profiles/r05k_walker_ab.log P4_CVT=1)
                    const double t = __builtin_trunc(p);
                    const uint32_t u = (uint32_t)t;
                    in = __builtin_amdgcn_ballot_w64(!(p >= loc && p < hic)) == 0ull;
                    const unsigned own = u * sc - c0;
                    unsigned off = own + (unsigned)__builtin_amdgcn_mov_dpp((int)own, 0xB1, 0xf, 0xf, false);
                    off = off < kWinBytes - (kPW + 2) * (unsigned)sizeof(double2) ? off : kWinBytes - (kPW + 2) * (unsigned)sizeof(double2);
                    const char* gq = base + off;
                    const double g00 = *reinterpret_cast<const double*>(gq);
                    const double g01 = *reinterpret_cast<const double*>(gq + sizeof(double2));
                    const double g10 = *reinterpret_cast<const double*>(gq + kPW * sizeof(double2));
                    const double g11 = *reinterpret_cast<const double*>(gq + (kPW + 1) * sizeof(double2));
                    const double f = p - t;  // fa (even) / fb (odd); in bounds t = i or j
                    fa = quad_perm_f64<0xA0>(f);
                    fb = quad_perm_f64<0xF5>(f);
                    d = interp2_general(fa, fb, g00, g01, g10, g11);  // dx (even) / dy (odd)
                    const double sq = d * d;
                    const double s1 = sq + pair_swap(sq);            // dx dx + dy dy in both lanes
                    double h1, h2;
                    const double nrm = sqrt_c1_h(s1, h1);
                    const double q1 = div_rs(d, nrm, h1);            // dxn (even) / dy / nrm (odd)
                    const double dxn = pair_swap(q1);                // odd lanes: dxn
                    const double r2 = sqrt_c1_h(dxn * dxn + sq, h2);
                    const double q2 = div_rs(d, r2, h2);             // odd lanes: dy / r2
                    const double dn = (yl && !(nrm < 0.01)) ? q2 : q1;
                    pn = p - tau * dn;                               // sx (even) / sy (odd)
                    // (a NaN d makes s1 NaN: odd)
                    const bool oddl = !(s1 >= 0x1p-767 && s1 <= 0x1p200) | ((d != 0.0) & (__builtin_fabs(d) < 0x1p-900));
                    const bool bad = __builtin_amdgcn_ballot_w64(oddl) != 0ull;
                    outl[2 * n] = pn;  // every lane: its component's address
                    leave = (int)!in | (int)bad | (int)(kk >= left);
                    ++n;
                    pp = p;
                    p = pn;
                    ++kk;
                } while (!leave);
                --n;  // the exit step is the handler's
                --kk;
                p = pp;
                k += kk;
                // the scalar state of the exit step for the handler below: lanes 0 (x) and 1 (y)
                // read into scalar registers, so the handler stays wave-uniform code
                px = readlane_f64(p, 0);
                py = readlane_f64(p, 1);
                i = (uint32_t)__builtin_trunc(px);
                j = (uint32_t)__builtin_trunc(py);
                o.dx = readlane_f64(d, 0);
                o.dy = readlane_f64(d, 1);
                o.sx = readlane_f64(pn, 0);
                o.sy = readlane_f64(pn, 1);
                odd = walk_odd(o.dx, o.dy, o.dx * o.dx + o.dy * o.dy);  // the loop's test, on lanes 0 / 1
                fa = px - i;
                fb = py - j;
            } else
            for (;;) {
                EIK_P2PROBE(0);
                i = (uint32_t)__builtin_trunc(px);
                j = (uint32_t)__builtin_trunc(py);
                in = !__builtin_isnan(px + py) && (int)i >= lo_x && (int)i <= hi_x && (int)j >= lo_y && (int)j <= hi_y;
                unsigned off = (unsigned)(((int)j - cy0i) * kPW + ((int)i - cx0i)) * (unsigned)sizeof(double2);
                off = off <= kWinBytes - (kPW + 2) * sizeof(double2) ? off : 0u;  // unsigned: negatives too
                const double2* g = reinterpret_cast<const double2*>(reinterpret_cast<const char*>(s.g[cur]) + off);
                EIK_P2PROBE(1);
                fa = px - i;
                fb = py - j;
                if constexpr (LOOP == 3)
                    o = step_math_rs(g[0], g[1], g[kPW], g[kPW + 1], fa, fb, odd);
                else if constexpr (LOOP == 2)
                    o = step_math_core(g[0], g[1], g[kPW], g[kPW + 1], fa, fb, odd);
                else
                    o = step_math(g[0], g[1], g[kPW], g[kPW + 1], fa, fb);
                EIK_P2PROBE(2);
                const double ex = o.sx - a.ex, ey = o.sy - a.ey;
                const bool stop = ex * ex + ey * ey < 2.25;  // :231-232, as in the loop below
                EIK_P2PROBE(3);
                // one branch: the conditions combined bitwise (a || chain becomes one branch each)
                const bool leave = (int)!in | (int)odd | (int)__builtin_isnan(o.dx + o.dy) | (int)stop |
                                   (int)(k + 1 >= kmax);
                if (leave) break;
                *reinterpret_cast<double2*>(out + 2 * n) = make_double2(o.sx, o.sy);
                ++n;
                px = o.sx;
                py = o.sy;
                ++k;
            }
            if (!in || odd) {  // window bookkeeping (or an error), then this step again -- exactly
                if (!in && !slow_step(i, j)) break;
                const int li = (int)i - cx0i, lj = (int)j - cy0i;
                o = step_math(s.g[cur][lj][li], s.g[cur][lj][li + 1], s.g[cur][lj + 1][li], s.g[cur][lj + 1][li + 1],
                              fa, fb);
            }
            // the reference-structured loop's end of step
            const double ex = o.sx - a.ex, ey = o.sy - a.ey;
            const bool stop = ex * ex + ey * ey < 2.25;
            if (__builtin_isnan(o.dx) || __builtin_isnan(o.dy)) {
                nan_fallback();
                break;
            }
            *reinterpret_cast<double2*>(out + 2 * n) = make_double2(o.sx, o.sy);
            ++n;
            px = o.sx;
            py = o.sy;
            if (stop) break;  // k counts completed non-final steps, as the for loop's ++k
            if (++k >= kmax) break;
        }
    } else {
        for (; k < kmax; ++k) {
            EIK_P2PROBE(0);
            const uint32_t i = (uint32_t)__builtin_trunc(px), j = (uint32_t)__builtin_trunc(py);
            // one test on the chain: NaN point, out of range, or window bookkeeping due
            if (__builtin_isnan(px + py) || (int)i < lo_x || (int)i > hi_x || (int)j < lo_y || (int)j > hi_y) {
                if (!slow_step(i, j)) break;
            }
            EIK_P2PROBE(1);
            const int li = (int)i - cx0i, lj = (int)j - cy0i;
            const double fa = px - i, fb = py - j;
            const StepOut o = step_math(s.g[cur][lj][li], s.g[cur][lj][li + 1], s.g[cur][lj + 1][li],
                                        s.g[cur][lj + 1][li + 1], fa, fb);
            EIK_P2PROBE(2);
            // :231-232  sqrt(e) < 1.5  <=>  e < 2.25 for a correctly rounded sqrt (2.25 = 1.5^2 exactly)
            const double ex = o.sx - a.ex, ey = o.sy - a.ey;
            const bool stop = ex * ex + ey * ey < 2.25;
            EIK_P2PROBE(3);
            // one test after the step: a NaN gradient (the fallback: nothing of this step is kept)
            // or the stop radius; NaN in dx + dy also catches inf - inf, re-tested precisely
            if (__builtin_isnan(o.dx + o.dy) || stop) {
                if (__builtin_isnan(o.dx) || __builtin_isnan(o.dy)) {
                    nan_fallback();
                    break;
                }
            }
            *reinterpret_cast<double2*>(out + 2 * n) = make_double2(o.sx, o.sy);  // every lane: same address and value
            ++n;
            px = o.sx;
            py = o.sy;
            if (stop) break;
        }
    }
    if (k == kmax && kmax < a.steps && status == kGdmDone) status = kGdmError;  // out of point budget
    __hip_atomic_store(&s.req_seq, -1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);  // builders exit
    EIK_P2FLUSH;
    if (lead) {
        if (status == kGdmDone && n < a.cap) {  // :234
            out[2 * n] = a.ex;
            out[2 * n + 1] = a.ey;
            ++n;
        }
        *a.n_out = n;
        *a.status = status;
    }
}

// Self-test of the 2D walker's fast-path arithmetic against the exact forms it stands in for,
// on n pseudo-random inputs per function drawn from the walker's fast-path domain (walk_odd
// false): sqrt_core(x) vs sqrt(x) for x in [2^-767, 2^1000]; div_core(n, d) vs n / d for d in
// [2^-900, 2^100], |n| <= d, n = 0 or |n| >= 2^-900 (a zero quotient may differ in sign only);
// interp2_general vs interp2_sel for corners in [-1, 1] and fractions in [0, 1) that are exactly
// 0 a quarter of the time; div_rs(n, sqrt_core_h(x, h), h) vs n / sqrt(x) for x in [2^-767, 2^200],
// |n| <= sqrt(x), n = 0 or |n| >= 2^-900.  counts[0..2]: mismatches of the first three;
// counts[3]: samples evaluated; counts[4]: mismatches of div_rs; counts[5]: sqrt_c1_h(x) vs sqrt(x)
// on the same x.
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {  // splitmix64
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ double dbl_exp(unsigned long long r, int e_lo, int e_hi) {  // 2^e * (1 + m)
    const int e = e_lo + (int)((r >> 52) % (unsigned long long)(e_hi - e_lo + 1));
    return __longlong_as_double((long long)(((unsigned long long)(e + 1023) << 52) | (r & 0xfffffffffffffull)));
}
__device__ __forceinline__ double unit_f(unsigned long long r) { return (double)(r >> 11) * 0x1p-53; }  // [0, 1)
__global__ void walker_math_selftest_kernel(long long n, unsigned long long seed, unsigned long long* counts) {
    unsigned long long bad[5] = {0, 0, 0, 0, 0}, done = 0;
    for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (long long)gridDim.x * blockDim.x) {
        ++done;
        const unsigned long long r0 = mix64(seed ^ (4 * t)), r1 = mix64(seed ^ (4 * t + 1)), r2 = mix64(seed ^ (4 * t + 2)),
                                 r3 = mix64(seed ^ (4 * t + 3));
        const double x = t == 0 ? 0x1p-767 : dbl_exp(r0, -767, 999);
        if (__double_as_longlong(sqrt_core(x)) != __double_as_longlong(__builtin_sqrt(x))) ++bad[0];
        const double d = dbl_exp(r1, -900, 99);
        double q = d * (2.0 * unit_f(r2) - 1.0);
        if (__builtin_fabs(q) < 0x1p-900 || (r2 & 15) == 0) q = (r2 & 16) ? -0.0 : 0.0;
        const double e1 = div_core(q, d), e0 = q / d;
        if (e0 == 0.0 ? e1 != 0.0 : __double_as_longlong(e1) != __double_as_longlong(e0)) ++bad[1];
        const double fa = (r3 & 3) == 0 ? 0.0 : unit_f(mix64(r3)), fb = (r3 & 12) == 0 ? 0.0 : unit_f(mix64(r3 + 1));
        double g[4];
        for (int c = 0; c < 4; ++c) g[c] = 2.0 * unit_f(mix64(r3 + 2 + c)) - 1.0;
        const double i1 = interp2_general(fa, fb, g[0], g[1], g[2], g[3]), i0 = interp2_sel(fa, fb, g[0], g[1], g[2], g[3]);
        if (i0 == 0.0 ? i1 != 0.0 : __double_as_longlong(i1) != __double_as_longlong(i0)) ++bad[2];
        const unsigned long long r4 = mix64(seed ^ ~(4 * t)), r5 = mix64(r4);
        const double xs = dbl_exp(r4, -767, 199);
        double hs;
        const double ds = sqrt_core_h(xs, hs);
        double ns = ds * (2.0 * unit_f(r5) - 1.0);
        if (__builtin_fabs(ns) < 0x1p-900 || (r5 & 15) == 0) ns = (r5 & 16) ? -0.0 : 0.0;
        if ((r5 & 0x300) == 0) ns = (r5 & 32) ? -ds : ds;  // |n| = d exactly (a unit component)
        const double f1 = div_rs(ns, ds, hs), f0 = ns / __builtin_sqrt(xs);
        if (f0 == 0.0 ? f1 != 0.0 : __double_as_longlong(f1) != __double_as_longlong(f0)) ++bad[3];
        double hc;
        if (__double_as_longlong(sqrt_c1_h(xs, hc)) != __double_as_longlong(__builtin_sqrt(xs))) ++bad[4];
    }
    for (int k = 0; k < 3; ++k)
        if (bad[k]) atomicAdd(&counts[k], bad[k]);
    if (bad[3]) atomicAdd(&counts[4], bad[3]);
    if (bad[4]) atomicAdd(&counts[5], bad[4]);
    if (done) atomicAdd(&counts[3], done);
}
hipError_t walker_math_selftest(long long n, unsigned long long seed, unsigned long long* d_counts, hipStream_t st) {
    hipLaunchKernelGGL(walker_math_selftest_kernel, dim3(1024), dim3(256), 0, st, n, seed, d_counts);
    return hipGetLastError();
}

hipError_t gdm2d(const Gdm2dArgs& a, bool f64, hipStream_t st) {
    const dim3 g(1), b(kPathThreads);
    if (f64) {
        if (a.fused == 4)      hipLaunchKernelGGL((gdm2d_kernel<double, 4>), g, b, 0, st, a);
        else if (a.fused == 3) hipLaunchKernelGGL((gdm2d_kernel<double, 3>), g, b, 0, st, a);
        else if (a.fused == 2) hipLaunchKernelGGL((gdm2d_kernel<double, 2>), g, b, 0, st, a);
        else if (a.fused == 1) hipLaunchKernelGGL((gdm2d_kernel<double, 1>), g, b, 0, st, a);
        else                   hipLaunchKernelGGL((gdm2d_kernel<double, 0>), g, b, 0, st, a);
    } else {
        if (a.fused == 4)      hipLaunchKernelGGL((gdm2d_kernel<float, 4>), g, b, 0, st, a);
        else if (a.fused == 3) hipLaunchKernelGGL((gdm2d_kernel<float, 3>), g, b, 0, st, a);
        else if (a.fused == 2) hipLaunchKernelGGL((gdm2d_kernel<float, 2>), g, b, 0, st, a);
        else if (a.fused == 1) hipLaunchKernelGGL((gdm2d_kernel<float, 1>), g, b, 0, st, a);
        else                   hipLaunchKernelGGL((gdm2d_kernel<float, 0>), g, b, 0, st, a);
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------- 3D path (FM3D)
// np.gradient(T) along `axis` (0 y, 1 x, 2 z) at (j, i, k): central differences / 2 inside,
// one-sided at the ends (numpy's edge_order=1), no inf awareness (FastMarching3D.py:200).
// The 3D walk is one wave (wave 0) with every lane running the same scalar step (LDS reads are
// broadcasts, so no lane divergence).  T is read from an LDS window [WY][WX][WZ] (z fastest, the
// volume's own order), double-buffered: waves 1..7 build windows, as the 2D kernel's builders do.
// When the step's 4x4x4 cube (trilinear corners +-1 for np.gradient) comes within kPre3 cells of
// an inner window edge, the walker requests the window centred on itself into the idle buffer and
// keeps walking; it waits only if the cube leaves the current window before that build is done
// (or the prefetched window does not hold it).  The integer-descent fallback reads outside the
// window from global memory.  The last kRing path points are mirrored in LDS, so the
// back-tracking of :231-249 does not wait on its own global stores.  The arithmetic, its order
// and every branch are FastMarching3D.py's (bit-identical to the oracle's restatement).
constexpr int kWin3Bytes = 48 * 1024;  // per buffer
constexpr int kRing = 256;
constexpr int kP3Threads = 512;        // walker + 7 builder waves
constexpr int kB3 = kP3Threads / 64 - 1;
constexpr int kPre3 = 14;              // cells from an inner window edge that trigger a prefetch

struct Path3Lds {
    __attribute__((aligned(16))) char wbuf[2][kWin3Bytes];
    double ring[kRing][3];
    double gsh[3][8], nsh[7];  // per-step lane exchange of the walker
    int nbad[7];
    long long req_y0, req_x0, req_z0;
    int req_seq;  // walker -> builders: request number (-1: quit)
    int req_b;    // target buffer
    int done;     // builders -> walker: finished builds x kB3
};

// window dimensions (walker and builders compute the same)
template <typename R>
__device__ __forceinline__ void win3_dims(int64_t H, int64_t W, int64_t L, int& WY, int& WX, int& WZ) {
    constexpr int cells = kWin3Bytes / (int)sizeof(R);
    WZ = (int)(L < 16 ? L : 16);
    int s = 1;
    while ((s + 1) * (s + 1) * WZ <= cells && s < 128) ++s;
    WY = (int)(H < s ? H : s);
    WX = (int)(W < s ? W : s);
}

// Builder wave w (0..kB3-1): cells w * 64 + lane + k * 64 kB3 of the window at (y0, x0, z0) into
// buffer b -- (yy, xx, zz) advanced by carries, 32 loads in flight per lane before their stores.
template <typename R>
__device__ void build3(Path3Lds& s, const R* __restrict__ T, int64_t H, int64_t W, int64_t L, int b, int64_t y0,
                       int64_t x0, int64_t z0, int w) {
    int WY, WX, WZ;
    win3_dims<R>(H, W, L, WY, WX, WZ);
    R* const wl = reinterpret_cast<R*>(s.wbuf[b]);
    const int lane = threadIdx.x & 63;
    const int nc = WY * WX * WZ;
    constexpr int S = 64 * kB3;
    const int sz = S % WZ, sx = (S / WZ) % WX, sy = (S / WZ) / WX;
    const int c00 = w * 64 + lane;
    int zz = c00 % WZ, xx = (c00 / WZ) % WX, yy = (c00 / WZ) / WX;
    constexpr int kB = 32;
    for (int c0 = c00; c0 < nc; c0 += S * kB) {
        R val[kB];
#pragma unroll
        for (int u = 0; u < kB; ++u) {
            if (c0 + S * u < nc) val[u] = T[((y0 + yy) * W + x0 + xx) * L + z0 + zz];
            zz += sz;
            if (zz >= WZ) { zz -= WZ; ++xx; }
            xx += sx;
            if (xx >= WX) { xx -= WX; ++yy; }
            yy += sy;
        }
#pragma unroll
        for (int u = 0; u < kB; ++u)
            if (c0 + S * u < nc) wl[c0 + S * u] = val[u];
    }
}

template <typename R>
__device__ void path3_builder(Path3Lds& s, const R* __restrict__ T, int64_t H, int64_t W, int64_t L) {
    const int w = (int)(threadIdx.x >> 6) - 1;
    int seen = 0;
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        const int q = __hip_atomic_load(&s.req_seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (q < 0) return;
        if (q == seen) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > kPathSpin) return;  // walker gone: give up
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        seen = q;
        build3<R>(s, T, H, W, L, s.req_b, s.req_y0, s.req_x0, s.req_z0, w);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(&s.done, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        t0 = __builtin_amdgcn_s_memrealtime();
    }
}

template <typename R>
struct Win3 {
    const R* __restrict__ T;
    int64_t H, W, L;
    const R* w;           // LDS window
    int64_t y0, x0, z0;   // window origin
    int WY, WX, WZ;
    __device__ __forceinline__ bool inside(int64_t y, int64_t x, int64_t z) const {
        return (uint64_t)(y - y0) < (uint64_t)WY && (uint64_t)(x - x0) < (uint64_t)WX && (uint64_t)(z - z0) < (uint64_t)WZ;
    }
    // T[y, x, z] (in range), from the window when it holds the cell
    __device__ __forceinline__ double at(int64_t y, int64_t x, int64_t z) const {
        if (inside(y, x, z)) return (double)w[((y - y0) * WX + (x - x0)) * WZ + (z - z0)];
        return (double)T[(y * W + x) * L + z];
    }
    // window-only read (the step's cube is always inside the window)
    __device__ __forceinline__ double atw(int64_t y, int64_t x, int64_t z) const {
        return (double)w[((int)(y - y0) * WX + (int)(x - x0)) * WZ + (int)(z - z0)];
    }
};

// FastMarching3D.interpolatePoint :275-314, interior branch (a7 coefficient as written, :290), on
// the eight corner values m[4 dj + 2 di + dk] = m{dj}{di}{dk}
__device__ __forceinline__ double tri3(const double* m, double a, double b, double c) {
    const double m000 = m[0], m001 = m[1], m010 = m[2], m011 = m[3];
    const double m100 = m[4], m101 = m[5], m110 = m[6], m111 = m[7];
    const double a0 = m000;
    const double a1 = m010 - m000;
    const double a2 = m100 - m000;
    const double a3 = m001 - m000;
    const double a4 = m110 + m000 - m010 - m100;
    const double a5 = m011 + m000 - m010 - m001;
    const double a6 = m101 + m000 - m100 - m001;
    const double a7 = m111 + m000 - m100 - m001 - m010;
    return a0 + a1 * a + a2 * b + a3 * c + a4 * a * b + a5 * a * c + a6 * b * c + a7 * a * b * c;
}

// sqrt(a*a + b*b + c*c) < t  <=>  a*a + b*b + c*c < t*t for t = 1 and 1.5 (t*t exact, sqrt correctly
// rounded and monotone; the largest double below t*t has a root that rounds below t): the
// distance tests of :238-240 and :266-267 without the square root on the walker's chain
__device__ __forceinline__ double sq3(double a, double b, double c) { return a * a + b * b + c * c; }

// The walk is ONE wave: its LDS accesses complete in issue order, so lanes exchange values through
// LDS with only a compiler fence (and an LDS-count wait) -- a workgroup barrier would also wait
// for the path's global stores.
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// (uint32_t)trunc(x) and rint(x) as int: one conversion each (the hardware truncates and clamps
// to the type's range, NaN -> 0).  The walker's coordinates are finite (a NaN point ends the walk)
// and below 2^31: out-of-range values clamp to 0 / INT_MIN / INT_MAX, which fail the same range
// tests as the 64-bit conversions did.
__device__ __forceinline__ uint32_t cvt_u32(double x) {
    uint32_t r;
    asm("v_cvt_u32_f64 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ int rint_i32(double x) {
    int r;
    asm("v_cvt_i32_f64 %0, %1" : "=v"(r) : "v"(__builtin_rint(x)));
    return r;
}

// v from lane - SH of the same 16-lane row (DPP row_shr); lanes with no source keep their own
template <int SH>
__device__ __forceinline__ double row_shr_f64(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp((int)(unsigned)b, (int)(unsigned)b, 0x110 + SH, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(unsigned)(b >> 32), (int)(unsigned)(b >> 32), 0x110 + SH, 0xf, 0xf, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// window origin along one axis: the needed span [lo, hi] (clipped to the volume) centred in a
// window of n cells that stays inside [0, len)
__device__ __forceinline__ int64_t win_origin(int64_t lo, int64_t hi, int n, int64_t len) {
    int64_t o = (lo + hi + 1) / 2 - n / 2;
    if (o + n > len) o = len - n;
    return o < 0 ? 0 : o;
}

template <typename R>
__global__ __launch_bounds__(kP3Threads) void gdm3d_kernel(Gdm3dArgs a) {
    __shared__ Path3Lds sl;
    if (threadIdx.x == 0) {
        sl.req_seq = 0;
        sl.done = 0;
    }
    __syncthreads();
    if (threadIdx.x >= 64) {
        path3_builder<R>(sl, static_cast<const R*>(a.T), a.H, a.W, a.L);
        return;
    }
    auto& ring = sl.ring;
    auto& gsh = sl.gsh;
    auto& nsh = sl.nsh;
    auto& nbad = sl.nbad;
    const int lane = threadIdx.x;
    const bool lead = lane == 0;
    Win3<R> v;
    v.T = static_cast<const R*>(a.T);
    v.H = a.H; v.W = a.W; v.L = a.L;
    const int64_t H = a.H, W = a.W, L = a.L;
    win3_dims<R>(a.H, a.W, a.L, v.WY, v.WX, v.WZ);
    // lane constants of the interior gather (see the step): lanes 0..23 sample np.gradient along
    // axis g_ax at corner (cj, ci, ck) of the cube -- window offset g_off from the cube's origin,
    // g_str the axis stride, g_c the corner's coordinate along its axis; lanes 24..30 read the
    // rint node (-1) and its six neighbours (0..5: y-1, y+1, x-1, x+1, z-1, z+1) at g_off from it
    const int sy = v.WX * v.WZ, sx = v.WZ;
    int g_ax = 0, g_c = 0, g_off = 0, g_str = 0;
    if (lane < 24) {
        g_ax = lane >> 3;
        const int cj = (lane >> 2) & 1, ci = (lane >> 1) & 1, ck = lane & 1;
        g_c = g_ax == 0 ? cj : g_ax == 1 ? ci : ck;
        g_off = cj * sy + ci * sx + ck;
        g_str = g_ax == 0 ? sy : g_ax == 1 ? sx : 1;
    } else if (lane < 31) {
        const int q = lane - 25;
        const int st = q < 0 ? 0 : (q >> 1) == 0 ? sy : (q >> 1) == 1 ? sx : 1;
        g_off = q < 0 ? 0 : (q & 1) ? st : -st;
    }
    v.w = reinterpret_cast<const R*>(sl.wbuf[0]);
    v.y0 = v.x0 = v.z0 = -((int64_t)1 << 40);  // empty: the first step requests a window
    // the two buffers' origins (scalars: no private array), the current one mirrored in v
    int64_t oy[2] = {v.y0, v.y0}, ox[2] = {v.x0, v.x0}, oz[2] = {v.z0, v.z0};
    int cur = 0, seq = 0;
    bool pending = false;
    auto issue = [&](int b, int64_t y0, int64_t x0, int64_t z0) {
        oy[b] = y0; ox[b] = x0; oz[b] = z0;
        sl.req_y0 = y0;
        sl.req_x0 = x0;
        sl.req_z0 = z0;
        sl.req_b = b;
        __hip_atomic_store(&sl.req_seq, ++seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    auto wait_built = [&]() -> bool {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(&sl.done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < seq * kB3) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > kPathSpin) return false;
            __builtin_amdgcn_s_sleep(1);
        }
        return true;
    };
    int bj_lo = 1, bj_hi = 0, bi_lo = 1, bi_hi = 0, bk_lo = 1, bk_hi = 0;  // empty: the first step decides
    // step bounds of the fast path (sufficient conditions for "holds and no prefetch trigger")
    auto set_bounds = [&]() {
        const int m = pending ? 0 : kPre3;
        auto lo = [&](int64_t o) { return o == 0 ? 0 : (int)(o + 1 + m); };
        auto hi = [&](int64_t o, int n, int64_t len) { return o + n >= len ? (int)(len - 1) : (int)(o + n - 3 - m); };
        bj_lo = lo(v.y0); bj_hi = hi(v.y0, v.WY, H);
        bi_lo = lo(v.x0); bi_hi = hi(v.x0, v.WX, W);
        bk_lo = lo(v.z0); bk_hi = hi(v.z0, v.WZ, L);
    };
    auto holds = [&](int b, int64_t ylo, int64_t xlo, int64_t zlo, int64_t yhi, int64_t xhi, int64_t zhi) {
        return ylo >= oy[b] && xlo >= ox[b] && zlo >= oz[b] && yhi < oy[b] + v.WY && xhi < ox[b] + v.WX &&
               zhi < oz[b] + v.WZ;
    };
    double* out = a.out;
    // path point q: the LDS ring while it holds it (the last kRing points), else global memory
    auto pt = [&](int64_t q, int c) -> double { return ring[(int)q & (kRing - 1)][c]; };  // q >= 0
    auto put = [&](int64_t q, double x, double y, double z) {
        out[3 * q] = x;  // every lane: same address and value (each lane reads back its own
        out[3 * q + 1] = y;  // stores when back-tracking below the ring)
        out[3 * q + 2] = z;
        ring[(int)q & (kRing - 1)][0] = x;
        ring[(int)q & (kRing - 1)][1] = y;
        ring[(int)q & (kRing - 1)][2] = z;
    };
    int64_t n = 0, lo = 0;  // ring holds points [lo, n); below lo: global
    auto point = [&](int64_t q, int c) -> double { return q >= lo ? pt(q, c) : out[3 * q + c]; };
    put(0, a.init[0], a.init[1], a.init[2]);
    n = 1;
    int status = kGdmDone;
    const double tau = a.tau;
    const int off[6][3] = {{0, -1, 0}, {0, 1, 0}, {-1, 0, 0}, {1, 0, 0}, {0, 0, -1}, {0, 0, 1}};
    double gx = a.init[0], gy = a.init[1], gz = a.init[2];  // the last point, out[n - 1]
    double ustep[6][3];  // (-off) / tau of the integer-descent moves (:244-252), divided once
#pragma unroll
    for (int q = 0; q < 6; ++q)
        for (int c = 0; c < 3; ++c) ustep[q][c] = (double)(-off[q][c]) / tau;
    // what the step's tail (:255-264) subtracts from the node after the descent move q: its
    // |(dx, dy, dz)| is the one nonzero |ustep| (sqrt(u*u) == |u| for a correctly rounded root), so
    // the branch and the products are known per move
    double mstep[6][3];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
        const double u = ustep[q][q >> 1 == 0 ? 1 : q >> 1 == 1 ? 0 : 2];
        const double nrm = __builtin_fabs(u);
        for (int c = 0; c < 3; ++c) mstep[q][c] = nrm < 0.01 ? tau * (ustep[q][c] / nrm) : tau * ustep[q][c];
    }
    double p2x = 0.0, p2y = 0.0, p2z = 0.0;  // path point n - 2 (point n - 1 is (gx, gy, gz))
    // the descent's moves are exact unit steps (tau * (-off / tau) == -off, e.g. tau = 0.5): after
    // an integer-node step the walk stays on nodes, and the run loop below takes the next ones
    bool int_moves = EIK_P3RUN != 0;
#pragma unroll
    for (int q = 0; q < 6; ++q)
        for (int c = 0; c < 3; ++c) int_moves &= mstep[q][c] == (double)(-off[q][c]);
    bool run = false;  // the previous step was an integer-node step and int_moves holds
    EIK_P3DECL;
    for (long k = 0; k < a.steps; ++k) {
        // Integer-descent run (the C5 regime).  After an integer-node step from node M to its
        // neighbour N the step at N, as the general body below takes it, is: the point test of
        // :238-240 pops N itself (distance 0) but not M (distance exactly 1), puts N back where
        // it was (the same value in the same slot), and -- when the fallback is taken (a T sample
        // of the gradient not finite, T[N] finite, every neighbour in range: an interior node) and
        // some neighbour is lower -- appends N + off[best] (the tail's N - mstep[best], exact).
        // The run loop does exactly that on scalar node coordinates; any other case (window
        // bookkeeping due, a face node, no lower neighbour, the point budget) leaves it for the
        // general body of the same step.
        if (run) {
            // every value the loop branches on is wave-uniform and held in scalar registers (the
            // window bounds come from the general body's VALU conversions: read them once)
            auto rfl = [](int q) { return __builtin_amdgcn_readfirstlane(q); };
            auto rfl64 = [](int64_t q) {
                return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)((uint64_t)q >> 32)) << 32) |
                                 (uint32_t)__builtin_amdgcn_readfirstlane((int)q));
            };
            int x = rfl((int)gx), y = rfl((int)gy), z = rfl((int)gz);
            const int wy0 = rfl((int)v.y0), wx0 = rfl((int)v.x0), wz0 = rfl((int)v.z0);
            // the fast window bounds and the interior test in one range per axis
            const int ylo = rfl(bj_lo > 1 ? bj_lo : 1), yhi = rfl(bj_hi < (int)H - 2 ? bj_hi : (int)H - 2);
            const int xlo = rfl(bi_lo > 1 ? bi_lo : 1), xhi = rfl(bi_hi < (int)W - 2 ? bi_hi : (int)W - 2);
            const int zlo = rfl(bk_lo > 1 ? bk_lo : 1), zhi = rfl(bk_hi < (int)L - 2 ? bk_hi : (int)L - 2);
            const int len = g_ax == 0 ? (int)H : g_ax == 1 ? (int)W : (int)L;  // lanes 0..23: the sample axis
            const int lane_xyz = g_ax;  // which coordinate a gradient lane's corner runs along
            const bool node_lane = lane >= 24 && lane < 31;
            const R* w = v.w;
            int64_t nn = rfl64(n), ll = rfl64(lo), kq = rfl64((int64_t)k);
            const int64_t cap = a.cap, steps = a.steps;
            bool fin = false, moved = false;
            int xp = 0, yp = 0, zp = 0;
            for (;;) {
                if (y < ylo || y > yhi || x < xlo || x > xhi || z < zlo || z > zhi) break;
                const int base = ((y - wy0) * v.WX + (x - wx0)) * v.WZ + (z - wz0);
                const int pc = (lane_xyz == 0 ? y : lane_xyz == 1 ? x : z) + g_c;  // >= 1: never the first
                const int idx = base + g_off;
                const R r_hi = w[idx + (pc == len - 1 ? 0 : g_str)];
                const R r_lo = w[idx - g_str];
                const double t_hi = (double)r_hi;
                const unsigned long long nonfin =
                    __ballot(lane < 24 && !(__builtin_isfinite(r_hi) && __builtin_isfinite(r_lo)));
                const double tnode = readlane_f64(t_hi, 24);
                // T[N] +inf (the general body's fallback test) or NaN (its ordered scan below never
                // moves; the minimum below would skip the NaN): the general body
                if (nonfin == 0ull || !(tnode < __builtin_inf())) break;
                // The reference's ordered scan (curT = T[N]; `if T[nb] < curT` over the six
                // neighbours) picks the FIRST neighbour attaining the minimum, if that minimum is
                // below T[N].  As a lane minimum over lanes 24..30 (the node first: a tie with it
                // keeps the node) and the lowest lane holding it; NaN neighbours are never taken by
                // either (v_min_f64 returns the other operand, NaN == m is false).
                double mv = node_lane ? t_hi : __builtin_inf();
                mv = __builtin_fmin(mv, row_shr_f64<1>(mv));
                mv = __builtin_fmin(mv, row_shr_f64<2>(mv));
                mv = __builtin_fmin(mv, row_shr_f64<4>(mv));
                const double m = readlane_f64(mv, 30);  // row_shr 1, 2, 4: lanes 23..30, lane 23 +inf
                const unsigned long long eq = __ballot(node_lane && t_hi == m);
                const int best = rfl(__builtin_ctzll(eq) - 25);  // -1: the node itself
                if (best < 0 || nn >= cap) break;
                const int nx = x + (best == 2 ? -1 : best == 3 ? 1 : 0);
                const int ny = y + (best == 0 ? -1 : best == 1 ? 1 : 0);
                const int nz = z + (best == 4 ? -1 : best == 5 ? 1 : 0);
                put(nn, (double)nx, (double)ny, (double)nz);
                ++nn;
                if (nn - ll > kRing) ll = nn - kRing;
                moved = true;
                xp = x;
                yp = y;
                zp = z;
                x = nx;
                y = ny;
                z = nz;
                if (sq3((double)nx - a.end[0], (double)ny - a.end[1], (double)nz - a.end[2]) < 2.25) {
                    fin = true;  // :266-267
                    break;
                }
                if (++kq >= steps) {
                    fin = true;
                    break;
                }
            }
            n = nn;
            lo = ll;
            k = (long)kq;
            if (moved) {  // the last two points: the current node and the node before it
                p2x = (double)xp;
                p2y = (double)yp;
                p2z = (double)zp;
                gx = (double)x;
                gy = (double)y;
                gz = (double)z;
            }
            if (fin) break;
        }
        EIK_P3PROBE(3);
        const uint32_t i = cvt_u32(gx), j = cvt_u32(gy), kk = cvt_u32(gz);
        if (i + 1 >= (uint64_t)W || j + 1 >= (uint64_t)H || kk + 1 >= (uint64_t)L) { status = kGdmError; break; }
        // fast path: while bj_lo <= j <= bj_hi (and for i, kk) the cube is in the current window and
        // not within kPre3 of an inner edge (or a build is pending): nothing to do this step
        if ((int)j < bj_lo || (int)j > bj_hi || (int)i < bi_lo || (int)i > bi_hi || (int)kk < bk_lo || (int)kk > bk_hi) {
            const int64_t ylo = j > 0 ? j - 1 : 0, yhi = j + 2 < H ? j + 2 : H - 1;
            const int64_t xlo = i > 0 ? i - 1 : 0, xhi = i + 2 < W ? i + 2 : W - 1;
            const int64_t zlo = kk > 0 ? kk - 1 : 0, zhi = kk + 2 < L ? kk + 2 : L - 1;
            const int64_t cy0 = win_origin(ylo, yhi, v.WY, H), cx0 = win_origin(xlo, xhi, v.WX, W),
                          cz0 = win_origin(zlo, zhi, v.WZ, L);
            if (!holds(cur, ylo, xlo, zlo, yhi, xhi, zhi)) {
                const int nb = seq == 0 ? 0 : 1 - cur;
                bool have = false;
                if (pending) {
                    pending = false;
                    if (!wait_built()) { status = kGdmError; break; }
                    have = holds(nb, ylo, xlo, zlo, yhi, xhi, zhi);
                }
                if (!have) {
                    issue(nb, cy0, cx0, cz0);
                    if (!wait_built()) { status = kGdmError; break; }
                }
                cur = nb;
                v.w = reinterpret_cast<const R*>(sl.wbuf[cur]);
                v.y0 = oy[cur];
                v.x0 = ox[cur];
                v.z0 = oz[cur];
            }
            // near an inner edge of the current window: build the window centred here, meanwhile
            if (!pending && ((ylo - v.y0 < kPre3 && v.y0 > 0) || (v.y0 + v.WY - 1 - yhi < kPre3 && v.y0 + v.WY < H) ||
                             (xlo - v.x0 < kPre3 && v.x0 > 0) || (v.x0 + v.WX - 1 - xhi < kPre3 && v.x0 + v.WX < W) ||
                             (zlo - v.z0 < kPre3 && v.z0 > 0) || (v.z0 + v.WZ - 1 - zhi < kPre3 && v.z0 + v.WZ < L)) &&
                (cy0 != v.y0 || cx0 != v.x0 || cz0 != v.z0)) {
                issue(1 - cur, cy0, cx0, cz0);
                pending = true;
            }
            set_bounds();
        }
        EIK_P3PROBE(0);
        const int64_t rx = rint_i32(gx), ry = rint_i32(gy), rz = rint_i32(gz);
        const bool rin = rx >= 0 && ry >= 0 && rz >= 0 && rx < W && ry < H && rz < L;
        // per-lane gather, kept in registers: lanes 0..23 the two T samples of one np.gradient value
        // (axis, corner), lanes 24..30 the node and its six neighbours (:244-252).  (The last two
        // path points, which the pops of :238-240 test, are (gx, gy, gz) and (p2x, p2y, p2z).)
        double t_hi = 0.0, t_lo = 0.0, gscale = 0.5, nv = 0.0;
        bool bad = false;
        if (ry >= 1 && ry + 1 < H && rx >= 1 && rx + 1 < W && rz >= 1 && rz + 1 < L) {
            // interior rint node: its six neighbours are in range (no wrap, none bad) and, like the
            // cube, inside the window -- every lane reads window cells at a lane-constant offset,
            // the same code on every lane (lanes 24..30 with stride 0 read their cell twice)
            const bool grad = lane < 24;
            const int base = grad ? (((int)(j - v.y0) * v.WX + (int)(i - v.x0)) * v.WZ + (int)(kk - v.z0))
                                  : (((int)(ry - v.y0) * v.WX + (int)(rx - v.x0)) * v.WZ + (int)(rz - v.z0));
            const int64_t pc = (g_ax == 0 ? (int64_t)j : g_ax == 1 ? (int64_t)i : (int64_t)kk) + g_c;
            const int64_t len = g_ax == 0 ? H : g_ax == 1 ? W : L;
            const bool first = pc == 0, last = !first && pc == len - 1;
            const int idx = lane < 31 ? base + g_off : base;
            const R* w = v.w;
            t_hi = (double)w[idx + (last ? 0 : g_str)];
            t_lo = (double)w[idx - (first ? 0 : g_str)];
            gscale = first || last ? 1.0 : 0.5;  // (/ 1.0 at the ends, / 2.0 inside: both exact)
            nv = t_hi;
        } else {
        if (lane >= 24 && lane < 31) {
            if (rin) {
                const int q = lane - 25;  // -1: the node; 0..5: y-1, y+1, x-1, x+1, z-1, z+1 (:244-252)
                int64_t cx = rx, cy = ry, cz = rz;
                if (q >= 0) {
                    const int64_t sg = (q & 1) ? 1 : -1;
                    cy += (q >> 1) == 0 ? sg : 0;
                    cx += (q >> 1) == 1 ? sg : 0;
                    cz += (q >> 1) == 2 ? sg : 0;
                }
                if (cx < 0) cx += W;  // python negative indices wrap
                if (cy < 0) cy += H;
                if (cz < 0) cz += L;
                bad = cx >= W || cy >= H || cz >= L;
                nv = bad ? __builtin_nan("") : v.at(cy, cx, cz);
            }
        }
        if (lane < 24) {
            const int axis = lane >> 3, cj = (lane >> 2) & 1, ci = (lane >> 1) & 1, ck = lane & 1;
            const int64_t y = j + cj, x = i + ci, z = kk + ck;
            const int64_t len = axis == 0 ? H : axis == 1 ? W : L;
            const int64_t p = axis == 0 ? y : axis == 1 ? x : z;
            const bool first = p == 0, last = !first && p == len - 1;
            const int64_t dlo = first ? 0 : 1, dhi = last ? 0 : 1;
            t_hi = v.atw(y + (axis == 0) * dhi, x + (axis == 1) * dhi, z + (axis == 2) * dhi);
            t_lo = v.atw(y - (axis == 0) * dlo, x - (axis == 1) * dlo, z - (axis == 2) * dlo);
            gscale = first || last ? 1.0 : 0.5;  // (/ 1.0 at the ends, / 2.0 inside: both exact)
        }
        }
        // Integer-node step (the C5 regime: on a z-padded few-layer volume every step is the
        // integer descent).  At a point whose three coordinates are integers every fraction of
        // the trilinear interpolation is 0, so each of dx, dy, dz is a0 + a1*0 + ... + a7*0*0*0:
        // NaN exactly when one of its coefficients is not finite (a*0 = NaN), i.e. when one of
        // its eight np.gradient samples is (every corner enters some a1..a7), i.e. when one of
        // their T samples is; otherwise a0.  So the fallback is taken iff a lane's T sample is not
        // finite -- a ballot, no interpolation and no lane exchange through LDS.  When it is
        // taken with the node reached and in range, no neighbour out of range and some
        // neighbour lower, the step is the descent below, in the reference's order with the
        // same operations as the general path (which handles every other case).
        double dx = 0.0, dy = 0.0, dz = 0.0;
        bool intstep = false;
        int best = -1;
        double tnode = 0.0;
        if (gx == (double)i && gy == (double)j && gz == (double)kk && rin) {
            const unsigned long long nonfin =
                __ballot(lane < 24 && !(__builtin_isfinite(t_hi) && __builtin_isfinite(t_lo)));
            const unsigned long long badm = __ballot(lane >= 24 && lane < 31 && bad);
            tnode = readlane_f64(nv, 24);
            if (nonfin != 0ull && badm == 0ull && !__builtin_isinf(tnode)) {
                double curT = tnode;
#pragma unroll
                for (int q = 0; q < 6; ++q) {  // the reference's ordered scan
                    const double tc = readlane_f64(nv, 25 + q);
                    if (tc < curT) {
                        curT = tc;
                        best = q;
                    }
                }
                intstep = best >= 0;
            }
        }
        if (intstep) {
            const int64_t nx = rx, ny = ry, nz = rz;
            bool deep = false;  // as the NaN branch below with fast = true
            if (n > 0 && sq3(gx - nx, gy - ny, gz - nz) < 1.0) {
                --n;
                if (n > 0 && sq3(p2x - nx, p2y - ny, p2z - nz) < 1.0) {
                    --n;
                    deep = true;
                }
            }
            if (deep)
                while (n > 0 && sq3(point(n - 1, 0) - nx, point(n - 1, 1) - ny, point(n - 1, 2) - nz) < 1.0) --n;
            if (n >= a.cap) { status = kGdmError; break; }
            if (n < lo) lo = n;
            put(n, (double)nx, (double)ny, (double)nz);
            ++n;
            gx = (double)nx;
            gy = (double)ny;
            gz = (double)nz;
        } else {
        if (lane < 24) gsh[lane >> 3][lane & 7] = (t_hi - t_lo) * gscale;
        if (lane >= 24 && lane < 31 && rin) {
            nsh[lane - 24] = nv;
            nbad[lane - 24] = bad;
        }
        wave_lds_sync();
        dx = tri3(gsh[1], gx - i, gy - j, gz - kk);
        dy = tri3(gsh[0], gx - i, gy - j, gz - kk);
        dz = tri3(gsh[2], gx - i, gy - j, gz - kk);
        EIK_P3PROBE(1);
        if (__builtin_isnan(dx) || __builtin_isnan(dy) || __builtin_isnan(dz)) {  // :212-253
            int64_t nx = rx, ny = ry, nz = rz;
            bool err = false;
            // fast: the node is in range and reached -- no back-tracking, the gathered values apply
            const bool fast = rin && !__builtin_isinf(nsh[0]);
            if (!fast) {
                for (;;) {
                    if (nx < 0 || ny < 0 || nz < 0 || nx >= W || ny >= H || nz >= L) { err = true; break; }
                    if (!__builtin_isinf(v.at(ny, nx, nz))) break;
                    --n;
                    if (n == 0) { err = true; break; }
                    nx = (int64_t)__builtin_rint(point(n - 1, 0));
                    ny = (int64_t)__builtin_rint(point(n - 1, 1));
                    nz = (int64_t)__builtin_rint(point(n - 1, 2));
                }
                if (err) { status = kGdmError; break; }
            }
            bool deep = !fast;  // pops beyond the two gathered points read the ring
            if (fast && n > 0 && sq3(gx - nx, gy - ny, gz - nz) < 1.0) {
                --n;
                if (n > 0 && sq3(p2x - nx, p2y - ny, p2z - nz) < 1.0) {
                    --n;
                    deep = true;
                }
            }
            if (deep)
                while (n > 0 && sq3(point(n - 1, 0) - nx, point(n - 1, 1) - ny, point(n - 1, 2) - nz) < 1.0) --n;
            if (n >= a.cap) { status = kGdmError; break; }
            if (n < lo) lo = n;
            put(n, (double)nx, (double)ny, (double)nz);
            ++n;
            if (!fast) {  // the six neighbours of a back-tracked node, in parallel (lanes 0..5)
                if (lane < 6) {
                    int64_t cx = nx + off[lane][0], cy = ny + off[lane][1], cz = nz + off[lane][2];
                    if (cx < 0) cx += W;  // python negative indices wrap
                    if (cy < 0) cy += H;
                    if (cz < 0) cz += L;
                    const bool bad = cx >= W || cy >= H || cz >= L;
                    nsh[lane + 1] = bad ? __builtin_nan("") : v.at(cy, cx, cz);
                    nbad[lane + 1] = bad;
                }
                wave_lds_sync();
            }
            double curT = fast ? nsh[0] : v.at(ny, nx, nz);
            for (int q = 0; q < 6; ++q) {  // the reference's ordered scan
                if (nbad[q + 1]) { err = true; break; }
                const double tc = nsh[q + 1];
                if (tc < curT) {
                    curT = tc;
                    dx = ustep[q][0];
                    dy = ustep[q][1];
                    dz = ustep[q][2];
                }
            }
            wave_lds_sync();  // nsh / nbad are rewritten by the next step
            if (err) { status = kGdmError; break; }
            gx = (double)nx;
            gy = (double)ny;
            gz = (double)nz;
        }
        }
        EIK_P3PROBE(2);
        double ax, ay, az;
        if (intstep) {  // the tail below for the move `best`, from the table
            double m0 = 0.0, m1 = 0.0, m2 = 0.0;
#pragma unroll
            for (int q = 0; q < 6; ++q)
                if (q == best) {
                    m0 = mstep[q][0];
                    m1 = mstep[q][1];
                    m2 = mstep[q][2];
                }
            ax = gx - m0;
            ay = gy - m1;
            az = gz - m2;
        } else {
            const double nrm = __builtin_sqrt(dx * dx + dy * dy + dz * dz);  // :255
            if (nrm < 0.01) {
                ax = gx - tau * (dx / nrm);
                ay = gy - tau * (dy / nrm);
                az = gz - tau * (dz / nrm);
            } else {  // unnormalised step (:262-264)
                ax = gx - tau * dx;
                ay = gy - tau * dy;
                az = gz - tau * dz;
            }
        }
        if (n >= a.cap) { status = kGdmError; break; }
        put(n, ax, ay, az);
        ++n;
        if (n - lo > kRing) lo = n - kRing;
        p2x = gx;  // (gx, gy, gz) is point n - 2 now
        p2y = gy;
        p2z = gz;
        gx = ax;
        gy = ay;
        gz = az;
        if (__builtin_isnan(ax) || __builtin_isnan(ay) || __builtin_isnan(az)) { status = kGdmError; break; }
        if (sq3(ax - a.end[0], ay - a.end[1], az - a.end[2]) < 2.25) break;  // :266-267
        run = int_moves && intstep;
    }
    if (pending) wait_built();  // no build may still be writing when the builders are told to quit
    __hip_atomic_store(&sl.req_seq, -1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (lead) {
        if (status == kGdmDone && n < a.cap) {  // :269
            out[3 * n] = a.end[0];
            out[3 * n + 1] = a.end[1];
            out[3 * n + 2] = a.end[2];
            ++n;
        }
        *a.n_out = n;
        *a.status = status;
    }
    EIK_P3FLUSH;
}

hipError_t gdm3d(const Gdm3dArgs& a, bool f64, hipStream_t st) {
    if (f64)
        hipLaunchKernelGGL(gdm3d_kernel<double>, dim3(1), dim3(kP3Threads), 0, st, a);
    else
        hipLaunchKernelGGL(gdm3d_kernel<float>, dim3(1), dim3(kP3Threads), 0, st, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------- full-field gradient
__global__ void gradient2d_kernel(const double* __restrict__ T, int64_t H, int64_t W, double* __restrict__ gnx,
                                  double* __restrict__ gny) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= H * W) return;
    const int64_t j = idx / W, i = idx - (idx / W) * W;
    double a, b;
    grad_at<double>(T, H, W, j, i, a, b);
    gnx[idx] = a;
    gny[idx] = b;
}

hipError_t gradient2d(const double* T, int64_t H, int64_t W, double* gnx, double* gny, hipStream_t st) {
    const int64_t n = H * W;
    hipLaunchKernelGGL(gradient2d_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, T, H, W, gnx, gny);
    return hipGetLastError();
}

}  // namespace eik
