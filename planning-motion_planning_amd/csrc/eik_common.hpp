// eik_common.hpp -- shared device helpers for the MI355X Eikonal kernels (gfx950 / CDNA4).
//
// Grid convention follows the reference (FastMarching.py): rasters are row-major [y][x], nodes
// are (x, y); +inf cost = impassable (closed, FastMarching.py:93-94); T = +inf = unreached.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace eik {

constexpr int kTile = 64;          // tile side (cells); one wave64 lane per tile column
constexpr int kThreads = 256;      // 4 waves per tile: one per quadrant sweep direction
constexpr int kLds = kTile + 2;    // LDS row stride: tile + 1-cell halo on each side

template <typename R> struct Real;
template <> struct Real<float> {
    using U = unsigned int;
    static __host__ __device__ constexpr float inf() { return __builtin_inff(); }
};
template <> struct Real<double> {
    using U = unsigned long long;
    static __host__ __device__ constexpr double inf() { return __builtin_inf(); }
};

// 2D Godunov upwind update -- the three branches of getEikonal (FastMarching.py:17-29):
//   both neighbours inf -> inf;  one inf -> other + c;  c < |a-b| -> min + c;
//   else 0.5 * (a + b + sqrt(2c^2 - (a-b)^2)).
// Branch-free: hi == inf covers the first two branches (lo + c, inf + c = inf).
// getEikonal FastMarching.py:17-29 in its own operation order, IEEE fp64 without contraction,
// correctly rounded sqrt (np.power(x, 2) of a numpy scalar is the exact product; the oracle's
// orc_eikonal): the exact band replay (bidir_exact.hip) and its fronts' solve (fim2d.hip REF)
__device__ __forceinline__ double eik_ref(double thor, double tver, double c) {
#pragma clang fp contract(off)
    const double inf = Real<double>::inf();
    if (thor == inf) return tver == inf ? inf : tver + c;
    if (tver == inf) return thor + c;
    const double d = thor - tver;
    if (c < __builtin_fabs(d)) return __builtin_fmin(thor, tver) + c;
    return 0.5 * (thor + tver + __builtin_sqrt(2.0 * (c * c) - d * d));
}

// FastMarching3D.py:59-75 in the reference's own arithmetic, for the fp64 solver: Tarray =
// [Tx, Ty, Tz]; Tmax = the FIRST largest entry (Python max); sumT = left fold of (Tmax - Ta)^2 from
// 0; accept when C^2 > sumT with Tr = (S + sqrt(n C^2 + S^2 - n Q)) / n, S and Q right-associated
// sums (sumlist, :103-107) in list order; else remove that Tmax (list.remove: first occurrence)
// and retry.  No contraction, correctly rounded sqrt and division: the same bits as the reference
// on the same neighbours, so exact ties stay exact ties (FastMarching3D.computeTmap's early exit
// compares against T[start], fim3d_early_kernel).  All +inf -> +inf (the reference never solves
// a cell without a popped neighbour).
__device__ __forceinline__ double solve3_ref(double v0, double v1, double v2, double C) {
#pragma clang fp contract(off)
    // select form of the reference's loop (no divergence): the three acceptance tests first, then
    // ONE square root and ONE division on the accepted list
    const double C2 = C * C;
    // n = 3: Tmax = first largest (Python max: replaced only by a strictly larger item)
    const bool m1 = v1 > v0;
    const double t01 = m1 ? v1 : v0;
    const bool m2 = v2 > t01;
    const double tmax = m2 ? v2 : t01;
    const int im = m2 ? 2 : (m1 ? 1 : 0);
    const double d0 = tmax - v0, d1 = tmax - v1, d2 = tmax - v2;
    const bool ok3 = C2 > (d0 * d0 + d1 * d1) + d2 * d2;  // ((0 + d0^2) + d1^2) + d2^2; NaN -> false
    // n = 2: the list without its first largest entry, in list order
    const double u0 = im == 0 ? v1 : v0, u1 = im == 2 ? v1 : v2;
    const bool n1 = u1 > u0;
    const double t2 = n1 ? u1 : u0;
    const double e0 = t2 - u0, e1 = t2 - u1;
    const bool ok2 = C2 > e0 * e0 + e1 * e1;
    // n = 1: the remaining entry (sumT = (w - w)^2: 0, or NaN for +inf)
    const double w = n1 ? u0 : u1;
    const double dw = w - w;
    const bool ok1 = C2 > dw * dw;
    double S, Q, nn;
    if (ok3) {
        S = v0 + (v1 + v2);  // sumlist: right-associated
        Q = v0 * v0 + (v1 * v1 + v2 * v2);
        nn = 3.0;
    } else if (ok2) {
        S = u0 + u1;
        Q = u0 * u0 + u1 * u1;
        nn = 2.0;
    } else {
        S = w;
        Q = w * w;
        nn = 1.0;
    }
    const double tr = (S + __builtin_sqrt((nn * C2 + S * S) - nn * Q)) / nn;
    return (ok3 || ok2 || ok1) ? tr : Real<double>::inf();
}

template <typename R>
__device__ __forceinline__ R godunov2(R a, R b, R c) {
    const R lo = a < b ? a : b;
    const R hi = a < b ? b : a;
    const R d = hi - lo;                     // NaN when both inf (never selected)
    const R t1 = lo + c;
    const R t2 = R(0.5) * (lo + hi + __builtin_sqrt(R(2) * (c * c) - d * d));
    return (hi == Real<R>::inf() || c < d) ? t1 : t2;
}
template <>
__device__ __forceinline__ float godunov2<float>(float a, float b, float c) {
    const float lo = fminf(a, b), hi = fmaxf(a, b);
    const float d = hi - lo;
    const float t1 = lo + c;
    const float t2 = 0.5f * (lo + hi + __builtin_amdgcn_sqrtf(2.f * (c * c) - d * d));  // v_sqrt_f32, <= 1 ulp
    return (hi == Real<float>::inf() || c < d) ? t1 : t2;
}

// min / max of non-negative floats (and +inf, and NaN, which sorts above +inf) on the bit
// patterns: v_min_u32 / v_max_u32, no NaN canonicalisation as fminf/fmaxf need.
__device__ __forceinline__ float umin(float a, float b) {
    return __uint_as_float(min(__float_as_uint(a), __float_as_uint(b)));
}
__device__ __forceinline__ float umax(float a, float b) {
    return __uint_as_float(max(__float_as_uint(a), __float_as_uint(b)));
}
__device__ __forceinline__ double umin(double a, double b) {
    const unsigned long long x = __double_as_longlong(a), y = __double_as_longlong(b);
    return __longlong_as_double(x < y ? x : y);
}
__device__ __forceinline__ double umax(double a, double b) {
    const unsigned long long x = __double_as_longlong(a), y = __double_as_longlong(b);
    return __longlong_as_double(x < y ? y : x);
}

// Sweep-step form: the one-inf case is folded into c < d (d = inf), and the both-inf case
// yields NaN, which the caller's unsigned min / ds_min / `<` tests all treat as "no update"
// -- shorter than godunov2.  Inputs are non-negative, +inf, never NaN.
__device__ __forceinline__ float godunov2_step(float a, float b, float c) {
    const float lo = umin(a, b), hi = umax(a, b);
    const float d = hi - lo;
    // 0.5 (a + b + sqrt(2c^2 - d^2)) written as lo + 0.5 (d + sqrt(.)): ONE rounding at the
    // magnitude of T instead of three -- the fp32 error then stays within 2e-5 on 4096^2 fields
    // with costs up to 300 (T ~ 1e5), where the direct form drifts past it.
    const float t2 = lo + 0.5f * (d + __builtin_amdgcn_sqrtf(2.f * (c * c) - d * d));
    return c < d ? lo + c : t2;
}
__device__ __forceinline__ double godunov2_step(double a, double b, double c) {
    const double lo = umin(a, b), hi = umax(a, b);
    const double d = hi - lo;
    const double t2 = lo + 0.5 * (d + __builtin_sqrt(2.0 * (c * c) - d * d));
    return c < d ? lo + c : t2;
}

// Sweep-step form without the 1D branch: with d clamped to c, lo + (d + sqrt(2c^2 - d^2)) / 2
// equals lo + c exactly when d >= c, i.e. the 1D update falls out of the 2D form.  The clamp is
// an unsigned min (no canonicalisation; a NaN d -- both neighbours +inf -- becomes c and the
// result stays +inf).  Inputs are non-negative, +inf, never NaN.
__device__ __forceinline__ float godunov2_fast(float a, float b, float c) {
    const float lo = umin(a, b), hi = umax(a, b);
    const float d = umin(hi - lo, c);
    const float c2 = c * c;
    const float q = __builtin_fmaf(-d, d, c2) + c2;  // 2c^2 - d^2 >= c^2 >= 0
    return __builtin_fmaf(0.5f, d + __builtin_amdgcn_sqrtf(q), lo);
}
__device__ __forceinline__ double godunov2_fast(double a, double b, double c) {
    const double lo = umin(a, b), hi = umax(a, b);
    const double d = umin(hi - lo, c);
    const double c2 = c * c;
    const double q = __builtin_fma(-d, d, c2) + c2;
    return __builtin_fma(0.5, d + __builtin_sqrt(q), lo);
}

// Sweep step with the shortest dependency chain from the upstream values (a, b) to the result:
//   d = min(|a - b|, c)      one v_sub + one v_min with the |.| source modifier (the legacy form
//                            needs min + max + sub + unsigned min);
//   q = 2c^2 - d^2           one fma against c2x2 = 2c^2, computed off the chain from the
//                            prefetched cost (one rounding instead of two);
//   w = lo + (d + sqrt(q))/2
// Special values as godunov2_fast: a = b = +inf gives |a - b| = NaN, which v_min turns into c,
// and w = +inf; c = +inf with one finite side gives NaN (no update).  v_min_f32 is written in
// asm so that no NaN canonicalisation is inserted (IEEE minNum: a NaN operand yields the other).
// EIK_CHAIN (fp64, default on): w = (lo + d/2) + sqrt(q)/2 with lo + d/2 formed beside the square
// root, one dependent operation fewer on the step's chain than lo + (d + sqrt(q))/2, at the price of
// one more rounding at T's magnitude (fp32 cannot afford it: the 4096^2 field then drifts past 2e-5
// relative; fp64 stays within the 1e-9 tolerance, tests/test_gpu_fullsize.py).  EIK_CHAIN 2 and 3 are
// the two fp64 forms below (one dependent operation fewer / one instruction fewer); all three ran
// within noise on C2 (profiles/r03n_chain_variants_ab.log) -- the fp64 solve is bound by its tile
// hops, not by the step -- and 3, the fewest instructions, is the default.
#ifndef EIK_CHAIN
#define EIK_CHAIN 3
#endif
__device__ __forceinline__ float godunov2_chain(float a, float b, float c, float c2x2) {
    const float lo = umin(a, b);
    const float diff = a - b;
    float d;
    asm("v_min_f32 %0, |%1|, %2" : "=v"(d) : "v"(diff), "v"(c));
    const float q = __builtin_fmaf(-d, d, c2x2);
    return __builtin_fmaf(0.5f, d + __builtin_amdgcn_sqrtf(q), lo);  // one rounding at T's magnitude
}
// fp64 sweep step (the headline arithmetic: the reference computes in float64).  Two savings over
// the generic form, 45 -> 28 instructions per step:
//  * minimum of two values that are >= 0, +inf or a quiet NaN (the only NaNs a sweep makes: inf - inf
//    and the all-ones lane-0 identity) as ONE v_min_f64: in IEEE mode it is minNum -- a quiet-NaN
//    operand yields the other one, exactly as the unsigned umin, which takes v_cmp_lt_u64 + 2
//    v_cndmask for 64-bit values;
//  * the square root of q = 2c^2 - d^2 in [c^2, 2c^2] without the range scaling of the compiler's
//    sequence (sqrt_sweep).
__device__ __forceinline__ double fmin_nn(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// sqrt(q) for q >= 0: v_rsq_f64, one Goldschmidt step and one Newton correction -- the compiler's
// correctly rounded sequence minus its ldexp range scaling (an identity for q in [2^-1000, 2^1000],
// so q is clamped below to 2^-1000: a zero-cost cell, q = 0, gives 2^-500, which vanishes against lo)
// and minus its last correction (result within ~1 ulp; the field tolerance is 1e-9 absolute).
// q = +inf or NaN (a +inf cost) gives NaN: no update, as sqrt's +inf / NaN did.
__device__ __forceinline__ double sqrt_sweep(double q) {
#if EIK_CHAIN
    // the staged costs are >= 2^-500 (fim2d.hip stage_cost), so q = 2c^2 - d^2 >= c^2 >= 2^-1000
    const double qc = q;
#else
    double qc;
    asm("v_max_f64 %0, %1, %2" : "=v"(qc) : "v"(q), "v"(0x1p-1000));
#endif
    const double y = __builtin_amdgcn_rsq(qc);
    double g = qc * y, h = 0.5 * y;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    const double e = __builtin_fma(-g, g, qc);
    return __builtin_fma(e, h, g);
}
__device__ __forceinline__ double godunov2_chain(double a, double b, double c, double c2x2) {
    const double lo = fmin_nn(a, b);
    const double diff = a - b;
    double d;
    asm("v_min_f64 %0, |%1|, %2" : "=v"(d) : "v"(diff), "v"(c));
    const double q = __builtin_fma(-d, d, c2x2);
#if EIK_CHAIN >= 3
    // two Newton steps from v_rsq_f64 (relative error ~2^-23 -> ~2^-47 -> ~2^-70), the second one's
    // correction applied with the unrefined h = y/2 (its error multiplies a residual of ~2^-47):
    // 9 instructions from q to w instead of 10, the same 6 dependent ones after v_rsq as EIK_CHAIN 1
    const double base = __builtin_fma(0.5, d, lo);
    const double y = __builtin_amdgcn_rsq(q);
    const double g = q * y, h = 0.5 * y;
    const double s1 = __builtin_fma(__builtin_fma(-g, g, q), h, g);
    const double e2 = __builtin_fma(-s1, s1, q);
    return __builtin_fma(0.5, __builtin_fma(e2, h, s1), base);
#elif EIK_CHAIN >= 2
    // sqrt_sweep's Newton correction folded into the result: w = (lo + d/2 + g1/2) + e * y/4, with
    // lo + d/2 + g1/2 formed beside e = q - g1^2.  The correction's multiplier is the unrefined
    // y/4 (h/2) instead of the Goldschmidt-refined h'/2: its relative error (v_rsq_f64, ~2^-23)
    // multiplies e, itself ~2^-44 of g1, so the correction is still exact to ~2^-67 of sqrt(q).
    // Chain after v_rsq: mul, fma, fma, fma, fma (one fewer than sqrt_sweep + the final fma), same
    // instruction count; one more rounding at T's magnitude.
    const double base = __builtin_fma(0.5, d, lo);
    const double y = __builtin_amdgcn_rsq(q);
    const double g = q * y, h = 0.5 * y, hq = 0.25 * y;
    const double r = __builtin_fma(-h, g, 0.5);
    const double g1 = __builtin_fma(g, r, g);
    const double e = __builtin_fma(-g1, g1, q);
    return __builtin_fma(e, hq, __builtin_fma(0.5, g1, base));
#elif EIK_CHAIN
    return __builtin_fma(0.5, sqrt_sweep(q), __builtin_fma(0.5, d, lo));
#else
    return __builtin_fma(0.5, d + sqrt_sweep(q), lo);
#endif
}

// Whole-wave shift by one lane (lane i <- lane i-1) on the DPP path: v_mov_b32_dpp wave_shr:1.
// Keeps the Gauss-Seidel dependency of the skewed sweep in registers (no LDS round trip).
__device__ __forceinline__ float wave_shr1(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xF, 0xF, false));
}
// Same, lane 0 receives `lane0` (bound_ctrl off: an out-of-range source keeps the old value).
__device__ __forceinline__ float wave_shr1(float v, float lane0) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(lane0), __float_as_int(v), 0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ double wave_shr1(double v, double lane0) {
    const unsigned long long u = __double_as_longlong(v), o = __double_as_longlong(lane0);
    const int lo = __builtin_amdgcn_update_dpp((int)(o & 0xffffffffu), (int)(u & 0xffffffffu), 0x138, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(u >> 32), 0x138, 0xF, 0xF, false);
    return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_shr1(double v) {
    const unsigned long long u = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(u & 0xffffffffu), 0x138, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(u >> 32), 0x138, 0xF, 0xF, false);
    return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// Whole-wave shift by one lane with the identity of an unsigned min in lane 0 (UINT_MAX, i.e. a
// NaN pattern above every value): umin(wave_shr1_umin_id(x), y) is one v_min_u32_dpp once the
// DPP combiner folds the move into its user, and lane 0 gets y.
__device__ __forceinline__ float wave_shr1_umin_id(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(-1, __float_as_int(v), 0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ double wave_shr1_umin_id(double v) {
    const unsigned long long u = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(-1, (int)(u & 0xffffffffu), 0x138, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(-1, (int)(u >> 32), 0x138, 0xF, 0xF, false);
    return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// LDS atomic min on a non-negative float/double (IEEE order == unsigned-integer order for x >= 0).
__device__ __forceinline__ void lds_min(float* p, float v) {
    atomicMin(reinterpret_cast<unsigned int*>(p), __float_as_uint(v));
}
__device__ __forceinline__ void lds_min(double* p, double v) {
    atomicMin(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v));
}

}  // namespace eik
