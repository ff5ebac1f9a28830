// costmap.hip -- the planner's cost-raster builder on gfx950: the producer of the Eikonal
// solver's input (Coupled_motion_planner.py:37-105 and :1101-1216).
//
//   DEM Z --(min, quadratic-extrapolated central differences, cross product)--> unit normals
//     --(arccos(Nz) > slope_max)--> obstacle mask --(flood fill, disk erode/dilate, ...)-->
//     --(300 * obstacle + 10 * distance ramp, 50 x 50 box blur)--> cost raster
//
// All stages are HBM-bound elementwise / stencil / line passes.  Morphology with the
// reference's disk structuring element (d <= r on integer offsets, structural_disk :96-105)
// is computed EXACTLY from squared Euclidean distances: dilate(A, disk r)(p) =
// [dist^2(p, A) <= r^2], erode(A, disk r)(p) = A(p) and [dist^2(p, not A) > r^2] (pixels outside
// the image take no part, as cv2's default morphology border) -- by a radius-bounded separable
// transform (only distances <= r matter).  The distance ramp needs the full exact EDT (its
// maximum normalises the ramp, :1196): column distances by 64-row segments with a carry scan,
// then per row an outward scan over LDS-staged column distances, in integers -- the squared
// distances scipy.ndimage.distance_transform_edt takes the sqrt of (:1194).  The flood fill of
// image_filling (:82-94, cv2.floodFill 4-connected from (0, 0)) is reachability, i.e. the
// block-FIM solver itself with cost 1 on the seed's value and +inf elsewhere (host side).
//
// Floating point: IEEE f64 without contraction, the reference's operation order where it is
// defined (stencils: two non-zero taps, exact halvings; normals; ramp); the box blur sums in a
// different order than scipy's convolve2d (relative 1e-15).
#include "eik_common.hpp"
#include "eik_kernels.hpp"

#pragma clang fp contract(off)

namespace eik {

constexpr int kCmThreads = 256;

// linspace(0, size, n)[i] as numpy computes it: i * step, the last element exactly `size`
__device__ __forceinline__ double lin(double size, int64_t n, int64_t i) {
    const double step = size / (double)(n - 1);
    return i == n - 1 ? size : (double)i * step;
}

// value of the quadratically extrapolated padding (Coupled_motion_planner.py:51-56) of a 1D grid
__device__ __forceinline__ double lin_pad(double size, int64_t n, int64_t i) {
    if (i < 0) return 3 * lin(size, n, 0) - 3 * lin(size, n, 1) + lin(size, n, 2);
    if (i >= n) return 3 * lin(size, n, n - 1) - 3 * lin(size, n, n - 2) + lin(size, n, n - 3);
    return lin(size, n, i);
}

// Z - zmin with the reference's padding: vertical padding first, then the horizontal padding of
// the vertically padded array (:51-56), so corners extrapolate the padded rows.
struct Zpad {
    const double* Z;
    int64_t H, W;
    double zmin;
    __device__ double at(int64_t y, int64_t x) const { return Z[y * W + x] - zmin; }
    __device__ double vpad(int64_t y, int64_t x) const {  // rows -1..H, x in [0, W)
        if (y < 0) return 3 * at(0, x) - 3 * at(1, x) + at(2, x);
        if (y >= H) return 3 * at(H - 1, x) - 3 * at(H - 2, x) + at(H - 3, x);
        return at(y, x);
    }
    __device__ double operator()(int64_t y, int64_t x) const {  // rows -1..H, cols -1..W
        if (x < 0) return 3 * vpad(y, 0) - 3 * vpad(y, 1) + vpad(y, 2);
        if (x >= W) return 3 * vpad(y, W - 1) - 3 * vpad(y, W - 2) + vpad(y, W - 3);
        return vpad(y, x);
    }
};

// min of Z (bit-pattern atomic on the order-preserving map of doubles)
__device__ __forceinline__ unsigned long long dkey(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    return (b >> 63) ? ~b : (b | (1ull << 63));
}
__device__ __forceinline__ double dval(unsigned long long k) {
    return __longlong_as_double((long long)((k >> 63) ? (k & ~(1ull << 63)) : ~k));
}

__global__ void cm_min_kernel(const double* __restrict__ Z, int64_t n, unsigned long long* out) {
    unsigned long long best = ~0ull;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const unsigned long long k = dkey(Z[i]);
        best = k < best ? k : best;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long v = __shfl_xor(best, o);
        best = v < best ? v : best;
    }
    if ((threadIdx.x & 63) == 0) atomicMin(out, best);
}

// surface_normal (:37-80) per node; obstacle = arccos(Nz) > slope_max (:1145-1154), border 0
// (:1157-1160).  Optional Nx/Ny/Nz outputs (the Python drop-in's surface_normal).
__global__ void cm_normals_kernel(const double* __restrict__ Z, int64_t H, int64_t W, double size,
                                  const unsigned long long* __restrict__ zmin_key, double slope_max,
                                  unsigned char* __restrict__ obst, double* __restrict__ Nx, double* __restrict__ Ny,
                                  double* __restrict__ Nz) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= H * W) return;
    const int64_t y = idx / W, x = idx - (idx / W) * W;
    const Zpad zp{Z, H, W, dval(*zmin_key)};
    // stencil1 (x): conv = 0.5 A[y][x+1] + (-0.5) A[y][x-1], a = -conv (:58-60)
    // stencil2 (y): conv = 0.5 A[y+1][x] + (-0.5) A[y-1][x], b = conv (:62-64)
    const double xp = lin_pad(size, W, x + 1), xm = lin_pad(size, W, x - 1);
    const double yp = lin_pad(size, H, y + 1), ym = lin_pad(size, H, y - 1);
    const double xc = lin_pad(size, W, x), yc = lin_pad(size, H, y);
    const double ax = -(0.5 * xp + -0.5 * xm);
    const double ay = -(0.5 * yc + -0.5 * yc);
    const double az = -(0.5 * zp(y, x + 1) + -0.5 * zp(y, x - 1));
    const double bx = 0.5 * xc + -0.5 * xc;
    const double by = 0.5 * yp + -0.5 * ym;
    const double bz = 0.5 * zp(y + 1, x) + -0.5 * zp(y - 1, x);
    const double nx = -(ay * bz - az * by);  // :70-72
    const double ny = -(az * bx - ax * bz);
    const double nz = -(ax * by - ay * bx);
    double mag = __builtin_sqrt(nx * nx + ny * ny + nz * nz);  // :74-75
    if (mag == 0) mag = 2.220446049250313e-16;
    const double nzn = nz / mag;
    if (Nx) {
        Nx[idx] = nx / mag;
        Ny[idx] = ny / mag;
        Nz[idx] = nzn;
    }
    if (obst) {
        const bool border = y == 0 || x == 0 || y == H - 1 || x == W - 1;
        obst[idx] = (!border && acos(nzn) > slope_max) ? 1 : 0;
    }
}

// ---- exact squared EDT to the pixels where feat(p) is true ------------------------------
// pass 1, one thread per column: g = |y - nearest feature row in the column| (or kFar)
constexpr int kFar = 1 << 29;

template <typename F>
__global__ void cm_edt_cols_kernel(F feat, int64_t H, int64_t W, int* __restrict__ g) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= W) return;
    int d = kFar;
    for (int64_t y = 0; y < H; ++y) {
        d = feat(y * W + x) ? 0 : (d >= kFar ? kFar : d + 1);
        g[y * W + x] = d;
    }
    d = kFar;
    for (int64_t y = H - 1; y >= 0; --y) {
        const int v = g[y * W + x];
        d = v == 0 ? 0 : (d >= kFar ? kFar : d + 1);
        if (d < v) g[y * W + x] = d;
    }
}

// pass 2, one thread per row: D(x) = min_q (x - q)^2 + g(q)^2 by the lower envelope of
// parabolas (Felzenszwalb-Huttenlocher), in exact integer arithmetic; kFar columns have no
// feature.  Scratch per row: v (W ints), z (W + 1 ints as doubles' stand-in: rationals compared
// by cross-multiplication).
__global__ void cm_edt_rows_kernel(const int* __restrict__ g, int64_t H, int64_t W, int* __restrict__ D,
                                   int* __restrict__ vbuf) {
    const int64_t y = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (y >= H) return;
    const int* gr = g + y * W;
    int* v = vbuf + y * W;  // parabola apexes of the envelope
    int* out = D + y * W;
    auto f = [&](int q) -> long long { const long long t = gr[q]; return t * t; };
    // intersection abscissa of parabolas q1 < q2: s = ((f(q2) + q2^2) - (f(q1) + q1^2)) / (2 (q2 - q1))
    int k = -1;
    for (int q = 0; q < (int)W; ++q) {
        if (gr[q] >= kFar) continue;
        while (k >= 0) {
            const int p = v[k];
            if (k == 0) break;
            const int pp = v[k - 1];
            // remove p if the new parabola q overtakes p before p overtakes pp:
            // s(pp, p) >= s(p, q)
            const long long num1 = (f(p) + (long long)p * p) - (f(pp) + (long long)pp * pp), den1 = 2ll * (p - pp);
            const long long num2 = (f(q) + (long long)q * q) - (f(p) + (long long)p * p), den2 = 2ll * (q - p);
            if (num1 * den2 >= num2 * den1) --k;
            else break;
        }
        v[++k] = q;
    }
    if (k < 0) {
        for (int x = 0; x < (int)W; ++x) out[x] = INT32_MAX;
        return;
    }
    int j = 0;
    for (int x = 0; x < (int)W; ++x) {
        // advance while the next parabola is lower at x
        while (j < k) {
            const long long a = (long long)(x - v[j]) * (x - v[j]) + f(v[j]);
            const long long b = (long long)(x - v[j + 1]) * (x - v[j + 1]) + f(v[j + 1]);
            if (b <= a) ++j;
            else break;
        }
        const long long d = (long long)(x - v[j]) * (x - v[j]) + f(v[j]);
        out[x] = d > INT32_MAX ? INT32_MAX : (int)d;
    }
}

// pass 1, segmented (parallel over 64-row segments of every column): per segment the first and
// last feature rows; per column a carry scan over the segments (nearest feature row above and
// below each segment); per segment the two sweeps seeded with the carries.
constexpr int kSeg = 64;

template <typename F>
__global__ void cm_seg_summary_kernel(F feat, int64_t H, int64_t W, int* __restrict__ first, int* __restrict__ last) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t sg = blockIdx.y;
    if (x >= W) return;
    const int64_t y0 = sg * kSeg, y1 = y0 + kSeg < H ? y0 + kSeg : H;
    int f = -1, l = -1;
    for (int64_t y = y0; y < y1; ++y)
        if (feat(y * W + x)) {
            if (f < 0) f = (int)y;
            l = (int)y;
        }
    first[sg * W + x] = f;
    last[sg * W + x] = l;
}

__global__ void cm_seg_carry_kernel(int64_t nseg, int64_t W, int* __restrict__ first, int* __restrict__ last) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= W) return;
    // in place: last[s] <- last feature row before segment s; first[s] <- first feature row after it
    int run = -1;
    for (int64_t sg = 0; sg < nseg; ++sg) {
        const int l = last[sg * W + x];
        last[sg * W + x] = run;
        if (l >= 0) run = l;
    }
    run = -1;
    for (int64_t sg = nseg - 1; sg >= 0; --sg) {
        const int f = first[sg * W + x];
        first[sg * W + x] = run;
        if (f >= 0) run = f;
    }
}

template <typename F>
__global__ void cm_seg_fill_kernel(F feat, int64_t H, int64_t W, const int* __restrict__ below,
                                   const int* __restrict__ above, int* __restrict__ g) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t sg = blockIdx.y;
    if (x >= W) return;
    const int64_t y0 = sg * kSeg, y1 = y0 + kSeg < H ? y0 + kSeg : H;
    int up = above[sg * W + x];
    for (int64_t y = y0; y < y1; ++y) {
        if (feat(y * W + x)) up = (int)y;
        g[y * W + x] = up >= 0 ? (int)y - up : kFar;
    }
    int dn = below[sg * W + x];
    for (int64_t y = y1 - 1; y >= y0; --y) {
        if (feat(y * W + x)) dn = (int)y;
        if (dn >= 0 && dn - (int)y < g[y * W + x]) g[y * W + x] = dn - (int)y;
    }
}

// pass 2, one workgroup per row (rows <= kEdtRowMax wide): the row's column distances staged in
// LDS; each pixel scans outward from its own column while k^2 < best -- the nearest feature's
// column offset k satisfies k^2 <= D(x), so the scan is exact and costs about the distance to
// the nearest feature (terrain rasters: tens of columns).
constexpr int kEdtRowMax = 8192;

__global__ __launch_bounds__(256) void cm_edt_rows_lds_kernel(const int* __restrict__ g, int64_t H, int64_t W,
                                                              int* __restrict__ D) {
    __shared__ int gs[kEdtRowMax];
    const int64_t y = blockIdx.x;
    const int w = (int)W;
    for (int x = threadIdx.x; x < w; x += blockDim.x) gs[x] = g[y * W + x];
    __syncthreads();
    for (int x = threadIdx.x; x < w; x += blockDim.x) {
        long long best = gs[x] >= kFar ? (long long)1 << 62 : (long long)gs[x] * gs[x];
        for (int k = 1; (long long)k * k < best && (x - k >= 0 || x + k < w); ++k) {
            const long long k2 = (long long)k * k;
            if (x - k >= 0 && gs[x - k] < kFar) {
                const long long v = k2 + (long long)gs[x - k] * gs[x - k];
                best = v < best ? v : best;
            }
            if (x + k < w && gs[x + k] < kFar) {
                const long long v = k2 + (long long)gs[x + k] * gs[x + k];
                best = v < best ? v : best;
            }
        }
        D[y * W + x] = best > INT32_MAX ? INT32_MAX : (int)best;
    }
}

// The EDT of :1194 feeds only od = dil * (1 - dist / max(dist)) (:1196): dist matters exactly where
// dil is set -- within r of an obstacle, i.e. D <= r^2 (dil = the disk dilation of the same mask,
// :1192) -- plus its maximum.  Exact scans of every kEdtSample-th pixel in both directions give Ds
// and a lower bound Mlb = max Ds of max D; a pixel lies within 15 rows and columns of the sample
// it is mapped to, so d <= sqrt(Ds) + 15 sqrt(2) (d is 1-Lipschitz).  Where that bound is <= Mlb the pixel cannot exceed the
// maximum: its outward scan stops at k = r (exact if D <= r^2, the dil pixels; else it stores a
// value <= Mlb, outside dil, where od is 0 either way).  Every other pixel is scanned in full.  Every
// D <= r^2 and the maximum stay exact, so dist, its maximum and od are bit-identical to the full
// transform's.
constexpr int kEdtSample = 16;
__global__ void cm_edt_sample_kernel(const int* __restrict__ g, int64_t H, int64_t W, unsigned* __restrict__ mlb,
                                     int* __restrict__ ds) {
    const int64_t ny = (H + kEdtSample - 1) / kEdtSample, nx = (W + kEdtSample - 1) / kEdtSample;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long best = 0;
    if (t < ny * nx) {
        const int64_t y = (t / nx) * kEdtSample, x = (t - (t / nx) * nx) * kEdtSample;
        const int* row = g + y * W;
        long long b = row[x] >= kFar ? (long long)1 << 62 : (long long)row[x] * row[x];
        for (long long k = 1; k * k < b && (x - k >= 0 || x + k < W); ++k) {
            if (x - k >= 0 && row[x - k] < kFar) { const long long v = k * k + (long long)row[x - k] * row[x - k]; b = v < b ? v : b; }
            if (x + k < W && row[x + k] < kFar) { const long long v = k * k + (long long)row[x + k] * row[x + k]; b = v < b ? v : b; }
        }
        best = b > INT32_MAX ? INT32_MAX : (unsigned long long)b;
        ds[t] = (int)best;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long v = __shfl_xor(best, o);
        best = v > best ? v : best;
    }
    if ((threadIdx.x & 63) == 0 && best) atomicMax(mlb, (unsigned)best);
}

__global__ __launch_bounds__(256) void cm_edt_rows_ramp_kernel(const int* __restrict__ g, int64_t H, int64_t W, int r,
                                                               const unsigned* __restrict__ mlb,
                                                               const int* __restrict__ ds, int* __restrict__ D) {
    __shared__ int gs[kEdtRowMax];
    const int64_t y = blockIdx.x;
    const int w = (int)W;
    const long long lb = (long long)*mlb;
    const int64_t ny = (H + kEdtSample - 1) / kEdtSample, nx = (W + kEdtSample - 1) / kEdtSample;
    const int64_t sy = (y + kEdtSample / 2) / kEdtSample < ny ? (y + kEdtSample / 2) / kEdtSample : ny - 1;
    for (int x = threadIdx.x; x < w; x += blockDim.x) gs[x] = g[y * W + x];
    __syncthreads();
    for (int x = threadIdx.x; x < w; x += blockDim.x) {
        const int64_t sx = (x + kEdtSample / 2) / kEdtSample < nx ? (x + kEdtSample / 2) / kEdtSample : nx - 1;
        // >= d(x): the sample is within 15 rows and 15 columns (8 + 8 inside, up to 15 at the clamped
        // last row / column of samples)
        const double ub = __builtin_sqrt((double)ds[sy * nx + sx]) + 21.22;
        const bool full = ub * ub > (double)lb;
        long long best = gs[x] >= kFar ? (long long)1 << 62 : (long long)gs[x] * gs[x];
        for (int k = 1; (long long)k * k < best && (k <= r || full) && (x - k >= 0 || x + k < w); ++k) {
            const long long k2 = (long long)k * k;
            if (x - k >= 0 && gs[x - k] < kFar) {
                const long long v = k2 + (long long)gs[x - k] * gs[x - k];
                best = v < best ? v : best;
            }
            if (x + k < w && gs[x + k] < kFar) {
                const long long v = k2 + (long long)gs[x + k] * gs[x + k];
                best = v < best ? v : best;
            }
        }
        // a capped scan that found nothing within r: outside dil; store a value <= Mlb <= max D
        if (!full && best > (long long)r * r && best > lb) best = lb;
        D[y * W + x] = best > INT32_MAX ? INT32_MAX : (int)best;
    }
}

struct FeatEq {  // feat = (m[i] == val)
    const unsigned char* m;
    unsigned char val;
    __device__ bool operator()(int64_t i) const { return m[i] == val; }
};

static hipError_t cm_edt_cols(const unsigned char* m, unsigned char val, int64_t H, int64_t W, int* g, int* vbuf,
                              hipStream_t st);

// :1194's transform as the ramp uses it (see cm_edt_sample_kernel); r = the dil radius of :1192
hipError_t cm_edt_ramp(const unsigned char* m, int64_t H, int64_t W, int r, int* g, int* D, int* vbuf, hipStream_t st) {
    if (W > kEdtRowMax) return cm_edt(m, 1, H, W, g, D, vbuf, st);
    hipError_t e = cm_edt_cols(m, 1, H, W, g, vbuf, st);
    if (e != hipSuccess) return e;
    unsigned* mlb = reinterpret_cast<unsigned*>(vbuf);  // (the column pass's scratch is free again)
    e = hipMemsetAsync(mlb, 0, sizeof(unsigned), st);
    if (e != hipSuccess) return e;
    const int64_t ns = ((H + kEdtSample - 1) / kEdtSample) * ((W + kEdtSample - 1) / kEdtSample);
    int* ds = vbuf + 1;  // ns <= n - 1 exact sample values (H, W >= 2)
    hipLaunchKernelGGL(cm_edt_sample_kernel, dim3((unsigned)((ns + 255) / 256)), dim3(256), 0, st, g, H, W, mlb, ds);
    hipLaunchKernelGGL(cm_edt_rows_ramp_kernel, dim3((unsigned)H), dim3(256), 0, st, g, H, W, r, mlb, ds, D);
    return hipGetLastError();
}

static hipError_t cm_edt_cols(const unsigned char* m, unsigned char val, int64_t H, int64_t W, int* g, int* vbuf,
                              hipStream_t st) {
    const int64_t nseg = (H + kSeg - 1) / kSeg;
    if (2 * nseg * W <= H * W) {
        int* first = vbuf;
        int* last = vbuf + nseg * W;
        const dim3 grid((unsigned)((W + 255) / 256), (unsigned)nseg);
        hipLaunchKernelGGL(cm_seg_summary_kernel<FeatEq>, grid, dim3(256), 0, st, FeatEq{m, val}, H, W, first, last);
        hipLaunchKernelGGL(cm_seg_carry_kernel, dim3((unsigned)((W + 255) / 256)), dim3(256), 0, st, nseg, W, first, last);
        hipLaunchKernelGGL(cm_seg_fill_kernel<FeatEq>, grid, dim3(256), 0, st, FeatEq{m, val}, H, W, first, last, g);
    } else {
        hipLaunchKernelGGL(cm_edt_cols_kernel<FeatEq>, dim3((unsigned)((W + 63) / 64)), dim3(64), 0, st,
                           FeatEq{m, val}, H, W, g);
    }
    return hipGetLastError();
}

hipError_t cm_edt(const unsigned char* m, unsigned char val, int64_t H, int64_t W, int* g, int* D, int* vbuf,
                  hipStream_t st) {
    const int64_t nseg = (H + kSeg - 1) / kSeg;
    if (2 * nseg * W <= H * W) {  // segment summaries fit in the envelope scratch (vbuf, H * W ints)
        int* first = vbuf;
        int* last = vbuf + nseg * W;
        const dim3 grid((unsigned)((W + 255) / 256), (unsigned)nseg);
        hipLaunchKernelGGL(cm_seg_summary_kernel<FeatEq>, grid, dim3(256), 0, st, FeatEq{m, val}, H, W, first, last);
        hipLaunchKernelGGL(cm_seg_carry_kernel, dim3((unsigned)((W + 255) / 256)), dim3(256), 0, st, nseg, W, first, last);
        hipLaunchKernelGGL(cm_seg_fill_kernel<FeatEq>, grid, dim3(256), 0, st, FeatEq{m, val}, H, W, first, last, g);
    } else {
        hipLaunchKernelGGL(cm_edt_cols_kernel<FeatEq>, dim3((unsigned)((W + 63) / 64)), dim3(64), 0, st,
                           FeatEq{m, val}, H, W, g);
    }
    if (W <= kEdtRowMax)
        hipLaunchKernelGGL(cm_edt_rows_lds_kernel, dim3((unsigned)H), dim3(256), 0, st, g, H, W, D);
    else
        hipLaunchKernelGGL(cm_edt_rows_kernel, dim3((unsigned)((H + 63) / 64)), dim3(64), 0, st, g, H, W, D, vbuf);
    return hipGetLastError();
}

// morphology from the squared EDT: dilate: out = D(to A) <= r^2; erode: out = A && D(to not A) > r^2
__global__ void cm_morph_kernel(const unsigned char* __restrict__ A, const int* __restrict__ D, int64_t n, int r2,
                                int erode, unsigned char* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = erode ? (unsigned char)(A[i] && D[i] > r2) : (unsigned char)(D[i] <= r2);
}

// Disk morphology needs distances only up to r: a radius-bounded separable transform.  Pass V:
// gv(p) = min |dy| <= r with a feature at (y + dy, x), else r + 1.  Pass H: p is within r of a
// feature iff some |dx| <= r has dx^2 + gv(y, x + dx)^2 <= r^2 (the nearest feature q has
// |qy - py| <= r and |qx - px| <= r) -- exact, like the full EDT.
// Round 4: O(1) reads per pixel instead of O(r).  Pass V scans a segment of kSeg rows per thread
// with r rows of context, keeping the nearest feature row above / below (forward, then backward);
// pass H uses the reach of every source s (gv(s) <= r covers |x - s| <= w(s) =
// floor(sqrt(r^2 - gv(s)^2))), rightward and leftward, per row (cm_bnd_rows_kernel).
__global__ void cm_bnd_cols_kernel(const unsigned char* __restrict__ A, int64_t H, int64_t W, int r,
                                   unsigned char want, unsigned char* __restrict__ gv) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= W) return;
    const int64_t y0 = (int64_t)blockIdx.y * kSeg, y1 = y0 + kSeg < H ? y0 + kSeg : H;
    const int64_t far = -(int64_t)r - 2;
    int64_t up = far;  // nearest feature row <= y
    for (int64_t y = y0 - r > 0 ? y0 - r : 0; y < y1; ++y) {
        if (A[y * W + x] == want) up = y;
        if (y >= y0) gv[y * W + x] = (unsigned char)(y - up <= r ? y - up : r + 1);
    }
    int64_t dn = -1;  // nearest feature row >= y (-1: none)
    for (int64_t y = (y1 - 1 + r < H - 1 ? y1 - 1 + r : H - 1); y >= y0; --y) {
        if (A[y * W + x] == want) dn = y;
        if (y < y1 && dn >= 0 && dn - y <= r && dn - y < gv[y * W + x]) gv[y * W + x] = (unsigned char)(dn - y);
    }
}

// w(g) = floor(sqrt(r^2 - g^2)) for g <= r (exact on integers), -1 when g > r
__device__ __forceinline__ int bnd_halfwidth(int g, int r) {
    if (g > r) return -1;
    const int v = r * r - g * g;
    int w = (int)__builtin_sqrtf((float)v);
    while (w * w > v) --w;
    while ((w + 1) * (w + 1) <= v) ++w;
    return w;
}

// Pass H, one workgroup per row (rows <= kBndRowMax wide): a thread scans a chunk of <= 32 pixels;
// the reach of the sources left of x is a prefix maximum of s + w(s), of those right of x a suffix
// minimum of s - w(s): chunk totals by a Hillis-Steele scan over the 256 threads in LDS.
constexpr int kBndRowMax = 8192;
__global__ __launch_bounds__(256) void cm_bnd_rows_kernel(const unsigned char* __restrict__ A,
                                                          const unsigned char* __restrict__ gv, int64_t H, int64_t W,
                                                          int r, int erode, unsigned char* __restrict__ out) {
    __shared__ int wt[256];     // g -> w(g), g <= r <= 250
    __shared__ int pm[2][256];  // chunk reach totals: prefix max (rightward), suffix min (leftward)
    const int y = (int)blockIdx.x, t = threadIdx.x;
    if (t <= r) wt[t] = bnd_halfwidth(t, r);
    const int w = (int)W, C = (w + 255) / 256, xa = t * C, xb = xa + C < w ? xa + C : w;
    const unsigned char* row = gv + (int64_t)y * W;
    __syncthreads();
    int reach = -1, lreach = 1 << 30;
    for (int x = xa; x < xb; ++x) {
        const int g = row[x];
        if (g <= r) {
            const int hw = wt[g];
            reach = x + hw > reach ? x + hw : reach;
            lreach = x - hw < lreach ? x - hw : lreach;
        }
    }
    pm[0][t] = reach;
    pm[1][t] = lreach;
    __syncthreads();
    for (int d = 1; d < 256; d <<= 1) {  // inclusive scans: max over threads <= t, min over threads >= t
        const int a0 = t >= d ? pm[0][t - d] : -1;
        const int b0 = t + d < 256 ? pm[1][t + d] : 1 << 30;
        __syncthreads();
        if (a0 > pm[0][t]) pm[0][t] = a0;
        if (b0 < pm[1][t]) pm[1][t] = b0;
        __syncthreads();
    }
    reach = t > 0 ? pm[0][t - 1] : -1;          // sources left of this chunk
    lreach = t < 255 ? pm[1][t + 1] : 1 << 30;  // sources right of it
    unsigned near = 0;  // bit x - xa (C <= 32)
    for (int x = xa; x < xb; ++x) {
        const int g = row[x];
        if (g <= r && x + wt[g] > reach) reach = x + wt[g];
        if (reach >= x) near |= 1u << (x - xa);
    }
    for (int x = xb - 1; x >= xa; --x) {
        const int g = row[x];
        if (g <= r && x - wt[g] < lreach) lreach = x - wt[g];
        if (lreach <= x) near |= 1u << (x - xa);
    }
    unsigned char* o = out + (int64_t)y * W;
    const unsigned char* a = A + (int64_t)y * W;
    for (int x = xa; x < xb; ++x) {
        const bool nr = (near >> (x - xa)) & 1u;
        o[x] = erode ? (unsigned char)(a[x] && !nr) : (unsigned char)nr;
    }
}

// rows wider than kBndRowMax: one thread per pixel scanning +-r (the round-3 form)
__global__ void cm_bnd_rows_wide_kernel(const unsigned char* __restrict__ A, const unsigned char* __restrict__ gv,
                                        int64_t H, int64_t W, int r, int erode, unsigned char* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= H * W) return;
    const int64_t y = i / W, x = i - (i / W) * W;
    const int r2 = r * r;
    bool near = false;
    for (int k = 0; k <= r && !near; ++k) {
        const int k2 = k * k;
        if (x - k >= 0) { const int g = gv[y * W + x - k]; near |= g <= r && k2 + g * g <= r2; }
        if (x + k < W) { const int g = gv[y * W + x + k]; near |= g <= r && k2 + g * g <= r2; }
    }
    out[i] = erode ? (unsigned char)(A[i] && !near) : (unsigned char)near;
}

hipError_t cm_morph(const unsigned char* A, int64_t H, int64_t W, int r, bool erode, unsigned char* out, int* g, int* D,
                    int* vbuf, hipStream_t st) {
    (void)D;
    (void)vbuf;
    const int64_t n = H * W;
    if (r > 250) {  // beyond the uint8 bounded form: the full EDT
        hipError_t e = cm_edt(A, erode ? 0 : 1, H, W, g, D, vbuf, st);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(cm_morph_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, A, D, n, r * r,
                           erode ? 1 : 0, out);
        return hipGetLastError();
    }
    unsigned char* gv = reinterpret_cast<unsigned char*>(g);
    const dim3 gcols((unsigned)((W + 255) / 256), (unsigned)((H + kSeg - 1) / kSeg));
    hipLaunchKernelGGL(cm_bnd_cols_kernel, gcols, dim3(256), 0, st, A, H, W, r, (unsigned char)(erode ? 0 : 1), gv);
    if (W <= kBndRowMax)
        hipLaunchKernelGGL(cm_bnd_rows_kernel, dim3((unsigned)H), dim3(256), 0, st, A, gv, H, W, r, erode ? 1 : 0, out);
    else
        hipLaunchKernelGGL(cm_bnd_rows_wide_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, A, gv, H, W, r,
                           erode ? 1 : 0, out);
    return hipGetLastError();
}

// ---- image_filling (:82-94) around a reachability solve ---------------------------------
// cost for the flood fill: 1 on pixels equal to the seed value m[0], +inf elsewhere
// Reachability by the block-FIM solver: cost 0 on the seed's value (+inf elsewhere), so a reached
// cell is 0 at once and never revisited for a refinement -- only connectivity is asked.  (The solve
// still takes ~2.3 ms at 4096^2, as with cost 1: a flood from the corner pixel is a chain of ~128
// tile hops across the raster, tools/rover_probe.py under rocprofv3.)
__global__ void cm_fill_cost_kernel(const unsigned char* __restrict__ m, int64_t n, float* __restrict__ c) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    c[i] = m[i] == m[0] ? 0.f : __builtin_inff();
}
// filled = seed pixel's component set to 1; out = m | (~filled - 254) (uint8): seed 0 -> holes
// (zeros not reached) become 1; seed 1 -> every pixel 1 (the reference's arithmetic)
__global__ void cm_fill_apply_kernel(unsigned char* __restrict__ m, const float* __restrict__ T, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned char seed = m[0];  // read before any write: m[0] is never changed by this kernel
    const unsigned char filled = (m[i] == seed && T[i] != __builtin_inff()) ? 1 : m[i];
    const unsigned char inv = (unsigned char)((unsigned char)~filled - 254);
    m[i] = m[i] | inv;
}

hipError_t cm_fill_cost(const unsigned char* m, int64_t n, float* c, hipStream_t st) {
    hipLaunchKernelGGL(cm_fill_cost_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, m, n, c);
    return hipGetLastError();
}
hipError_t cm_fill_apply(unsigned char* m, const float* T, int64_t n, hipStream_t st) {
    hipLaunchKernelGGL(cm_fill_apply_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, m, T, n);
    return hipGetLastError();
}

// ---- image_filling (:82-94) as connected components: the 4-connected component of pixel (0, 0)
// among the pixels equal to m[0], by lock-free union-find (links always from the larger to the
// smaller index, so the component of pixel 0 has root 0).  The block-FIM flood (cm_fill_cost /
// cm_fill_apply above) is a chain of ~128 tile hops from the corner across a 4096^2 raster
// (2.3 ms); here no information travels tile by tile:
//  1. per 32 x 32 tile, union-find in LDS over the tile's pixels, each pixel's local root written
//     as a global index (lroot; -1: not the seed value);
//  2. one thread per pixel pair across a tile border: union of their local roots in `parent`;
//  3. every local root resolved to its final root, then the fill applied from parent[lroot[i]].
constexpr int kCcl = 32;
__device__ __forceinline__ int ccl_ld(const int* p, int x, int scope) {
    return scope == 0 ? __hip_atomic_load(p + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
                      : __hip_atomic_load(p + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ccl_find(const int* p, int x, int scope) {
    for (int y = ccl_ld(p, x, scope); y != x; y = ccl_ld(p, x, scope)) x = y;
    return x;
}
__device__ __forceinline__ void ccl_union(int* p, int a, int b, int scope) {
    for (;;) {
        a = ccl_find(p, a, scope);
        b = ccl_find(p, b, scope);
        if (a == b) return;
        if (a > b) { const int t = a; a = b; b = t; }
        const int old = atomicCAS(p + b, b, a);  // link root b under a, unless b stopped being a root
        if (old == b) return;
        b = old;
    }
}

// Each pixel starts linked to the first pixel of its horizontal run (a wave holds two 32-pixel tile
// rows: run starts from one ballot), so only vertical neighbours are unioned, and of those only the
// first column of each stretch where two runs touch (the pixels to its left already joined them).
__global__ __launch_bounds__(256) void cm_ccl_local_kernel(const unsigned char* __restrict__ m, int64_t H, int64_t W,
                                                           int* __restrict__ lroot, int* __restrict__ parent) {
    static_assert(kCcl == 32, "a wave holds two tile rows");
    __shared__ int lp[kCcl * kCcl];
    const unsigned char v = m[0];
    const int64_t y0 = (int64_t)blockIdx.y * kCcl, x0 = (int64_t)blockIdx.x * kCcl;
    const int lane = threadIdx.x & 63;
    bool s[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int q = threadIdx.x + 256 * k;
        const int64_t gy = y0 + q / kCcl, gx = x0 + q % kCcl;
        s[k] = gy < H && gx < W && m[gy * W + gx] == v;
        const unsigned long long sm = __ballot(s[k]);
        // a run starts where the pixel is set and its left neighbour (same row) is not
        const unsigned long long starts = sm & ~((sm << 1) & ~0x0000000100000001ull);
        const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
        const int rs = 63 - __clzll(starts & upto);  // the run's first lane (same row: col 0 starts a run)
        lp[q] = s[k] ? q - (lane - rs) : -1;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int q = threadIdx.x + 256 * k;
        if (!s[k]) continue;
        const int lx = q % kCcl, ly = q / kCcl;
        if (ly + 1 >= kCcl || ccl_ld(lp, q + kCcl, 0) < 0) continue;
        if (lx > 0 && ccl_ld(lp, q - 1, 0) >= 0 && ccl_ld(lp, q + kCcl - 1, 0) >= 0) continue;  // joined on the left
        ccl_union(lp, q, q + kCcl, 0);  // (-1 entries never change: pixels not set)
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int q = threadIdx.x + 256 * k;
        const int64_t gy = y0 + q / kCcl, gx = x0 + q % kCcl;
        if (gy >= H || gx >= W) continue;
        const int64_t g = gy * W + gx;
        int r = -1;
        if (s[k]) {
            const int lr = ccl_find(lp, q, 0);
            r = (int)((y0 + lr / kCcl) * W + x0 + lr % kCcl);
        }
        lroot[g] = r;
        parent[g] = (int)g;
    }
}

// pairs across tile borders: n_v = H * (ntx - 1) vertical-border pairs, then W * (nty - 1) horizontal
__global__ void cm_ccl_border_kernel(int64_t H, int64_t W, const int* __restrict__ lroot, int* parent, int64_t nv,
                                     int64_t total) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= total) return;
    int64_t a, b;
    if (t < nv) {
        const int64_t y = t % H, k = t / H + 1;  // border between columns k*32 - 1 and k*32
        a = y * W + k * kCcl - 1;
        b = a + 1;
    } else {
        const int64_t u = t - nv, x = u % W, k = u / W + 1;
        a = (k * kCcl - 1) * W + x;
        b = a + W;
    }
    const int ra = lroot[a], rb = lroot[b];
    if (ra < 0 || rb < 0 || ra == rb) return;
    // the previous pair along the same border (y - 1 / x - 1) joins the same two local components in
    // most places: only the first pair of such a run unions (a union is idempotent; the run's first
    // pair always does it).  Most pixels are in one component, whose root every union would contend on.
    const int64_t pa = t < nv ? a - W : a - 1, pb = t < nv ? b - W : b - 1;
    const bool has_prev = t < nv ? (t % H) > 0 : ((t - nv) % W) > 0;
    if (has_prev && lroot[pa] == ra && lroot[pb] == rb) return;
    ccl_union(parent, ra, rb, 1);
}

__global__ void cm_ccl_resolve_kernel(int64_t n, const int* __restrict__ lroot, int* parent) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || lroot[i] != (int)i) return;  // local roots only
    parent[i] = ccl_find(parent, (int)i, 1);
}

// the fill of cm_fill_apply_kernel with "reached" = in pixel 0's component
__global__ void cm_ccl_apply_kernel(unsigned char* __restrict__ m, const int* __restrict__ lroot,
                                    const int* __restrict__ parent, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned char seed = m[0];  // read before any write: m[0] is never changed by this kernel
    const int r = lroot[i];
    const bool reached = r >= 0 && parent[r] == 0;
    const unsigned char filled = (m[i] == seed && reached) ? 1 : m[i];
    const unsigned char inv = (unsigned char)((unsigned char)~filled - 254);
    m[i] = m[i] | inv;
}

hipError_t cm_fill_ccl(unsigned char* m, int64_t H, int64_t W, int* lroot, int* parent, hipStream_t st) {
    const int64_t n = H * W;
    if (n >= (1ll << 31)) return hipErrorInvalidValue;
    const int64_t ntx = (W + kCcl - 1) / kCcl, nty = (H + kCcl - 1) / kCcl;
    hipLaunchKernelGGL(cm_ccl_local_kernel, dim3((unsigned)ntx, (unsigned)nty), dim3(256), 0, st, m, H, W, lroot, parent);
    const int64_t nv = H * (ntx - 1), total = nv + W * (nty - 1);
    if (total > 0)
        hipLaunchKernelGGL(cm_ccl_border_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, H, W, lroot,
                           parent, nv, total);
    const unsigned grid = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(cm_ccl_resolve_kernel, dim3(grid), dim3(256), 0, st, n, lroot, parent);
    hipLaunchKernelGGL(cm_ccl_apply_kernel, dim3(grid), dim3(256), 0, st, m, lroot, parent, n);
    return hipGetLastError();
}

__global__ void cm_border_kernel(unsigned char* __restrict__ m, int64_t H, int64_t W, unsigned char v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < W) {
        m[i] = v;
        m[(H - 1) * W + i] = v;
    }
    if (i < H) {
        m[i * W] = v;
        m[i * W + W - 1] = v;
    }
}

// ---- cost (:1187-1205) ---------------------------------------------------------------------
// dist = res * sqrt(D); atomic max of dist (non-negative doubles: bit order = value order)
__global__ void cm_dist_kernel(const int* __restrict__ D, int64_t n, double res, double* __restrict__ dist,
                               unsigned long long* maxbits) {
    unsigned long long best = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double d = res * __builtin_sqrt((double)D[i]);
        dist[i] = d;
        const unsigned long long b = (unsigned long long)__double_as_longlong(d);
        best = b > best ? b : best;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long v = __shfl_xor(best, o);
        best = v > best ? v : best;
    }
    if ((threadIdx.x & 63) == 0) atomicMax(maxbits, best);
}

// od = dil * (1 - dist / max) (:1196), written into dist; atomic min over od > 0
__global__ void cm_ramp_kernel(const unsigned char* __restrict__ dil, double* __restrict__ dist, int64_t n,
                               const unsigned long long* __restrict__ maxbits, unsigned long long* minbits) {
    const double mx = __longlong_as_double((long long)*maxbits);
    unsigned long long best = ~0ull;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double od = (double)dil[i] * (1 - dist[i] / mx);
        dist[i] = od;
        if (od > 0) {
            const unsigned long long b = (unsigned long long)__double_as_longlong(od);
            best = b < best ? b : best;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long v = __shfl_xor(best, o);
        best = v < best ? v : best;
    }
    if ((threadIdx.x & 63) == 0) atomicMin(minbits, best);
}

// base = 1 + (300 obst + (od - min[od > 0]) * gradient) (:1187, :1197-1205), [y][x]
__global__ void cm_base_kernel(const unsigned char* __restrict__ obst, const double* __restrict__ od, int64_t n,
                               const unsigned long long* __restrict__ minbits, double high, double gradient,
                               double* __restrict__ base) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double v = od[i];
    if (v > 0) v = v - __longlong_as_double((long long)*minbits);
    base[i] = 1 + ((double)obst[i] * high + v * gradient);
}

// 50 x 50 box blur with fill value 300 (:1208-1210): window [-25, +24] on both axes (scipy
// 'same' for an even kernel), separable: rows with fill 300, then columns with fill 50 * 300.
// The reference's cMap is the transpose of `base`; the window treats both axes alike, so the
// blur of base equals the transpose of the reference's blurred cMap.
constexpr int kBox = 50, kBoxLo = 25, kBoxHi = kBox - 1 - kBoxLo;

__global__ void cm_box_rows_kernel(const double* __restrict__ in, int64_t H, int64_t W, double fill,
                                   double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= H * W) return;
    const int64_t y = i / W, x = i - (i / W) * W;
    double s = 0;
    for (int k = -kBoxLo; k <= kBoxHi; ++k) {
        const int64_t xx = x + k;
        s += (xx >= 0 && xx < W) ? in[y * W + xx] : fill;
    }
    out[i] = s;
}

__global__ void cm_box_cols_kernel(const double* __restrict__ in, int64_t H, int64_t W, double fill, double scale,
                                   double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= H * W) return;
    const int64_t y = i / W, x = i - (i / W) * W;
    double s = 0;
    for (int k = -kBoxLo; k <= kBoxHi; ++k) {
        const int64_t yy = y + k;
        s += (yy >= 0 && yy < H) ? in[yy * W + x] : fill;
    }
    const bool border = y == 0 || x == 0 || y == H - 1 || x == W - 1;  // :1213-1216
    out[i] = border ? __builtin_inf() : s * scale;
}

// The same two passes from LDS tiles (round 4): a 64 x 64 block of outputs with its 49 cells of
// filter context staged once by coalesced loads; each output then sums its 50 taps from LDS in the
// same order as the kernels above (bit-identical results).  The global form read every input 50
// times through the caches (~0.38 ms per pass at 4096^2).
constexpr int kBoxT = 64, kBoxSpan = kBoxT + kBox - 1;
template <bool ROWS>
__global__ __launch_bounds__(256) void cm_box_tile_kernel(const double* __restrict__ in, int64_t H, int64_t W,
                                                          double fill, double scale, double* __restrict__ out) {
    // ROWS: a[r][c] = in[y0 + r][x0 - lo + c]; COLS: a[r][c] = in[y0 - lo + r][x0 + c]
    __shared__ double a[ROWS ? kBoxT * kBoxSpan : kBoxSpan * kBoxT];
    const int64_t y0 = (int64_t)blockIdx.y * kBoxT, x0 = (int64_t)blockIdx.x * kBoxT;
    constexpr int nr = ROWS ? kBoxT : kBoxSpan, nc = ROWS ? kBoxSpan : kBoxT;
    for (int q = threadIdx.x; q < nr * nc; q += blockDim.x) {
        const int r = q / nc, c = q - (q / nc) * nc;
        const int64_t y = ROWS ? y0 + r : y0 - kBoxLo + r, x = ROWS ? x0 - kBoxLo + c : x0 + c;
        double v = fill;
        if (ROWS ? (x >= 0 && x < W && y < H) : (y >= 0 && y < H && x < W)) v = in[y * W + x];
        a[q] = v;
    }
    __syncthreads();
    for (int q = threadIdx.x; q < kBoxT * kBoxT; q += blockDim.x) {
        const int r = q / kBoxT, c = q - (q / kBoxT) * kBoxT;
        const int64_t y = y0 + r, x = x0 + c;
        if (y >= H || x >= W) continue;
        double s = 0;
        if (ROWS) {
#pragma unroll 10
            for (int k = 0; k < kBox; ++k) s += a[r * kBoxSpan + c + k];
            out[y * W + x] = s;
        } else {
#pragma unroll 10
            for (int k = 0; k < kBox; ++k) s += a[(r + k) * kBoxT + c];
            const bool border = y == 0 || x == 0 || y == H - 1 || x == W - 1;  // :1213-1216
            out[y * W + x] = border ? __builtin_inf() : s * scale;
        }
    }
}

// ------------------------------------------------------------------------- host launchers
hipError_t cm_normals(const double* Z, int64_t H, int64_t W, double size, unsigned long long* zmin, double slope_max,
                      unsigned char* obst, double* Nx, double* Ny, double* Nz, hipStream_t st) {
    const int64_t n = H * W;
    hipError_t e = hipMemsetAsync(zmin, 0xff, sizeof(unsigned long long), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(cm_min_kernel, dim3((unsigned)std::min<int64_t>(1024, (n + 255) / 256)), dim3(256), 0, st, Z, n,
                       zmin);
    hipLaunchKernelGGL(cm_normals_kernel, dim3((unsigned)((n + kCmThreads - 1) / kCmThreads)), dim3(kCmThreads), 0, st,
                       Z, H, W, size, zmin, slope_max, obst, Nx, Ny, Nz);
    return hipGetLastError();
}

hipError_t cm_border(unsigned char* m, int64_t H, int64_t W, unsigned char v, hipStream_t st) {
    const int64_t n = H > W ? H : W;
    hipLaunchKernelGGL(cm_border_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, m, H, W, v);
    return hipGetLastError();
}

hipError_t cm_cost(const unsigned char* obst, const unsigned char* dil, const int* Dobst, int64_t H, int64_t W,
                   double res, double high, double gradient, double* work, double* tmp, double* cost,
                   unsigned long long* red, hipStream_t st) {
    const int64_t n = H * W;
    const unsigned grid_red = (unsigned)std::min<int64_t>(1024, (n + 255) / 256), grid = (unsigned)((n + 255) / 256);
    hipError_t e = hipMemsetAsync(red, 0, sizeof(unsigned long long), st);  // max
    if (e == hipSuccess) e = hipMemsetAsync(red + 1, 0xff, sizeof(unsigned long long), st);  // min
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(cm_dist_kernel, dim3(grid_red), dim3(256), 0, st, Dobst, n, res, work, red);
    hipLaunchKernelGGL(cm_ramp_kernel, dim3(grid_red), dim3(256), 0, st, dil, work, n, red, red + 1);
    hipLaunchKernelGGL(cm_base_kernel, dim3(grid), dim3(256), 0, st, obst, work, n, red + 1, high, gradient, tmp);
    (void)grid;
    const dim3 tiles((unsigned)((W + kBoxT - 1) / kBoxT), (unsigned)((H + kBoxT - 1) / kBoxT));
    hipLaunchKernelGGL(cm_box_tile_kernel<true>, tiles, dim3(256), 0, st, tmp, H, W, 300.0, 1.0, work);
    hipLaunchKernelGGL(cm_box_tile_kernel<false>, tiles, dim3(256), 0, st, work, H, W, 300.0 * kBox,
                       1.0 / (kBox * kBox), cost);
    return hipGetLastError();
}

// ------------------------------------------------------------------ input validation
// The host entry points' cost check (costs must be >= 0 or +inf; a negative or NaN cost has no
// reference result) on the device copy: the first offending index, by atomicMin, into *first
// (~0: none).  A host scan of a 4096^2 f64 raster runs at memory speed on one core (~19 ms).
template <typename R>
__global__ void cost_check_kernel(const R* __restrict__ c, int64_t n, unsigned long long* __restrict__ first) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    unsigned long long bad = ~0ull;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        if (!(c[i] >= R(0)) && (unsigned long long)i < bad) bad = (unsigned long long)i;
    if (__any(bad != ~0ull) && bad != ~0ull) atomicMin(first, bad);
}

hipError_t cost_check(const void* cost, int64_t n, bool f64, unsigned long long* first, hipStream_t st) {
    hipError_t e = hipMemsetAsync(first, 0xff, sizeof(unsigned long long), st);
    if (e != hipSuccess) return e;
    const int64_t want = (n + 255) / 256;
    const int grid = (int)(want < 4096 ? (want > 0 ? want : 1) : 4096);
    if (f64)
        hipLaunchKernelGGL(cost_check_kernel<double>, dim3(grid), dim3(256), 0, st, (const double*)cost, n, first);
    else
        hipLaunchKernelGGL(cost_check_kernel<float>, dim3(grid), dim3(256), 0, st, (const float*)cost, n, first);
    return hipGetLastError();
}

}  // namespace eik
