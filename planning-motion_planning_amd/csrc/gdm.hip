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

__device__ __forceinline__ double norm2(double a, double b) { return __builtin_sqrt(a * a + b * b); }

enum { kGdmDone = 0, kGdmFallback = 1, kGdmError = 2 };

// LDS window around the walker: the inf-aware normalised gradient (Gnx, Gny) of a 32 x 32 node
// block is computed by all 64 lanes when the walker's 2 x 2 interpolation corners leave the
// block (every ~30 steps at tau = 0.5); each step then reads 8 values from LDS.  The gradient at
// a node depends on T only, so precomputing it is exactly the reference's per-step
// computeGradient evaluated earlier.
constexpr int kG = 32;  // gradient block side (nodes)

struct Win {
    double gx[kG][kG + 1], gy[kG][kG + 1];
    double t[kG + 2][kG + 3];  // T on the block + 1-node margin
    int64_t x0, y0;
};

// computeGradient body at (j, i) reading the T window (FastMarching.py:262-297)
__device__ void grad_win(const Win& w, int64_t m, int64_t n, int64_t j, int64_t i, double& gnx, double& gny) {
#define TW(J, I) w.t[(J) - w.y0 + 1][(I) - w.x0 + 1]
    double gy, gx;
    if (j == 0)
        gy = TW(1, i) - TW(0, i);
    else if (j == m - 1)
        gy = TW(j, i) - TW(j - 1, i);
    else if (__builtin_isinf(TW(j + 1, i)))
        gy = __builtin_isinf(TW(j - 1, i)) ? 0.0 : TW(j, i) - TW(j - 1, i);
    else
        gy = __builtin_isinf(TW(j - 1, i)) ? TW(j + 1, i) - TW(j, i) : (TW(j + 1, i) - TW(j - 1, i)) / 2;
    if (i == 0)
        gx = TW(j, 1) - TW(j, 0);
    else if (i == n - 1)
        gx = TW(j, i) - TW(j, i - 1);
    else if (__builtin_isinf(TW(j, i + 1)))
        gx = __builtin_isinf(TW(j, i - 1)) ? 0.0 : TW(j, i) - TW(j, i - 1);
    else
        gx = __builtin_isinf(TW(j, i - 1)) ? TW(j, i + 1) - TW(j, i) : (TW(j, i + 1) - TW(j, i - 1)) / 2;
#undef TW
    const double den = __builtin_sqrt(gx * gx + gy * gy);
    gnx = gx / den;
    gny = gy / den;
}

template <typename R>
__device__ void win_load(Win& w, const R* __restrict__ T, int64_t H, int64_t W, int64_t i, int64_t j) {
    int64_t x0 = i - kG / 2, y0 = j - kG / 2;
    x0 = x0 + kG > W ? W - kG : x0;
    y0 = y0 + kG > H ? H - kG : y0;
    x0 = x0 < 0 ? 0 : x0;
    y0 = y0 < 0 ? 0 : y0;
    __syncthreads();
    const int lane = threadIdx.x;
    if (lane == 0) {
        w.x0 = x0;
        w.y0 = y0;
    }
    for (int e = lane; e < (kG + 2) * (kG + 2); e += 64) {
        const int r = e / (kG + 2), c = e - r * (kG + 2);
        const int64_t gy = y0 - 1 + r, gx = x0 - 1 + c;
        w.t[r][c] = (gy >= 0 && gy < H && gx >= 0 && gx < W) ? (double)T[gy * W + gx] : 0.0;
    }
    __syncthreads();
    for (int e = lane; e < kG * kG; e += 64) {
        const int r = e / kG, c = e - r * kG;
        const int64_t gy = y0 + r, gx = x0 + c;
        if (gy < H && gx < W) grad_win(w, H, W, gy, gx, w.gx[r][c], w.gy[r][c]);
    }
    __syncthreads();
}

template <typename R>
__global__ __launch_bounds__(64) void gdm2d_kernel(Gdm2dArgs a) {
    __shared__ Win w;
    const R* __restrict__ T = static_cast<const R*>(a.T);
    const int64_t H = a.H, W = a.W;
    const bool lead = threadIdx.x == 0;
    double* out = a.out;
    int status = kGdmDone;
    double px = a.ix, py = a.iy;  // gamma[-1], kept in registers (all lanes)
    if (lead) {
        out[0] = px;
        out[1] = py;
    }
    int64_t n = 1;
    const double tau = a.tau;
    w.x0 = -((int64_t)1 << 40);
    w.y0 = -((int64_t)1 << 40);
    __syncthreads();
    for (long k = 0; k < a.steps; ++k) {
        if (__builtin_isnan(px) || __builtin_isnan(py)) { status = kGdmError; break; }
        const uint32_t i = (uint32_t)__builtin_trunc(px), j = (uint32_t)__builtin_trunc(py);
        if (i + 1 >= (uint64_t)W || j + 1 >= (uint64_t)H) { status = kGdmError; break; }
        // the 2 x 2 interpolation corners must lie in the gradient block
        if ((int64_t)i < w.x0 || (int64_t)j < w.y0 || (int64_t)i + 1 >= w.x0 + kG || (int64_t)j + 1 >= w.y0 + kG)
            win_load<R>(w, T, H, W, i, j);
        const int li = (int)(i - w.x0), lj = (int)(j - w.y0);
        const double gx[2][2] = {{w.gx[lj][li], w.gx[lj][li + 1]}, {w.gx[lj + 1][li], w.gx[lj + 1][li + 1]}};
        const double gy[2][2] = {{w.gy[lj][li], w.gy[lj][li + 1]}, {w.gy[lj + 1][li], w.gy[lj + 1][li + 1]}};
        const double fa = px - i, fb = py - j;
        double dx = interp2_patch(fa, fb, gx);
        double dy = interp2_patch(fa, fb, gy);
        if (__builtin_isnan(dx) || __builtin_isnan(dy)) {
            // NaN fallback (:178-218) as the reference behaves under numpy 2: the neighbour
            // probe `np.uint32(nearN + [0,-1])` raises OverflowError, caught at :217.
            if (lead) {
                int64_t nx = (int64_t)__builtin_rint(px), ny = (int64_t)__builtin_rint(py);
                bool empty = false, oob = false;
                for (;;) {
                    const int64_t wx = nx < 0 ? nx + W : nx, wy = ny < 0 ? ny + H : ny;
                    if (wx < 0 || wy < 0 || wx >= W || wy >= H) { oob = true; break; }
                    if (!__builtin_isinf(tv(T, W, wy, wx))) break;
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
            break;
        }
        double sx, sy;
        if (norm2(dx, dy) < 0.01) {  // :220-224
            const double dnx = dx / __builtin_sqrt(dx * dx + dy * dy);
            const double dny = dy / __builtin_sqrt(dx * dx + dy * dy);
            sx = px - tau * dnx;
            sy = py - tau * dny;
        } else {  // :225-229 (dy normalised with the already-normalised dx)
            dx = dx / __builtin_sqrt(dx * dx + dy * dy);
            dy = dy / __builtin_sqrt(dx * dx + dy * dy);
            sx = px - tau * dx;
            sy = py - tau * dy;
        }
        if (n >= a.cap) { status = kGdmError; break; }
        if (lead) {
            out[2 * n] = sx;
            out[2 * n + 1] = sy;
        }
        ++n;
        px = sx;
        py = sy;
        if (norm2(sx - a.ex, sy - a.ey) < 1.5) break;  // :231-232
    }
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

hipError_t gdm2d(const Gdm2dArgs& a, bool f64, hipStream_t st) {
    if (f64)
        hipLaunchKernelGGL(gdm2d_kernel<double>, dim3(1), dim3(64), 0, st, a);
    else
        hipLaunchKernelGGL(gdm2d_kernel<float>, dim3(1), dim3(64), 0, st, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------- 3D path (FM3D)
// np.gradient(T) along `axis` (0 y, 1 x, 2 z) at (j, i, k): central differences / 2 inside,
// one-sided at the ends (numpy's edge_order=1), no inf awareness (FastMarching3D.py:200).
template <typename R>
__device__ __forceinline__ double npgrad(const R* __restrict__ T, int64_t H, int64_t W, int64_t L, int axis,
                                         int64_t j, int64_t i, int64_t k) {
    const int64_t len = axis == 0 ? H : axis == 1 ? W : L;
    const int64_t p = axis == 0 ? j : axis == 1 ? i : k;
    const int64_t st = axis == 0 ? W * L : axis == 1 ? L : 1;
    const R* c = T + (j * W + i) * L + k;
    if (p == 0) return ((double)c[st] - (double)c[0]) / 1.0;
    if (p == len - 1) return ((double)c[0] - (double)c[-st]) / 1.0;
    return ((double)c[st] - (double)c[-st]) / 2.0;
}

// FastMarching3D.interpolatePoint :275-314, interior branch (a7 coefficient as written, :290)
template <typename R>
__device__ double interp3(const R* __restrict__ T, int64_t H, int64_t W, int64_t L, int axis, double px, double py,
                          double pz, bool& oob) {
    const uint32_t i = (uint32_t)__builtin_trunc(px), j = (uint32_t)__builtin_trunc(py), k = (uint32_t)__builtin_trunc(pz);
    oob = i + 1 >= (uint64_t)W || j + 1 >= (uint64_t)H || k + 1 >= (uint64_t)L;
    if (oob) return 0.0;
    const double a = px - i, b = py - j, c = pz - k;
    const double m000 = npgrad(T, H, W, L, axis, j, i, k), m010 = npgrad(T, H, W, L, axis, j, i + 1, k);
    const double m100 = npgrad(T, H, W, L, axis, j + 1, i, k), m001 = npgrad(T, H, W, L, axis, j, i, k + 1);
    const double m110 = npgrad(T, H, W, L, axis, j + 1, i + 1, k), m011 = npgrad(T, H, W, L, axis, j, i + 1, k + 1);
    const double m101 = npgrad(T, H, W, L, axis, j + 1, i, k + 1), m111 = npgrad(T, H, W, L, axis, j + 1, i + 1, k + 1);
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

__device__ __forceinline__ double norm3(double a, double b, double c) { return __builtin_sqrt(a * a + b * b + c * c); }

template <typename R>
__global__ __launch_bounds__(64) void gdm3d_kernel(Gdm3dArgs a) {
    if (threadIdx.x != 0) return;
    const R* __restrict__ T = static_cast<const R*>(a.T);
    const int64_t H = a.H, W = a.W, L = a.L;
    double* out = a.out;
    int64_t n = 1;
    int status = kGdmDone;
    out[0] = a.init[0];
    out[1] = a.init[1];
    out[2] = a.init[2];
    const double tau = a.tau;
    const int off[6][3] = {{0, -1, 0}, {0, 1, 0}, {-1, 0, 0}, {1, 0, 0}, {0, 0, -1}, {0, 0, 1}};
    for (long k = 0; k < a.steps; ++k) {
        const double* g = out + 3 * (n - 1);
        bool o1, o2, o3;
        double dx = interp3<R>(T, H, W, L, 1, g[0], g[1], g[2], o1);
        double dy = interp3<R>(T, H, W, L, 0, g[0], g[1], g[2], o2);
        double dz = interp3<R>(T, H, W, L, 2, g[0], g[1], g[2], o3);
        if (o1 || o2 || o3) { status = kGdmError; break; }
        if (__builtin_isnan(dx) || __builtin_isnan(dy) || __builtin_isnan(dz)) {  // :212-253
            int64_t nx = (int64_t)__builtin_rint(g[0]), ny = (int64_t)__builtin_rint(g[1]), nz = (int64_t)__builtin_rint(g[2]);
            bool err = false;
            for (;;) {
                if (nx < 0 || ny < 0 || nz < 0 || nx >= W || ny >= H || nz >= L) { err = true; break; }
                if (!__builtin_isinf((double)T[(ny * W + nx) * L + nz])) break;
                --n;
                if (n == 0) { err = true; break; }
                const double* q = out + 3 * (n - 1);
                nx = (int64_t)__builtin_rint(q[0]);
                ny = (int64_t)__builtin_rint(q[1]);
                nz = (int64_t)__builtin_rint(q[2]);
            }
            if (err) { status = kGdmError; break; }
            while (n > 0 && norm3(out[3 * (n - 1)] - nx, out[3 * (n - 1) + 1] - ny, out[3 * (n - 1) + 2] - nz) < 1) --n;
            if (n >= a.cap) { status = kGdmError; break; }
            out[3 * n] = (double)nx;
            out[3 * n + 1] = (double)ny;
            out[3 * n + 2] = (double)nz;
            ++n;
            double curT = (double)T[(ny * W + nx) * L + nz];
            for (int q = 0; q < 6; ++q) {
                int64_t cx = nx + off[q][0], cy = ny + off[q][1], cz = nz + off[q][2];
                if (cx < 0) cx += W;  // python negative indices wrap
                if (cy < 0) cy += H;
                if (cz < 0) cz += L;
                if (cx >= W || cy >= H || cz >= L) { err = true; break; }
                const double tc = (double)T[(cy * W + cx) * L + cz];
                if (tc < curT) {
                    curT = tc;
                    dx = (double)(-off[q][0]) / tau;
                    dy = (double)(-off[q][1]) / tau;
                    dz = (double)(-off[q][2]) / tau;
                }
            }
            if (err) { status = kGdmError; break; }
        }
        g = out + 3 * (n - 1);
        const double nrm = __builtin_sqrt(dx * dx + dy * dy + dz * dz);  // :255
        double ax, ay, az;
        if (nrm < 0.01) {
            ax = g[0] - tau * (dx / nrm);
            ay = g[1] - tau * (dy / nrm);
            az = g[2] - tau * (dz / nrm);
        } else {  // unnormalised step (:262-264)
            ax = g[0] - tau * dx;
            ay = g[1] - tau * dy;
            az = g[2] - tau * dz;
        }
        if (n >= a.cap) { status = kGdmError; break; }
        out[3 * n] = ax;
        out[3 * n + 1] = ay;
        out[3 * n + 2] = az;
        ++n;
        if (__builtin_isnan(ax) || __builtin_isnan(ay) || __builtin_isnan(az)) { status = kGdmError; break; }
        if (norm3(ax - a.end[0], ay - a.end[1], az - a.end[2]) < 1.5) break;  // :266-267
    }
    if (status == kGdmDone && n < a.cap) {  // :269
        out[3 * n] = a.end[0];
        out[3 * n + 1] = a.end[1];
        out[3 * n + 2] = a.end[2];
        ++n;
    }
    *a.n_out = n;
    *a.status = status;
}

hipError_t gdm3d(const Gdm3dArgs& a, bool f64, hipStream_t st) {
    if (f64)
        hipLaunchKernelGGL(gdm3d_kernel<double>, dim3(1), dim3(64), 0, st, a);
    else
        hipLaunchKernelGGL(gdm3d_kernel<float>, dim3(1), dim3(64), 0, st, a);
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
