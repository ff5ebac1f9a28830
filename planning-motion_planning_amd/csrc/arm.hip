// arm.hip -- the planner's end-effector cost volume on gfx950.
//
// Coupled_motion_planner.py builds the volume the arm's FM3D solve runs on from two pieces:
//  * GetObstMap (:319-358): 2 everywhere, +inf on the DEM surface cell of every column and on the
//    volume's faces -- one thread per DEM column (arm_obst_*);
//  * TunnelCost (:505-725): a Python triple loop that "paints" a tunnel of radius rlim around the
//    arm base path, closes it behind the first base point and caps it with a half sphere at the
//    last one.  Each loop iteration is an EVENT on one cell: an assign (value v only if the cell
//    still holds 10) or a close (+inf, unconditional; never at the start / sample nodes).  Closes
//    are absorbing and an assign after any write is a no-op, so the final value of a cell is +inf
//    if any close hits it, else the value of the first assign (in loop order) that hits it, else 10
//    (oracle/arm_oracle.py derives this and is pinned to the reference's own outputs).  On the GPU
//    every event is one thread, numbered in the reference's loop order: pass 1 marks closes and
//    takes the atomic minimum of the assigns' sequence numbers per cell, pass 2 lets the winning
//    assign store its value, a per-cell pass resolves and multiplies with GetObstMap's map (the
//    planner's Cmap = Cmap1 * Cmap2, :1580).
// Arithmetic follows the reference bit for bit: the transforms' trig and the linspace / norm /
// value tables are formed on the host in Python-float order; positions are column 3 of Toa . Tap
// in the order numpy's dot evaluates it (OpenBLAS dgemm: a0 x, then fused multiply-adds of the
// remaining terms, pinned by tests/test_arm_oracle.py); node indices are round-half-even of
// position / resolution.  Memory: the volume and one u32 + one u8 per cell; events are recomputed
// in pass 2 instead of stored.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "eik_kernels.hpp"

namespace eik {

__device__ __forceinline__ double tdot(const double* t, double x, double y, double z) {
    // numpy dot (OpenBLAS): ((t0 x + t1 y) + t2 z) + t3 . 1 as a chain of fused multiply-adds
    return __fma_rn(t[3], 1.0, __fma_rn(t[2], z, __fma_rn(t[1], y, __dmul_rn(t[0], x))));
}

struct Ev {
    long long cell;  // -1: no write
    bool close;
    double v;
};

__device__ __forceinline__ Ev arm_event(const ArmArgs& a, unsigned long long s) {
    double X, Y, Z, v = 0.0;
    const double* T;
    bool want = false, close = false;
    if (s < a.nA) {  // :524-611 -- per base point j, per (i, k): the point, then the forward neighbour
        const unsigned long long per = 2ull * a.nX * a.nZ;
        const int j = (int)(s / per);
        const unsigned r = (unsigned)(s - (unsigned long long)j * per);
        const unsigned ik = r >> 1, sub = r & 1u;
        X = a.tabI[ik / a.nZ];
        Z = a.tabK[ik % a.nZ];
        Y = sub ? a.resY : 0.0;
        T = a.toaA + 12 * j;
        const bool inside = a.norm[ik] < a.rlim;
        v = a.valA[ik];
        want = inside || sub == 0;
        close = !inside;  // sub 0 outside the reach: close; sub 1 outside: nothing (want false)
    } else if (s < a.nA + a.nB) {  // :613-650 -- the first base point, one step back
        const unsigned ik = (unsigned)(s - a.nA);
        X = a.tabI[ik / a.nZ];
        Z = a.tabK[ik % a.nZ];
        Y = -a.resY;
        T = a.toaB;
        want = a.norm[ik] < a.rlim;
        close = true;
    } else {  // :652-723 -- the half sphere at the last base point
        const unsigned long long c = s - a.nA - a.nB;
        const unsigned kk = (unsigned)(c % (unsigned long long)(a.nK + 1));
        const unsigned ts = (unsigned)(c / (unsigned long long)(a.nK + 1));
        const unsigned si = ts % 90u, ti = ts / 90u;
        const double ct = a.ct[ti], st = a.st[ti], cs = a.cs[si], ss = a.ss[si];
        const double k = kk < (unsigned)a.nK ? a.ks[kk] : a.rad;
        const double kc = __dmul_rn(k, ct);
        X = __dmul_rn(kc, cs);
        Y = __dmul_rn(kc, ss);
        Z = __dmul_rn(k, st);
        T = a.toaC;
        want = true;
        close = kk == (unsigned)a.nK;
        if (!close) v = a.valC[kk];
    }
    Ev e{-1, close, v};
    if (!want) return e;
    const long long ix = (long long)rint(__ddiv_rn(tdot(T, X, Y, Z), a.resX));
    const long long iy = (long long)rint(__ddiv_rn(tdot(T + 4, X, Y, Z), a.resY));
    const long long iz = (long long)rint(__ddiv_rn(tdot(T + 8, X, Y, Z), a.resZ));
    if (ix < 0 || iy < 0 || iz < 0 || ix >= a.sX || iy >= a.sY || iz >= a.sZ) return e;
    if (close && ((ix == a.fw[0] && iy == a.fw[1] && iz == a.fw[2]) || (ix == a.iw[0] && iy == a.iw[1] && iz == a.iw[2])))
        return e;  // never the sample / start node
    e.cell = (iy * a.sX + ix) * a.sZ + iz;
    return e;
}

__global__ void arm_events_mark(ArmArgs a) {
    const unsigned long long n = a.nA + a.nB + a.nC;
    for (unsigned long long s = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; s < n;
         s += (unsigned long long)gridDim.x * blockDim.x) {
        const Ev e = arm_event(a, s);
        if (e.cell < 0) continue;
        if (e.close)
            a.closed[e.cell] = 1;  // every writer stores 1: benign
        else
            atomicMin(a.first + e.cell, (unsigned)s);
    }
}

__global__ void arm_events_assign(ArmArgs a) {
    const unsigned long long n = a.nA + a.nB + a.nC;
    for (unsigned long long s = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; s < n;
         s += (unsigned long long)gridDim.x * blockDim.x) {
        const Ev e = arm_event(a, s);
        if (e.cell >= 0 && !e.close && a.first[e.cell] == (unsigned)s) a.tunnel[e.cell] = e.v;  // one winner
    }
}

// tunnel = inf / first assign / 10; out (nullable) = obst_final * tunnel (:1580)
__global__ void arm_resolve(ArmArgs a, long long ncell) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ncell) return;
    const double t = a.closed[i] ? __builtin_inf() : (a.first[i] == 0xffffffffu ? 10.0 : a.tunnel[i]);
    a.tunnel[i] = t;
    if (a.out) a.out[i] = a.fmap[i] * t;
}

// GetObstMap :323-355.  fill: obstMap = groundMap = 1, finalMap = 2, faces +inf
__global__ void arm_obst_fill(double* fmap, double* omap, double* gmap, long long sXY, long long sY, long long sZ) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long n = sXY * sZ;
    if (i >= n) return;
    const long long z = i % sZ, c = i / sZ, x = c % sY, y = c / sY;  // [y][x][z], sX rows of sY
    const long long sX = sXY / sY;
    const bool face = x == 0 || x == sY - 1 || y == 0 || y == sX - 1 || z == 0 || z == sZ - 1;
    fmap[i] = face ? __builtin_inf() : 2.0;
    if (omap) omap[i] = 1.0;
    if (gmap) gmap[i] = 1.0;
}

// one thread per DEM column (j, i): the surface cell becomes +inf in obstMap or groundMap and so
// in finalMap (:327-345).  A negative z index wraps as numpy's does; *bad flags one that cannot.
__global__ void arm_obst_columns(const double* Zs, const double* obst, long long m, long long n, double resX,
                                 double resY, double resZ, long long sX, long long sY, long long sZ, double xm,
                                 double ym, double* fmap, double* omap, double* gmap, unsigned* bad) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= m * n) return;
    const long long j = t / n, i = t % n;  // j: DEM row (y), i: column (x)
    if (__dmul_rn(resX, (double)i) == xm || __dmul_rn(resY, (double)j) == ym) return;
    long long iz = (long long)rint(__ddiv_rn(Zs[t], resZ));
    if (!(i < sX && j < sY && iz < sZ)) return;
    if (iz < 0) iz += sZ;
    if (iz < 0) {
        atomicOr(bad, 1u);
        return;
    }
    const long long c = (j * sY + i) * sZ + iz;
    if (obst[t] == 1.0) {
        if (omap) omap[c] = __builtin_inf();
    } else {
        if (gmap) gmap[c] = __builtin_inf();
    }
    fmap[c] = __builtin_inf();
}

hipError_t arm_obst_map(const double* Zs, const double* obst, int64_t m, int64_t n, double resX, double resY,
                        double resZ, int64_t sX, int64_t sY, int64_t sZ, double xm, double ym, double* fmap,
                        double* omap, double* gmap, unsigned* bad, hipStream_t st) {
    const long long nc = (long long)sX * sY * sZ;
    hipLaunchKernelGGL(arm_obst_fill, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, st, fmap, omap, gmap,
                       (long long)sX * sY, (long long)sY, (long long)sZ);
    const long long nt = (long long)m * n;
    if (nt > 0)
        hipLaunchKernelGGL(arm_obst_columns, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, st, Zs, obst,
                           (long long)m, (long long)n, resX, resY, resZ, (long long)sX, (long long)sY, (long long)sZ,
                           xm, ym, fmap, omap, gmap, bad);
    return hipGetLastError();
}

hipError_t arm_tunnel(const ArmArgs& a, hipStream_t st) {
    const long long nc = (long long)a.sX * a.sY * a.sZ;
    hipError_t e = hipMemsetAsync(a.first, 0xff, sizeof(unsigned) * nc, st);
    if (e == hipSuccess) e = hipMemsetAsync(a.closed, 0, nc, st);
    if (e != hipSuccess) return e;
    const unsigned long long n = a.nA + a.nB + a.nC;
    const unsigned grid = (unsigned)std::min<unsigned long long>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(arm_events_mark, dim3(grid), dim3(256), 0, st, a);
    hipLaunchKernelGGL(arm_events_assign, dim3(grid), dim3(256), 0, st, a);
    hipLaunchKernelGGL(arm_resolve, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, st, a, nc);
    return hipGetLastError();
}

}  // namespace eik
