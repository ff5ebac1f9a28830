// Accuracy probe (not product code): ulp error of the fp64 sweep's square-root forms against the
// correctly rounded __builtin_sqrt, on q = 2c^2 - d^2 drawn as the sweep draws it (c in
// [2^-20, 2^20], d in [0, c]).
//   hipcc --offload-arch=gfx950 -O3 tools/sqrt_ulp.hip -o tools/sqrt_ulp && tools/sqrt_ulp
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ unsigned long long mix(unsigned long long z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__device__ double u01(unsigned long long r) { return (double)(r >> 11) * 0x1p-53; }

// the product's form (eik_common.hpp sqrt_sweep): rsq, Goldschmidt step, one Newton correction
__device__ double sqrt_full(double q) {
    const double y = __builtin_amdgcn_rsq(q);
    double g = q * y, h = 0.5 * y;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    const double e = __builtin_fma(-g, g, q);
    return __builtin_fma(e, h, g);
}
// candidate: the Goldschmidt step only
__device__ double sqrt_gs(double q) {
    const double y = __builtin_amdgcn_rsq(q);
    const double g = q * y, h = 0.5 * y;
    const double r = __builtin_fma(-h, g, 0.5);
    return __builtin_fma(g, r, g);
}
// candidate: one Newton correction of g = q * rsq(q)
__device__ double sqrt_nt(double q) {
    const double y = __builtin_amdgcn_rsq(q);
    const double g = q * y;
    const double e = __builtin_fma(-g, g, q);
    return __builtin_fma(e, 0.5 * y, g);
}

__device__ long long ulps(double a, double b) {
    const long long x = __double_as_longlong(a), y = __double_as_longlong(b);
    return x > y ? x - y : y - x;
}

__global__ void probe(long long n, unsigned long long* hist) {  // hist[3][8]: |ulp| 0,1,2,3,4..7,8..63,>=64, NaN
    const long long i0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long loc[24] = {};
    for (long long i = i0; i < n; i += (long long)gridDim.x * blockDim.x) {
        const unsigned long long r1 = mix(2 * i + 1), r2 = mix(2 * i + 2);
        const double c = __builtin_ldexp(1.0 + u01(r1), (int)(r1 % 41) - 20);
        const double d = c * u01(r2);
        const double q = __builtin_fma(-d, d, 2 * c * c);
        const double ref = __builtin_sqrt(q);
        const double v[3] = {sqrt_full(q), sqrt_gs(q), sqrt_nt(q)};
        for (int k = 0; k < 3; ++k) {
            const long long u = ulps(v[k], ref);
            const int b = v[k] != v[k] ? 7 : u == 0 ? 0 : u == 1 ? 1 : u == 2 ? 2 : u == 3 ? 3 : u < 8 ? 4 : u < 64 ? 5 : 6;
            loc[8 * k + b]++;
        }
    }
    for (int k = 0; k < 24; ++k)
        if (loc[k]) atomicAdd(&hist[k], loc[k]);
}

int main() {
    unsigned long long* h;
    (void)hipMalloc(&h, 24 * 8);
    (void)hipMemset(h, 0, 24 * 8);
    const long long n = 1ll << 28;
    hipLaunchKernelGGL(probe, dim3(4096), dim3(256), 0, 0, n, h);
    unsigned long long hh[24];
    (void)hipMemcpy(hh, h, sizeof hh, hipMemcpyDeviceToHost);
    const char* names[3] = {"full (product)", "goldschmidt only", "one newton"};
    printf("ulp buckets: 0 1 2 3 4-7 8-63 >=64 NaN  over %lld samples\n", n);
    for (int k = 0; k < 3; ++k) {
        printf("%-18s", names[k]);
        for (int b = 0; b < 8; ++b) printf(" %llu", hh[8 * k + b]);
        printf("\n");
    }
    return 0;
}
