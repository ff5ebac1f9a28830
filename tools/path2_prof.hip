// Phase timing of the 2D path walker (not product code): gdm.hip built with EIK_P2PROBE stamps
// (s_memtime by lane 0, accumulated per phase) on a smooth synthetic field (T = distance).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/path2_prof.hip -o /tmp/p2 && /tmp/p2
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
__device__ unsigned long long g_p2[16];
// accumulators in SGPRs (uniform), one store at the end: the stamp costs ~40 cycles + its wait
// (-DP2_NOPROBE: the product kernel, for the un-instrumented time)
#ifndef P2_NOPROBE
#define EIK_P2DECL unsigned long long p2a_[4] = {0, 0, 0, 0}, p2t_ = 0
#define EIK_P2PROBE(k) do { unsigned long long t_; asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_) :: "memory"); \
    if (p2t_) p2a_[k] += t_ - p2t_; p2t_ = t_; } while (0)
#define EIK_P2FLUSH do { if (threadIdx.x == 0) for (int q_ = 0; q_ < 4; ++q_) g_p2[q_] = p2a_[q_]; } while (0)
#endif
#include "../planning-motion_planning_amd/csrc/gdm.hip"
using namespace eik;
int main(int argc, char** argv) {
    // default: smooth synthetic field; or: p2 <T.f32 file> (4096^2, the bench field, goal 2048,2048, start 256,256)
    const int H = 4096, W = 4096;
    std::vector<float> hT((size_t)H * W);
    int gx = W - 300, gy = H - 200, sx = 200, sy = 300;
    if (argc > 1) {
        FILE* f = fopen(argv[1], "rb");
        if (!f || fread(hT.data(), 4, hT.size(), f) != hT.size()) { printf("bad T file\n"); return 2; }
        fclose(f);
        gx = 2048; gy = 2048; sx = 256; sy = 256;
    } else {
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) hT[(size_t)y * W + x] = std::hypot(x - gx, (y - gy) * 1.3f) + 20.f * std::sin(x * 0.01f);
    }
    float* T; double* out; long long* n; int* st;
    (void)hipMalloc(&T, hT.size() * 4); (void)hipMalloc(&out, 30004 * 16); (void)hipMalloc(&n, 8); (void)hipMalloc(&st, 4);
    (void)hipMemcpy(T, hT.data(), hT.size() * 4, hipMemcpyHostToDevice);
    Gdm2dArgs a{};
    a.T = T; a.H = H; a.W = W; a.ix = sx; a.iy = sy; a.ex = gx; a.ey = gy; a.tau = 0.5; a.steps = 30000;
    a.out = out; a.cap = 30004; a.n_out = (int64_t*)n; a.status = st; a.fused = getenv("FUSED") ? atoi(getenv("FUSED")) : 2;
    unsigned long long z[16] = {0};
    for (int rep = 0; rep < 2; ++rep) {
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_p2), z, sizeof z);
        hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        (void)gdm2d(a, false, 0);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        long long hn; int hs; (void)hipMemcpy(&hn, n, 8, hipMemcpyDeviceToHost); (void)hipMemcpy(&hs, st, 4, hipMemcpyDeviceToHost);
        unsigned long long p[16]; (void)hipMemcpyFromSymbol(p, HIP_SYMBOL(g_p2), sizeof p);
        printf("rep %d: %.3f ms, %lld points (%.3f us/step), status %d\n", rep, ms, hn, ms * 1e3 / hn, hs);
        const char* nm[4] = {"stop check->top", "window", "corners+interp", "normalise+step"};
        for (int k = 0; k < 4; ++k) printf("  %-18s %8.1f cycles/step\n", nm[k], (double)p[k] / hn);
    }
    return 0;
}
