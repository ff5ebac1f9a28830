// Microbenchmark (not product code): the PRODUCT quadrant sweep (fim2d.hip sweep_quadrant, with
// whatever -D flags the build gets) on one staged 64x64 fp32 tile per workgroup, the four
// directions run concurrently by the four waves, `reps` passes; cycles per sweep step.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 [-DEIK_OMOD=1 ...] tools/step_bench.hip -o /tmp/step_bench
#include "../planning-motion_planning_amd/csrc/fim2d.hip"
#include <cstdio>
using namespace eik;

__global__ __launch_bounds__(256) void kern(const float* cost, float* out, unsigned long long* cyc, int reps) {
    __shared__ TileLds<float> L;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < (kLds + 2 * kGuard) * kLds; i += 256) {
        const int row = i / kLds - kGuard, colx = i % kLds;
        const bool inner = row >= 1 && row <= kTile && colx >= 1 && colx <= kTile;
        L.Tc[i].t = (i % 97 == 0 && inner) ? 0.f : __builtin_inff();
        L.Tc[i].c = inner ? cost[(row - 1) * kTile + colx - 1] : __builtin_inff();
    }
    __syncthreads();
    Cell<float>* Ts = L.Tc + kGuard * kLds;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        if (wave == 0) sweep_quadrant<float, +1, +1, false>(Ts, lane, 1.f);
        else if (wave == 1) sweep_quadrant<float, -1, +1, false>(Ts, lane, 1.f);
        else if (wave == 2) sweep_quadrant<float, +1, -1, false>(Ts, lane, 1.f);
        else sweep_quadrant<float, -1, -1, false>(Ts, lane, 1.f);
        __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 256 + tid] = Ts[tid * 3 + kLds].t;
}

int main() {
    float* cost; float* out; unsigned long long* cyc;
    hipMalloc(&cost, 4 * kTile * kTile); hipMalloc(&out, 4 * 256 * 2048); hipMalloc(&cyc, 8 * 2048);
    static float h[kTile * kTile]; for (int i = 0; i < kTile * kTile; ++i) h[i] = 1.f + (i % 7);
    hipMemcpy(cost, h, sizeof h, hipMemcpyHostToDevice);
    const int reps = 200;
    for (int grid : {1, 256, 768, 1024}) {
        auto launch = [&]() { hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, cost, out, cyc, reps); };
        launch();
        hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
        hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        unsigned long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("grid %5d: %.2f us per pass (event), %.1f memtime ticks/step (block 0), %.1f ps/cell-update chip-wide\n",
               grid, ms * 1e3 / reps, (double)c / reps / 128.0, ms * 1e9 / reps / (grid * 4096.0 * 4));
    }
    return 0;
}
