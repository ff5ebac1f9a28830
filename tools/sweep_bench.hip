// Microbenchmark (not product code): cycles per skewed-sweep step of the FIM tile body in
// isolation, for variants of the step.  (A register-resident variant -- each wave's tile copy in
// VGPRs with a skewed layout, no LDS per step -- measured 108 cycles/step alone and 138 with its
// per-pass LDS load/merge, vs 126 for V0, and lost intra-pass sharing between waves: dropped.)  One 64x64 fp32 tile staged in LDS per workgroup, the
// four quadrant sweeps run concurrently by the four waves, R repetitions, s_memtime around them.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/sweep_bench.hip -o /tmp/sweep_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "../planning-motion_planning_amd/csrc/fim2d.hip"
using namespace eik;

template <int V, int DX, int DY>
__device__ __forceinline__ void sweepv(float* Ts, int lane) {
    constexpr int S = 4, kRow = kLds * S, D = 4;
    char* const base = reinterpret_cast<char*>(Ts);
    auto ld = [&](int off) { return *reinterpret_cast<const float*>(base + off); };
    const int col = (DX > 0 ? lane : kTile - 1 - lane) + 1;
    const int lo_b = col * S, hi_b = (kLds - 1) * kRow + col * S;
    int raw = DY > 0 ? (1 - lane) * kRow + col * S : (kTile + lane) * kRow + col * S;
    auto clampb = [&](int x) { int r; asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(lo_b), "v"(hi_b)); return r; };
    float cur = ld((DY > 0 ? 0 : kLds - 1) * kRow + col * S);
    int q_o[D];
    float q_old[D], q_dnx[D], q_dny[D], q_upx[D], q_c[D];
    auto fetch = [&](int u) {
        const int o = clampb(raw);
        raw += DY * kRow;
        q_o[u] = o;
        q_old[u] = ld(o);
        q_dnx[u] = ld(o + DX * S);
        q_dny[u] = ld(o + DY * kRow);
        q_upx[u] = ld(o - DX * S);
        q_c[u] = ld(o + kCsOff * S);
    };
#pragma unroll
    for (int u = 0; u < D; ++u) fetch(u);
    for (int s = 0; s < 2 * kTile; s += D) {
#pragma unroll
        for (int u = 0; u < D; ++u) {
            const float upx = wave_shr1(cur, q_upx[u]);
            float w;
            if constexpr (V == 3) w = umin(umin(upx, q_dnx[u]), umin(cur, q_dny[u])) + q_c[u];  // no sqrt
            else w = godunov2_fast(umin(upx, q_dnx[u]), umin(cur, q_dny[u]), q_c[u]);
            if constexpr (V == 0 || V == 3) lds_min(reinterpret_cast<float*>(base + q_o[u]), w);
            if constexpr (V == 1) *reinterpret_cast<float*>(base + q_o[u]) = umin(w, q_old[u]);
            cur = umin(w, q_old[u]);
            if constexpr (V != 2) fetch(u); else { q_old[u] = cur; }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    if constexpr (V == 2) *reinterpret_cast<float*>(base + q_o[0]) = cur;
}

// V6: (T, cost) interleaved per cell (float2); per step ONE ds_read_b64 (the next row's pair)
// + the ds_min.  dny = own next pair; dnx = lane l+1's next pair (DPP wave_shl:1); upstream x
// (DPP wave_shr:1) as V0; the halo columns come from registers (lane k = tile row k) by readlane.
template <int DX, int DY>
__device__ __forceinline__ void sweep_pair(float2* TC, int lane, float hw, float he) {
    constexpr int S = 8, kRow = kLds * S, D = 4;
    char* const base = reinterpret_cast<char*>(TC);
    auto ld = [&](int off) { return *reinterpret_cast<const float2*>(base + off); };
    const int col = (DX > 0 ? lane : kTile - 1 - lane) + 1;
    const int lo_b = col * S, hi_b = (kLds - 1) * kRow + col * S;
    int raw = DY > 0 ? (1 - lane) * kRow + col * S : (kTile + lane) * kRow + col * S;
    auto clampb = [&](int x) { int r; asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(lo_b), "v"(hi_b)); return r; };
    float cur = ld((DY > 0 ? 0 : kLds - 1) * kRow + col * S).x;
    int o_cur = clampb(raw);
    float2 p_cur = ld(o_cur);
    raw += DY * kRow;
    const float hu = DX > 0 ? hw : he, hd = DX > 0 ? he : hw;
    int q_o[D];
    float2 q_p[D];
    auto fetch = [&](int u) {
        const int o = clampb(raw);
        raw += DY * kRow;
        q_o[u] = o;
        q_p[u] = ld(o);
    };
#pragma unroll
    for (int u = 0; u < D; ++u) fetch(u);
    for (int s = 0; s < 2 * kTile; s += D) {
#pragma unroll
        for (int u = 0; u < D; ++u) {
            const int t = s + u;
            const int iu = (DY > 0 ? t : kTile - 1 - t) & (kTile - 1);
            const int id = (DY > 0 ? t - (kTile - 1) : 2 * (kTile - 1) - t) & (kTile - 1);
            const int uh = __builtin_amdgcn_readlane(__float_as_int(hu), iu);
            const int dh = __builtin_amdgcn_readlane(__float_as_int(hd), id);
            const float ux = __int_as_float(__builtin_amdgcn_update_dpp(uh, __float_as_int(cur), 0x138, 0xF, 0xF, false));
            const float dx = __int_as_float(__builtin_amdgcn_update_dpp(dh, __float_as_int(q_p[u].x), 0x130, 0xF, 0xF, false));
            const float w = godunov2_fast(umin(ux, dx), umin(cur, q_p[u].x), p_cur.y);
            lds_min(reinterpret_cast<float*>(base + o_cur), w);
            cur = umin(w, p_cur.x);
            p_cur = q_p[u];
            o_cur = q_o[u];
            fetch(u);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

__global__ __launch_bounds__(256) void kern_pair(const float* cost, float* out, unsigned long long* cyc, int reps) {
    __shared__ float2 TC[(kLds + 2) * kLds];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < (kLds + 2) * kLds; i += 256) {
        const int j = i - kLds;  // ring index
        TC[i] = make_float2((i % 97 == 0) ? 0.f : __builtin_inff(), (j >= 0 && j < kLds * kLds) ? cost[j] : __builtin_inff());
    }
    __syncthreads();
    float2* Ts = TC + kLds;
    const float hw = Ts[(lane + 1) * kLds].x, he = Ts[(lane + 1) * kLds + kLds - 1].x;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        if (wave == 0) sweep_pair<+1, +1>(Ts, lane, hw, he);
        else if (wave == 1) sweep_pair<-1, +1>(Ts, lane, hw, he);
        else if (wave == 2) sweep_pair<+1, -1>(Ts, lane, hw, he);
        else sweep_pair<-1, -1>(Ts, lane, hw, he);
        __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 256 + tid] = Ts[tid * 3].x;
}

template <int V>
__global__ __launch_bounds__(256) void kern(const float* cost, float* out, unsigned long long* cyc, int reps) {
    __shared__ float Tbuf[(kLds + 2) * kLds];
    __shared__ float Cs[kLds * kLds];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < (kLds + 2) * kLds; i += 256) Tbuf[i] = (i % 97 == 0) ? 0.f : __builtin_inff();
    for (int i = tid; i < kLds * kLds; i += 256) Cs[i] = cost[i];
    __syncthreads();
    float* Ts = Tbuf + kLds;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        if (wave == 0) sweepv<V, +1, +1>(Ts, lane);
        else if (wave == 1) sweepv<V, -1, +1>(Ts, lane);
        else if (wave == 2) sweepv<V, +1, -1>(Ts, lane);
        else sweepv<V, -1, -1>(Ts, lane);
        __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 256 + tid] = Ts[tid * 3];
}

template <int V>
void run(const char* name, const float* cost, float* out, unsigned long long* cyc, int grid, int reps) {
    auto launch = [&]() {
        if constexpr (V == 6) hipLaunchKernelGGL(kern_pair, dim3(grid), dim3(256), 0, 0, cost, out, cyc, reps);
        else hipLaunchKernelGGL(kern<V>, dim3(grid), dim3(256), 0, 0, cost, out, cyc, reps);
    };
    launch();
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    launch();
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("%-28s grid %5d: %.2f us per sweep pass (event), %.1f memtime ticks/step (block 0)\n", name, grid,
           ms * 1e3 / reps, (double)c / reps / 128.0);
}

int main() {
    float* cost; float* out; unsigned long long* cyc;
    hipMalloc(&cost, 4 * kLds * kLds); hipMalloc(&out, 4 * 256 * 2048); hipMalloc(&cyc, 8 * 2048);
    float h[kLds * kLds]; for (int i = 0; i < kLds * kLds; ++i) h[i] = 1.f + (i % 7);
    hipMemcpy(cost, h, sizeof h, hipMemcpyHostToDevice);
    const int reps = 200;
    for (int grid : {1, 256, 1024}) {
        run<0>("V0 ds_min (product)", cost, out, cyc, grid, reps);
        run<1>("V1 plain ds_write", cost, out, cyc, grid, reps);
        run<2>("V2 no LDS in loop", cost, out, cyc, grid, reps);
        run<3>("V3 ds_min, no sqrt", cost, out, cyc, grid, reps);
        run<6>("V6 (T,c) pairs, 1 read", cost, out, cyc, grid, reps);
    }
    return 0;
}
