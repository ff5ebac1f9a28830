// Profiling harness (not product code): the persistent FIM kernel built with per-workgroup
// phase timers through the EIK_PROBE / EIK_VISIT hooks of fim2d.hip.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/qprof.hip -o tools/qprof
//   python tools/dumpcost.py 4096 /tmp/c.f32 && tools/qprof 4096 1024 /tmp/c.f32

#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>
__device__ unsigned long long* g_prof;
#define EIK_PROBE(k) do { if (threadIdx.x == 0) { const unsigned long long t_ = __builtin_amdgcn_s_memrealtime(); \
    unsigned long long* p_ = g_prof + blockIdx.x * 32; if (p_[15]) { p_[k] += t_ - p_[15]; p_[8 + k]++; } p_[15] = t_; } } while (0)
#define EIK_VISIT(tile, trig, dirs) do { unsigned long long* p_ = g_prof + blockIdx.x * 32; p_[16] += __builtin_popcount(dirs); p_[17] += ((trig) & 64u) ? 1 : 0; } while (0)
#include "../planning-motion_planning_amd/csrc/fim2d.hip"
using namespace eik;
#define CK(x) do { hipError_t e = (x); if (e) { printf("%s -> %s\n", #x, hipGetErrorString(e)); exit(2);} } while (0)
int main(int argc, char** argv) {
    int N = atoi(argv[1]), grid = atoi(argv[2]);
    const char* cf = argc > 3 && strcmp(argv[3], "-") != 0 ? argv[3] : nullptr;  // "-": uniform cost
    int rounds = argc > 4 ? atoi(argv[4]) : 1;
    std::vector<float> hc((size_t)N * N, 1.f);
    if (cf) { FILE* f = fopen(cf, "rb"); if (!f || fread(hc.data(), 4, hc.size(), f) != hc.size()) { printf("bad cost file\n"); return 2; } fclose(f); }
    unsigned long long* prof; CK(hipMalloc(&prof, 8ull * 32 * grid));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_prof), &prof, sizeof prof));
    Fim2dArgs a{};
    int ntx = (N + 63) / 64, tiles = ntx * ntx;
    float *cost, *T; CK(hipMalloc(&cost, 4ull * N * N)); CK(hipMalloc(&T, 4ull * N * N));
    CK(hipMemcpy(cost, hc.data(), 4ull * N * N, hipMemcpyHostToDevice));
    a.cost = cost; a.T = T; a.H = N; a.W = N; a.ntx = ntx; a.nty = ntx; a.tiles_per_map = tiles;
    CK(hipMalloc(&a.lists, 12ull * tiles)); CK(hipMalloc(&a.counts, 256)); CK(hipMalloc(&a.mark, 4ull * tiles));
    a.capacity = tiles; a.max_rounds = rounds; a.keep = 1.f - (argc > 5 ? (float)atof(argv[5]) : 0.f); CK(hipMalloc(&a.key, 4ull * tiles)); a.minkey = (unsigned*)a.counts + 16;
    a.delta = __builtin_inff(); CK(hipMalloc(&a.visits, 16));
    char* q; CK(hipMalloc(&q, 256)); a.qhead = (unsigned long long*)q; a.qtail = (unsigned long long*)(q + 64);
    a.qactive = (int*)(q + 128); a.qerror = (unsigned*)(q + 192); a.mode = kModePersistent;
    unsigned qn = 4096; while (qn < 8u * tiles) qn <<= 1;
    a.qmask = qn - 1; CK(hipMalloc(&a.qslot, 4ull * qn)); CK(hipMalloc(&a.qstate, 4ull * tiles));
    a.qtimeout = 1000000000ull; a.qbudget = 1ull << 40; a.max_passes = 8;
    a.ls = 1; a.z0 = 0;
    a.fresh_first = getenv("EIK_FRESH_FIRST") && atoi(getenv("EIK_FRESH_FIRST")) == 1;
    a.sched = getenv("EIK_SCHED") ? atoi(getenv("EIK_SCHED")) : 0;
    int64_t* goals; CK(hipMalloc(&goals, 16)); int64_t hg[2] = {N / 2, N / 2}; CK(hipMemcpy(goals, hg, 16, hipMemcpyHostToDevice));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    float ms = 0;
    for (int rep = 0; rep < 4; ++rep) {
        CK(hipMemset(a.visits, 0, 16)); CK(hipMemset(prof, 0, 8ull * 32 * grid));
        CK(fim2d_init(a, false, 1, goals, 0));
        CK(hipEventRecord(e0, 0));
        CK(fim2d_persist(a, false, grid, 0));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
    }
    unsigned hq[64]; CK(hipMemcpy(hq, q, 256, hipMemcpyDeviceToHost));
    unsigned long long vv[2]; CK(hipMemcpy(vv, a.visits, 16, hipMemcpyDeviceToHost)); unsigned long long v = vv[0];
    std::vector<unsigned long long> hp(32ull * grid); CK(hipMemcpy(hp.data(), prof, 8ull * 32 * grid, hipMemcpyDeviceToHost));
    double acc[8] = {0}, cnt[8] = {0};
    for (int b = 0; b < grid; ++b) for (int k = 0; k < 7; ++k) { if (k == 7) continue; acc[k] += hp[b * 32 + k] * 1e-2; cnt[k] += hp[b * 32 + 8 + k]; }
    const char* nm[7] = {"to-stage", "stage", "sweep", "wback+drain", "to-post", "post(act+fin)", "grab+barrier"};
    printf("N=%d grid=%d rounds=%d keep=1-%.1e: kernel %.3f ms, visits %llu (+%llu in place), err %u, active %d\n", N, grid, rounds, 1.0 - a.keep, ms, v, vv[1], hq[48], (int)hq[32]);
    double sw = 0, self = 0; for (int b = 0; b < grid; ++b) { sw += hp[b * 32 + 16]; self += hp[b * 32 + 17]; }
    printf("  sweeps/visit %.3f, self-triggered visits %.1f%%\n", sw / v, 100.0 * self / v);
    double busy = 0;
    for (int k = 0; k < 7; ++k) {
        printf("  %-14s total %10.1f us  per-event %7.2f us  (n=%.0f)\n", nm[k], acc[k], cnt[k] ? acc[k] / cnt[k] : 0, cnt[k]);
        if (k != 6) busy += acc[k];
    }
    printf("  avg busy WGs %.1f of %d (%.1f%%)\n", busy / (ms * 1e3), grid, 100.0 * busy / (ms * 1e3) / grid);
    return 0;
}
