// Event-trace harness (not product code): the persistent FIM kernel built with per-workgroup
// event logs through the EIK_PROBE / EIK_VISIT / EIK_ACT hooks of fim2d.hip / fim_engine.hpp.
// Unlike tools/qprof.hip a probe only stores (no dependent global load), so the trace costs a
// few hundred cycles per event.  tools/trace_an.py reconstructs every visit and the solve's
// critical chain of activations from the logs.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/trace.hip -o tools/trace
//   tools/trace N grid cost.f32|- out.bin [passes]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>

constexpr unsigned kCap = 8192;  // events per workgroup
__device__ unsigned long long* g_ev;
__shared__ unsigned tr_n;
// event: type:4 | aux:8 | tile:20 | time:32 (s_memrealtime, 100 MHz, low 32 bits)
__device__ __forceinline__ void tr_put(unsigned type, unsigned aux, unsigned tile) {
    const unsigned i = atomicAdd(&tr_n, 1u);
    if (i < kCap) {
        const unsigned long long t = __builtin_amdgcn_s_memrealtime();
        g_ev[(unsigned long long)blockIdx.x * kCap + i] =
            ((unsigned long long)type << 60) | ((unsigned long long)(aux & 0xff) << 52) |
            ((unsigned long long)(tile & 0xfffff) << 32) | (t & 0xffffffffull);
    }
}
#define EIK_KSTART() do { if (threadIdx.x == 0) tr_n = 0; __syncthreads(); } while (0)
#define EIK_PROBE(k) do { if (threadIdx.x == 0) tr_put(1 + (k), 0, 0); } while (0)
#define EIK_VISIT(tile, trig, dirs) tr_put(9, (trig), (tile))
#define EIK_ACT(tile, old) do { if (gridDim.x > 1) tr_put(10, (old), (tile)); } while (0)
#include "../planning-motion_planning_amd/csrc/fim2d.hip"
using namespace eik;
#define CK(x) do { hipError_t e = (x); if (e) { printf("%s -> %s\n", #x, hipGetErrorString(e)); exit(2);} } while (0)
int main(int argc, char** argv) {
    if (argc < 5) { printf("usage: trace N grid cost.f32|- out.bin [passes]\n"); return 2; }
    int N = atoi(argv[1]), grid = atoi(argv[2]);  // grid 0: the co-resident workgroups (as the library)
    const char* cf = strcmp(argv[3], "-") != 0 ? argv[3] : nullptr;  // "-": uniform cost
    const int passes = argc > 5 ? atoi(argv[5]) : 24;
    std::vector<float> hc((size_t)N * N, 1.f);
    if (cf) { FILE* f = fopen(cf, "rb"); if (!f || fread(hc.data(), 4, hc.size(), f) != hc.size()) { printf("bad cost file\n"); return 2; } fclose(f); }
    unsigned long long* ev; CK(hipMalloc(&ev, 8ull * kCap * grid));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_ev), &ev, sizeof ev));
    Fim2dArgs a{};
    int ntx = (N + 63) / 64, tiles = ntx * ntx;
    // EIK_TRACE_F64=1: the fp64 kernel (the bench headline) on the same (float32-exact) costs
    const bool f64 = getenv("EIK_TRACE_F64") && atoi(getenv("EIK_TRACE_F64")) == 1;
    const size_t esz = f64 ? 8 : 4;
    void *cost, *T; CK(hipMalloc(&cost, esz * N * N)); CK(hipMalloc(&T, esz * N * N));
    if (f64) {
        std::vector<double> hd(hc.begin(), hc.end());
        CK(hipMemcpy(cost, hd.data(), 8ull * N * N, hipMemcpyHostToDevice));
    } else {
        CK(hipMemcpy(cost, hc.data(), 4ull * N * N, hipMemcpyHostToDevice));
    }
    a.cost = cost; a.T = T; a.H = N; a.W = N; a.ntx = ntx; a.nty = ntx; a.tiles_per_map = tiles;
    CK(hipMalloc(&a.lists, 12ull * tiles)); CK(hipMalloc(&a.counts, 256)); CK(hipMalloc(&a.mark, 4ull * tiles));
    a.capacity = tiles; a.max_rounds = 1; a.keep = 1.f; CK(hipMalloc(&a.key, 4ull * tiles)); a.minkey = (unsigned*)a.counts + 16;
    a.delta = __builtin_inff(); CK(hipMalloc(&a.visits, 256));  // (the init kernel clears 22 words)
    char* q; CK(hipMalloc(&q, 256)); a.qhead = (unsigned long long*)q; a.qtail = (unsigned long long*)(q + 64);
    a.qactive = (int*)(q + 128); a.qerror = (unsigned*)(q + 192); a.mode = kModePersistent;
    unsigned qn = 4096; while (qn < 8u * tiles) qn <<= 1;
    a.qmask = qn - 1; CK(hipMalloc(&a.qslot, 4ull * qn)); CK(hipMalloc(&a.qstate, 4ull * tiles));
    a.qtimeout = 1000000000ull; a.qbudget = 1ull << 40; a.max_passes = passes;
    a.ls = 1; a.z0 = 0; a.lzs = 1;
    if (grid == 0) {
        int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
        grid = fim2d_persist_resident(f64, cus, false);
        CK(hipFree(ev)); CK(hipMalloc(&ev, 8ull * kCap * grid));
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_ev), &ev, sizeof ev));
        printf("grid: %d co-resident workgroups\n", grid);
    }
    // the W / E edge-column copies (fim2d.hip kEcol: on in fp64) and, with EIK_TRACE_PRIO=1, the
    // priority bands as eikonal_api.cpp sets them up (width multiplier 1)
    CK(hipMalloc(&a.ecol, esz * 2 * 64ull * tiles));
    const bool prio = getenv("EIK_TRACE_PRIO") && atoi(getenv("EIK_TRACE_PRIO")) == 1;
    // (rings of >= 2 x the tiles, then the per-tile band-membership words, as setup_bands lays them
    // out; width EIK_TRACE_PRIO_W, default 0.25 = the library's default at 4096^2; dispatch batch 16)
    size_t bbytes = 0;
    if (prio) {
        unsigned long long bc = 1024; while (bc < 2ull * tiles) bc <<= 1;
        const size_t ring = 4ull * kBands * bc, moff = (ring + 255) & ~(size_t)255;
        bbytes = moff + 8ull * tiles;
        CK(hipMalloc(&a.bslot, bbytes)); CK(hipMemset(a.bslot, 0, bbytes));
        a.bmem = (unsigned long long*)((char*)a.bslot + moff);
        CK(hipMalloc(&a.bctl, 128 * kBands + 128)); a.bmask = (unsigned)(bc - 1);
        float* pd = (float*)((char*)a.bctl + 128 * kBands);
        const float w = getenv("EIK_TRACE_PRIO_W") ? (float)atof(getenv("EIK_TRACE_PRIO_W")) : 0.25f;
        CK(fim2d_prio_delta(cost, f64, (int64_t)N * N, w, pd, 0));
        a.pdelta = pd;
        a.disp = 16;
    }
    a.fresh_first = getenv("EIK_FRESH_FIRST") && atoi(getenv("EIK_FRESH_FIRST")) == 1;
    a.sched = getenv("EIK_SCHED") ? atoi(getenv("EIK_SCHED")) : 1;  // library default
    int64_t* goals; CK(hipMalloc(&goals, 16)); int64_t hg[2] = {N / 2, N / 2}; CK(hipMemcpy(goals, hg, 16, hipMemcpyHostToDevice));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    float ms = 0;
    for (int rep = 0; rep < 4; ++rep) {
        CK(hipMemset(a.visits, 0, 256)); CK(hipMemset(ev, 0, 8ull * kCap * grid));
        if (a.bctl) CK(hipMemset(a.bctl, 0, 128 * kBands));
        if (a.bslot) CK(hipMemset(a.bslot, 0, bbytes));
        CK(fim2d_init(a, f64, 1, goals, nullptr, 0));
        CK(hipEventRecord(e0, 0));
        CK(fim2d_persist(a, f64, grid, 0));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
    }
    unsigned hq[64]; CK(hipMemcpy(hq, q, 256, hipMemcpyDeviceToHost));
    unsigned long long vv[2]; CK(hipMemcpy(vv, a.visits, 16, hipMemcpyDeviceToHost));
    printf("%s%s N=%d grid=%d passes=%d: kernel %.3f ms, visits %llu (+%llu in place), err %u\n", f64 ? "f64" : "f32", a.bctl ? " prio" : "", N, grid, passes, ms, vv[0], vv[1], hq[48]);
    std::vector<unsigned long long> he(1ull * kCap * grid);
    CK(hipMemcpy(he.data(), ev, 8ull * kCap * grid, hipMemcpyDeviceToHost));
    FILE* o = fopen(argv[4], "wb");
    const int hdr[4] = {N, grid, (int)kCap, ntx};
    fwrite(hdr, 4, 4, o);
    fwrite(he.data(), 8, he.size(), o);
    fclose(o);
    return 0;
}
