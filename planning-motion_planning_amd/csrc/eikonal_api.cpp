// eikonal_api.cpp -- C ABI (include/eikonal.h) over the HIP kernels: contexts, device buffers,
// the outer FIM iteration driver and the synchronous host-buffer drop-ins.
//
// Every entry point fails loudly (status + eik_last_error) -- there is no CPU fallback: a
// missing device is EIK_ERR_NODEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/eikonal.h"
#include "eik_common.hpp"
#include "eik_kernels.hpp"

using namespace eik;

int rover_assemble(const double* pathS, int64_t nS, const double* pathG, int64_t nG, const double* Z, int64_t H,
                   int64_t W, const eik_rover_query* q, double* path_xyz, double* heading, int64_t cap, int64_t* n_out,
                   double zmin_known);  // rover.cpp

namespace {

thread_local std::string g_create_err;

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t n) {
        if (n <= bytes) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        hipError_t e = hipMalloc(&p, n);
        if (e == hipSuccess) bytes = n;
        return e;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

// Host memcpy split over a few worker threads and the caller (the pinned-staging copies below).
// ONE pool per process, shared by every context (8 DD ranks sharing a node each started
// their own threads), created on the first large copy; concurrent callers take turns.
class CopyPool {
  public:
    static CopyPool* shared() {
        static CopyPool* p = new CopyPool((int)std::max(1u, std::min(3u, std::thread::hardware_concurrency() / 2)));
        return p;  // (never destroyed: workers outlive the contexts, the process ends them)
    }
    explicit CopyPool(int workers) {
        for (int i = 0; i < workers; ++i) th_.emplace_back([this] { loop(); });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            quit_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void copy(void* dst, const void* src, size_t len) {
        std::lock_guard<std::mutex> turn(caller_);  // one copy at a time (contexts of other threads wait)
        const int parts = (int)th_.size() + 1;
        {
            std::lock_guard<std::mutex> g(m_);
            dst_ = static_cast<char*>(dst);
            src_ = static_cast<const char*>(src);
            len_ = len;
            parts_ = parts;
            next_ = 1;  // part 0 is the caller's
            left_ = parts - 1;
            ++gen_;
        }
        cv_.notify_all();
        part(0, parts);
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [&] { return left_ == 0; });
    }

  private:
    std::mutex caller_;
    void part(int k, int parts) {
        const size_t a = len_ * k / parts, e = len_ * (k + 1) / parts;
        std::memcpy(dst_ + a, src_ + a, e - a);
    }
    void loop() {
        for (;;) {
            int k, parts;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return quit_ || next_ < parts_; });
                if (quit_) return;
                k = next_++;
                parts = parts_;
            }
            part(k, parts);
            {
                std::lock_guard<std::mutex> g(m_);
                if (--left_ == 0) done_.notify_one();
            }
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    char* dst_ = nullptr;
    const char* src_ = nullptr;
    size_t len_ = 0;
    int parts_ = 0, next_ = 0, left_ = 0;
    unsigned long long gen_ = 0;
    bool quit_ = false;
};

}  // namespace

constexpr double kFrontsMargin = 1.25;  // capped bidirectional fronts (solve_fronts)

struct eik_ctx {
    int device = 0;
    int cu_count = 256;
    hipStream_t stream = nullptr;
    std::string err;
    int max_rounds = 1;
    double tol = 0.0;
    double delta = 0.0;  // 0: unordered FIM
    int sync_every = 8;
    int mode = kModePersistent;  // EIK_OPT_MODE
    double qtimeout_s = 30.0;    // EIK_OPT_QTIMEOUT: persistent-mode spin limit
    unsigned long long max_visits = 0;  // EIK_OPT_MAX_VISITS (0: per-solver default)
    int passes = 0;              // EIK_OPT_PASSES: in-place passes per persistent visit (0: adaptive)
    bool fresh_first = false;    // EIK_OPT_FRESH_FIRST: fresh tiles jump a backlogged FIFO
    int sched = 1;               // EIK_OPT_SCHED: in-place scheduling of persistent visits
    int live_pack = 0;           // EIK_OPT_LIVE_PACK: the halo agent packs only idle tiles' edges
    // EIK_OPT_PRIO: the priority bands' width in units of 64 x the cost's geometric mean (0: the
    // plain FIFO; < 0, the default: default_prio() in fp64, on the layered solver and on one fp32 2D map of
    // >= kWideTiles tiles, else 0 in fp32 2D;
    // round 5's first default was 1 in fp64).  fp64 at 1: C2 2.44-2.50 -> 2.37 ms, C4 at
    // one GPU 10.5 -> 13.8 Gcells/s; 0.5 / 2 lose on C4 (6.9 / 12.9; profiles/r05i_prio_ab.log).  fp32
    // solves are twice as fast per pass and the one-dispatcher bands held them back: C2 fp32 1.6 ->
    // 1.9 ms, C4 fp32 18.7 -> 10.8 Gcells/s (profiles/r05j_bench.json) -- until the 128-entry dispatches of
    // round 6 (C4 fp32 with bands 18.4 -> 19.5).  Batches of > 2 maps: FIFO.
    // The layered solver's bands (both dtypes, default_prio()): C5 fp64 1.92 -> 3.65, fp32 4.73 -> 6.2
    // Gcells/s (profiles/r05ac_layered_prio_ab.log, r05ad_prio_width_ab.log).
    double prio = -1.0;
    int prio_ring = 0;           // EIK_OPT_PRIO_RING: slots per priority band (0: pow2 >= 2 x the tiles)
    int prio_dispatch = 0;       // EIK_OPT_PRIO_DISPATCH: band entries per dispatch (0: 128 on maps of >= kWideTiles, else 16)
    // EIK_OPT_LAYER_PLANAR (default 1): the layered solver works on layer-planar copies.  C5 kernel
    // traffic per launch 9.06 -> 3.92 GB (fp32), 20.3 -> 8.6 GB (fp64), the time within noise
    // (the layered sweep is VALU-bound; profiles/r05c_pmc_traffic_c5*.json, r05h_prio_planar_ab.log)
    int layer_planar = 1;
    DevBuf lp_cost, lp_T;        // those copies (solve_layered)
    int path_loop = 4;           // EIK_OPT_PATH_LOOP: 2D walker loop form (4: lane pairs, round 5,
                                 // 0.405 -> 0.30 us/step on the bench path, profiles/r05k_walker_ab.log)
    int timing = 0;
    int grid = 0;
    eik_stats last{};
    eik_fim2d* cached = nullptr;  // solver reused by the host-buffer entry points
    eik_fim2d* cached_l = nullptr;  // queue state of the layered 3D solver (fim2dl.hip), fp32 tiles
    eik_fim2d* cached_l64 = nullptr;  // the same for the fp64 layered solver's 40-row tiles
    eik_fim2d* cached_fill = nullptr;  // reachability solver of the cost builder's hole filling
    eik_fim2d* cached_fronts = nullptr;  // coarse B = 2 solver of the capped bidirectional fronts
    double fronts_cap = 1.25;          // EIK_OPT_FRONTS_CAP: cap margin (0: full fronts)
    DevBuf fronts;                     // capped fronts: coarse cost (2 maps) | coarse T (2 maps) | FrontsCheck
    int64_t fronts_info[10] = {};      // eik_fronts_info: capped, fallback, kept G / S, members G / S,
                                       // band cells G / S, band relaxation sweeps G / S
    bool exact_band = false;           // EIK_OPT_EXACT_BAND: replay the reference's band (bidir_exact.hip)
    DevBuf exact;                      // its scratch: events, ranks, sort keys
    unsigned long long exact_info[5] = {};  // eik_exact_info: passes, sweeps G / S, tie launches, microseconds
    DevBuf cm_u8, cm_i32, cm_f32, cm_f64;  // cost-builder scratch
    DevBuf arm;                            // end-effector volume scratch (arm.hip)
    int resident_l[2][5] = {};  // co-resident workgroups of fim2dl_persist_kernel<R, nl> (f32, f64)
    DevBuf cost, T, T2, goals, work, misc;
    DevBuf l3, c3, m3, v3;             // 3D solver scratch (lists, counts, marks, visits)
    int max_passes3 = 24;
    int* h3 = nullptr;                 // 3D solver: pinned count + visits words (made once)
    DevBuf q3ctl, q3slot, q3state, q3vis;  // 3D persistent driver: tile FIFO (fim_engine.hpp)
    unsigned* h_q3 = nullptr;          // pinned copy of q3ctl + the two visit counters
    int resident3[2] = {0, 0};         // co-resident workgroups of fim3d_persist_kernel (f32, f64)
    hipStream_t stream2 = nullptr;     // second stream: the rover path's two walks run side by side
    // pinned staging of large host <-> device copies (host_to_dev / dev_to_host)
    char* stage[2] = {nullptr, nullptr};
    hipEvent_t stage_ev[2] = {nullptr, nullptr};
    CopyPool* pool = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    hipEvent_t e3[2] = {nullptr, nullptr};
};

struct eik_fim2d {
    eik_ctx* ctx = nullptr;
    int64_t B = 0, H = 0, W = 0;
    bool f64 = false;
    Fim2dArgs a{};
    hipStream_t stream = nullptr;
    DevBuf lists, counts, mark, edge, goals, key;
    DevBuf ecol;                         // every tile's two edge columns (Fim2dArgs::ecol)
    DevBuf qctl, qslot, qstate;          // persistent-mode FIFO
    DevBuf bslot, bctl;                  // priority bands (EIK_OPT_PRIO)
    int* h_counts = nullptr;             // pinned
    unsigned* h_q = nullptr;             // pinned copy of qctl
    unsigned long long* h_visits = nullptr;
    int64_t* h_goals = nullptr;          // pinned: the goals' upload does not stall the host
    int64_t iterations = 0, host_syncs = 0, max_iters = 0;
    hipEvent_t ev_start = nullptr, ev_stop = nullptr;
    std::vector<hipEvent_t> ev_pool;     // per-launch timing pairs (timing option)
    size_t ev_used = 0;
    double sweep_ms = 0.0, solve_ms = 0.0;
    bool started = false;
    bool defer_sync = false;             // eik_fim2d_solve: the launch's read-back syncs with the finish
    bool need_rewind = false;            // a launch without its queue rewind ran since the last init
    bool band_overflow = false;          // the last launch stopped on a full priority band (qerror bit 4)
    bool no_bands = false;               // ... so this solver's next starts use the FIFO
    int persist_grid = 0;                // co-resident workgroups of the persistent kernel
    // live domain decomposition: hold word on the device, mailbox of the halo agent on the host
    DevBuf hold;
    LiveBox* box = nullptr;              // pinned, coherent
    bool live_on = false;
    // a layered volume's block (eik_fim3dl_create: the layered solver, fim2dl.hip): nl > 0
    int lnl = 0, lz0 = 0;
    int64_t lL = 1;
};

static int set_err(eik_ctx* c, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (c)
        c->err = buf;
    else
        g_create_err = buf;
    return code;
}

#define HIPCHK(ctx, expr)                                                                          \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess)                                                                      \
            return set_err((ctx), e_ == hipErrorOutOfMemory ? EIK_ERR_NOMEM : EIK_ERR_HIP, "%s: %s (%s:%d)", \
                           #expr, hipGetErrorString(e_), __FILE__, __LINE__);                      \
    } while (0)

static int bytes_per_visit(bool f64) { return (f64 ? 8 : 4) * (3 * kTile * kTile + 4 * kTile); }
// in-place pass of a busy tile (persistent mode): T write-back + halo ring re-read
static int bytes_per_pass(bool f64) { return (f64 ? 8 : 4) * (kTile * kTile + 4 * kTile); }

// Large host <-> device copies through a pinned ring of two 8 MiB chunks, host memcpy by a few
// threads overlapped with the DMA of the other chunk.  A pageable hipMemcpyAsync of a FRESH host
// buffer (every numpy array the drop-in receives or returns) ran at ~8 GB/s: 16 ms per 128 MiB,
// 3 ms only once the runtime had seen the buffer; staged: ~4 ms either way (tools/h2d_probe.cpp).
// Staged (pageable) buffers: host_to_dev returns once the source has been read (the DMA of the last
// chunk may still run on st); dev_to_host returns with the data in dst (it waits for st's earlier
// work).  A buffer wholly inside a pinned block (eik_host_alloc) goes as ONE hipMemcpyAsync on st
// and both return at once: the source must stay unchanged, and dst is valid, only after st is
// synchronised -- every caller synchronises st before it returns to its own caller.
constexpr size_t kStageChunk = 8ull << 20;
// pinned host blocks handed out by eik_host_alloc: a copy wholly inside one goes as one DMA
static std::mutex g_pin_mu;
static std::vector<std::pair<uintptr_t, size_t>> g_pinned;
static bool is_pinned(const void* p, size_t bytes) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    std::lock_guard<std::mutex> lk(g_pin_mu);
    for (const auto& b : g_pinned)
        if (a >= b.first && a + bytes <= b.first + b.second) return true;
    return false;
}
static hipError_t stage_init(eik_ctx* c) {
    for (int b = 0; b < 2; ++b) {
        if (!c->stage[b]) {
            hipError_t e = hipHostMalloc((void**)&c->stage[b], kStageChunk);
            if (e != hipSuccess) return e;
        }
        if (!c->stage_ev[b]) {
            hipError_t e = hipEventCreateWithFlags(&c->stage_ev[b], hipEventDisableTiming);
            if (e != hipSuccess) return e;
        }
    }
    if (!c->pool) c->pool = CopyPool::shared();
    return hipSuccess;
}
static hipError_t host_to_dev(eik_ctx* c, void* dst, const void* src, size_t bytes, hipStream_t st) {
    if (bytes < 2 * kStageChunk || is_pinned(src, bytes)) return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st);
    hipError_t e = stage_init(c);
    if (e != hipSuccess) return e;
    int k = 0;
    for (size_t off = 0; off < bytes; off += kStageChunk, ++k) {
        const int b = k & 1;
        const size_t len = std::min(kStageChunk, bytes - off);
        if ((e = hipEventSynchronize(c->stage_ev[b])) != hipSuccess) return e;  // its last DMA is done
        c->pool->copy(c->stage[b], static_cast<const char*>(src) + off, len);
        if ((e = hipMemcpyAsync(static_cast<char*>(dst) + off, c->stage[b], len, hipMemcpyHostToDevice, st)) != hipSuccess)
            return e;
        if ((e = hipEventRecord(c->stage_ev[b], st)) != hipSuccess) return e;
    }
    return hipSuccess;
}
static hipError_t dev_to_host(eik_ctx* c, void* dst, const void* src, size_t bytes, hipStream_t st) {
    if (bytes < 2 * kStageChunk || is_pinned(dst, bytes)) return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st);
    hipError_t e = stage_init(c);
    if (e != hipSuccess) return e;
    const size_t nch = (bytes + kStageChunk - 1) / kStageChunk;
    // a host_to_dev on another stream may still be reading the staging buffers
    for (int b = 0; b < 2; ++b)
        if ((e = hipStreamWaitEvent(st, c->stage_ev[b], 0)) != hipSuccess) return e;
    auto issue = [&](size_t k) -> hipError_t {
        const int b = (int)(k & 1);
        const size_t off = k * kStageChunk, len = std::min(kStageChunk, bytes - off);
        hipError_t r = hipMemcpyAsync(c->stage[b], static_cast<const char*>(src) + off, len, hipMemcpyDeviceToHost, st);
        return r == hipSuccess ? hipEventRecord(c->stage_ev[b], st) : r;
    };
    if ((e = issue(0)) != hipSuccess) return e;
    for (size_t k = 0; k < nch; ++k) {
        // the next chunk's DMA lands in the buffer chunk k - 1 used, already copied out
        if (k + 1 < nch && (e = issue(k + 1)) != hipSuccess) return e;
        const int b = (int)(k & 1);
        if ((e = hipEventSynchronize(c->stage_ev[b])) != hipSuccess) return e;
        const size_t off = k * kStageChunk;
        c->pool->copy(static_cast<char*>(dst) + off, c->stage[b], std::min(kStageChunk, bytes - off));
    }
    return hipSuccess;
}

extern "C" {

const char* eik_version(void) { return "eikonal-mi355x 0.1 (gfx950 block-FIM, 64x64 tiles)"; }

int eik_create(int device, eik_ctx** out) {
    if (!out) return set_err(nullptr, EIK_ERR_ARG, "out is NULL");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return set_err(nullptr, EIK_ERR_NODEVICE, "no HIP device visible (the Eikonal solver has no CPU path)");
    if (device < 0 || device >= n) return set_err(nullptr, EIK_ERR_ARG, "device %d out of range [0,%d)", device, n);
    if (hipSetDevice(device) != hipSuccess) return set_err(nullptr, EIK_ERR_HIP, "hipSetDevice(%d) failed", device);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess)
        return set_err(nullptr, EIK_ERR_HIP, "hipGetDeviceProperties failed");
    auto* c = new eik_ctx();
    c->device = device;
    c->cu_count = prop.multiProcessorCount;
    c->grid = 4 * c->cu_count;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return set_err(nullptr, EIK_ERR_HIP, "hipStreamCreate failed");
    }
    *out = c;
    return EIK_OK;
}

void eik_destroy(eik_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->cached) eik_fim2d_destroy(c->cached);
    if (c->cached_l) eik_fim2d_destroy(c->cached_l);
    if (c->cached_l64) eik_fim2d_destroy(c->cached_l64);
    if (c->cached_fill) eik_fim2d_destroy(c->cached_fill);
    if (c->cached_fronts) eik_fim2d_destroy(c->cached_fronts);
    if (c->h3) (void)hipHostFree(c->h3);
    if (c->h_q3) (void)hipHostFree(c->h_q3);
    for (hipEvent_t e : c->e3)
        if (e) (void)hipEventDestroy(e);
    if (c->stream2) (void)hipStreamDestroy(c->stream2);
    for (int b = 0; b < 2; ++b) {
        if (c->stage[b]) (void)hipHostFree(c->stage[b]);
        if (c->stage_ev[b]) (void)hipEventDestroy(c->stage_ev[b]);
    }
    c->pool = nullptr;  // (the process-wide pool stays)
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* eik_last_error(const eik_ctx* c) { return c ? c->err.c_str() : g_create_err.c_str(); }

int eik_set_option(eik_ctx* c, int opt, double v) {
    if (!c) return EIK_ERR_ARG;
    switch (opt) {
        case EIK_OPT_MAX_ROUNDS: c->max_rounds = std::max(1, (int)v); break;
        case EIK_OPT_SYNC_EVERY: c->sync_every = std::max(1, (int)v); break;
        case EIK_OPT_TIMING: c->timing = v != 0; break;
        case EIK_OPT_GRID: c->grid = v > 0 ? (int)v : 4 * c->cu_count; break;
        case EIK_OPT_TOL: c->tol = v > 0 ? v : 0.0; break;
        case EIK_OPT_DELTA: c->delta = v > 0 ? v : 0.0; break;
        case EIK_OPT_MODE:
            if (v != EIK_MODE_LIST && v != EIK_MODE_PERSISTENT) return set_err(c, EIK_ERR_ARG, "bad mode %g", v);
            c->mode = (int)v;
            break;
        case EIK_OPT_QTIMEOUT: c->qtimeout_s = v > 0 ? v : 30.0; break;
        case EIK_OPT_MAX_VISITS: c->max_visits = v > 0 ? (unsigned long long)v : 0ull; break;
        case EIK_OPT_PASSES: c->passes = std::max(0, std::min(64, (int)v)); break;
        case EIK_OPT_FRESH_FIRST: c->fresh_first = v != 0; break;
        case EIK_OPT_SCHED: c->sched = std::max(0, std::min(3, (int)v)); break;
        case EIK_OPT_LIVE_PACK: c->live_pack = v != 0; break;
        case EIK_OPT_PRIO: c->prio = v; break;
        case EIK_OPT_PRIO_RING: c->prio_ring = v < 0 ? 0 : (int)std::min(v, 1073741824.0); break;
        case EIK_OPT_PRIO_DISPATCH: c->prio_dispatch = v < 0 ? 0 : (int)std::min(v, 128.0); break;
        case EIK_OPT_LAYER_PLANAR: c->layer_planar = v != 0; break;
        case EIK_OPT_PATH_LOOP: c->path_loop = std::max(0, std::min(4, (int)v)); break;
        case EIK_OPT_EXACT_BAND: c->exact_band = v != 0; break;
        case EIK_OPT_FRONTS_CAP: c->fronts_cap = v <= 0 ? 0.0 : v == 1 ? kFrontsMargin : std::max(1.0, v); break;
        default: return set_err(c, EIK_ERR_ARG, "unknown option %d", opt);
    }
    return EIK_OK;
}

int eik_get_stats(const eik_ctx* c, eik_stats* out) {
    if (!c || !out) return EIK_ERR_ARG;
    *out = c->last;
    return EIK_OK;
}

// ------------------------------------------------------------------------------ fim2d
// th: tile rows (64; the fp64 layered solver's tiles have fim2dl_rows(true) = 40)
// The default priority-band width (EIK_OPT_PRIO < 0; fp64 2D solves and the layered solver): 0.25 on
// a 4096^2 raster, growing with the raster's side -- the front's T range grows with it, and bands too
// narrow for it leave the queue to the open-ended last band.  Band-width A/B, 0.25 / 0.5 / 1:
//   C2 4096^2 fp64 2.14-2.16 / 2.15-2.19 / 2.17-2.20 ms; C4 16384^2 fp64 3.9-4.0 / 9.0-9.1 / 16.3-16.7
//   Gcells/s (profiles/r05ad_prio_width_ab.log, r05ae_c4_width_ab.log);
//   layered (C5's volume, tools/layered_scale_probe.py) fp64 4096^2 3.79 / 3.75 / 3.61, 8192^2 4.16 /
//   4.33 / 4.19, 16384^2 1.65 / 3.95 / 4.30; fp32 6.80 / 6.83 / 6.79, 7.78 / 8.02 / 7.86, 4.84 / 8.13 /
//   8.50 Gcells/s (the FIFO: fp64 2.89, 1.77, 1.29; fp32 6.63, 4.62, 3.11; profiles/r05af_*, r05ah_*).
// Below a side of min_side the FIFO is the default: the bands' dispatch latency outweighs the order on
// small rasters.  fp64 2D FIFO vs bands (0.25), ms: 1024^2 0.48 / 0.57, 2048^2 0.79 / 0.92, 2560^2 1.06 /
// 1.20, 3072^2 1.22 / 1.37, 3584^2 1.43 / 1.58, the C4 DEM at 4096^2 1.79 / 1.85 but C2's raster 2.35 /
// 2.15 (profiles/r05an_prio_size_2d.log, r05ao_prio_crossover.log, r05ap_c2_prio_vs_fifo_ab.log): 2D
// min_side 4096.  Layered (C5's volume) fp64 / fp32 FIFO vs bands, ms: 1024^2 2.34 / 2.55, 1.55 / 1.70;
// 2048^2 4.37 / 4.46, 2.61 / 2.86; 3072^2 8.49 / 7.75, 4.29 / 4.35: layered min_side 3072.
static double default_prio(int64_t H, int64_t W, double min_side) {
    const double side = std::sqrt((double)H * (double)W);
    if (side < min_side) return 0.0;
    return 0.25 * std::max(1.0, side / 4096.0);
}

// Priority bands' buffers for a solve of `tiles` tiles (fim_engine.hpp): kBands rings of a power of
// two >= 2 x the tiles (EIK_OPT_PRIO_RING: any power of two, tests), the per-tile band-membership
// words (at most one entry per (tile, band): a ring of >= tiles slots cannot lap) and the head /
// tail words, all cleared on the stream.  Fills a.bslot / bmask / bmem / bctl.  (The band-tagged
// FIFO entries hold tile + 1 in kBandTagShift bits: bands need tiles < 2^25 - 1.)
static hipError_t setup_bands(eik_ctx* c, DevBuf& bslot, DevBuf& bctl, int64_t tiles, Fim2dArgs& a, hipStream_t st) {
    uint64_t bc = 1024;
    while (bc < 2 * (uint64_t)tiles) bc <<= 1;
    if (c->prio_ring > 0) {  // (tests: a ring below the tile count can lap -> qerror bit 4 -> FIFO re-solve)
        bc = 1;
        while (bc < (uint64_t)c->prio_ring) bc <<= 1;
    }
    const size_t ring_bytes = sizeof(unsigned) * kBands * bc;
    const size_t mem_off = (ring_bytes + 255) & ~(size_t)255;
    const size_t bytes = mem_off + sizeof(unsigned long long) * (size_t)tiles;
    hipError_t e = bslot.ensure(bytes);
    if (e == hipSuccess) e = bctl.ensure(128 * kBands + 128);  // + the band width's word
    if (e == hipSuccess) e = hipMemsetAsync(bslot.p, 0, bytes, st);
    if (e == hipSuccess) e = hipMemsetAsync(bctl.p, 0, 128 * kBands, st);
    if (e != hipSuccess) return e;
    a.bslot = (unsigned*)bslot.p;
    a.bmask = (unsigned)(bc - 1);
    a.bmem = (unsigned long long*)((char*)bslot.p + mem_off);
    a.bctl = (unsigned long long*)bctl.p;
    return hipSuccess;
}

static int fim2d_create_rows(eik_ctx* c, int64_t B, int64_t H, int64_t W, int dtype, int th, eik_fim2d** out) {
    if (!c || !out) return EIK_ERR_ARG;
    *out = nullptr;
    if (B < 1 || H < 1 || W < 1) return set_err(c, EIK_ERR_ARG, "bad shape B=%ld H=%ld W=%ld", (long)B, (long)H, (long)W);
    if (dtype != EIK_F32 && dtype != EIK_F64) return set_err(c, EIK_ERR_ARG, "bad dtype %d", dtype);
    const int64_t ntx = (W + kTile - 1) / kTile, nty = (H + th - 1) / th;
    const int64_t tiles = B * ntx * nty;
    if (tiles >= (1ll << 31) - 8) return set_err(c, EIK_ERR_ARG, "too many tiles");
    HIPCHK(c, hipSetDevice(c->device));
    auto* f = new eik_fim2d();
    f->ctx = c;
    f->B = B;
    f->H = H;
    f->W = W;
    f->f64 = dtype == EIK_F64;
    f->stream = c->stream;
    Fim2dArgs& a = f->a;
    a.H = H;
    a.W = W;
    a.ntx = (int)ntx;
    a.nty = (int)nty;
    a.tiles_per_map = (int)(ntx * nty);
    a.capacity = (int)tiles;
    for (auto& g : a.ghost) g = nullptr;
    a.ls = 1;
    a.z0 = 0;
    a.lzs = 1;
    // FIFO slots: a power of two with ample headroom over the tiles (each tile holds at most one
    // filled slot; the margin keeps a slow poller's slot from being lapped by the tail)
    uint64_t q = 4096;
    while (q < 8 * (uint64_t)tiles) q <<= 1;
    hipError_t e = hipSuccess;
    if ((e = f->lists.ensure(sizeof(int) * 3 * tiles)) != hipSuccess ||
        (e = f->qctl.ensure(kQueueCtlBytes)) != hipSuccess || (e = f->qslot.ensure(sizeof(unsigned) * q)) != hipSuccess ||
        (e = f->qstate.ensure(sizeof(unsigned) * tiles)) != hipSuccess ||
        (e = hipHostMalloc((void**)&f->h_q, kQueueCtlBytes)) != hipSuccess ||
        (e = f->counts.ensure(sizeof(int) * 64)) != hipSuccess || (e = f->mark.ensure(sizeof(unsigned) * tiles)) != hipSuccess ||
        (e = f->key.ensure(sizeof(unsigned) * tiles)) != hipSuccess ||
        (e = f->edge.ensure(sizeof(unsigned) * 4)) != hipSuccess || (e = f->goals.ensure(sizeof(int64_t) * 2 * B)) != hipSuccess ||
        (e = f->ecol.ensure((dtype == EIK_F64 ? 8 : 4) * 2 * kTile * (size_t)tiles)) != hipSuccess ||
        (e = hipHostMalloc((void**)&f->h_counts, sizeof(int) * 64)) != hipSuccess ||
        (e = hipHostMalloc((void**)&f->h_visits, 3 * sizeof(unsigned long long))) != hipSuccess ||
        (e = hipHostMalloc((void**)&f->h_goals, sizeof(int64_t) * 2 * B)) != hipSuccess ||
        (e = hipEventCreate(&f->ev_start)) != hipSuccess || (e = hipEventCreate(&f->ev_stop)) != hipSuccess) {
        eik_fim2d_destroy(f);
        return set_err(c, EIK_ERR_NOMEM, "fim2d allocation: %s", hipGetErrorString(e));
    }
    a.lists = (int*)f->lists.p;
    a.ecol = f->ecol.p;
    a.counts = (int*)f->counts.p;
    a.mark = (unsigned*)f->mark.p;
    a.key = (unsigned*)f->key.p;
    a.minkey = (unsigned*)f->counts.p + 16;
    // the visit counters sit in the queue words' block (own 128-B line): one read-back after a
    // persistent launch brings both
    a.visits = (unsigned long long*)((char*)f->qctl.p + kVisitsOff);
    a.edge_dirty = nullptr;
    a.qhead = (unsigned long long*)f->qctl.p;
    a.qtail = (unsigned long long*)((char*)f->qctl.p + 64);
    a.qactive = (int*)((char*)f->qctl.p + 128);
    a.qerror = (unsigned*)((char*)f->qctl.p + 192);
    a.qslot = (unsigned*)f->qslot.p;
    a.qmask = (unsigned)(q - 1);
    a.qstate = (unsigned*)f->qstate.p;
    // safety cap: a monotone solve visits each tile a bounded number of times; negative costs
    // (invalid input on a device buffer) would otherwise iterate forever.
    f->max_iters = 64 * (ntx + nty) + 8 * tiles / B + 4096;
    *out = f;
    return EIK_OK;
}

int eik_fim2d_create(eik_ctx* c, int64_t B, int64_t H, int64_t W, int dtype, eik_fim2d** out) {
    return fim2d_create_rows(c, B, H, W, dtype, kTile, out);
}

void eik_fim2d_destroy(eik_fim2d* f) {
    if (!f) return;
    if (f->h_counts) (void)hipHostFree(f->h_counts);
    if (f->h_visits) (void)hipHostFree(f->h_visits);
    if (f->h_goals) (void)hipHostFree(f->h_goals);
    if (f->h_q) (void)hipHostFree(f->h_q);
    if (f->ev_start) (void)hipEventDestroy(f->ev_start);
    if (f->ev_stop) (void)hipEventDestroy(f->ev_stop);
    if (f->box) (void)hipHostFree(f->box);
    for (auto ev : f->ev_pool) (void)hipEventDestroy(ev);
    delete f;
}

// the queue counters of the last persistent launch (EIK_QDEBUG builds; zeros otherwise)
int eik_fim2d_qcount(const eik_fim2d* f, uint64_t out[8]) {
    if (!f || !out) return EIK_ERR_ARG;
    memcpy(out, (const char*)f->h_q + kVisitsOff + 24, 8 * sizeof(uint64_t));
    return EIK_OK;
}

int eik_fim2d_set_ghosts(eik_fim2d* f, void* n, void* s, void* w, void* e) {
    if (!f) return EIK_ERR_ARG;
    if (f->B != 1) return set_err(f->ctx, EIK_ERR_ARG, "ghost strips need B == 1");
    f->a.ghost[0] = n;
    f->a.ghost[1] = s;
    f->a.ghost[2] = w;
    f->a.ghost[3] = e;
    f->a.edge_dirty = (n || s || w || e) ? (unsigned*)f->edge.p : nullptr;
    return EIK_OK;
}

int eik_fim2d_start(eik_fim2d* f, const void* d_cost, void* d_T, const int64_t* goals, void* stream) {
    if (!f || !d_cost || !d_T || !goals) return EIK_ERR_ARG;
    eik_ctx* c = f->ctx;
    HIPCHK(c, hipSetDevice(c->device));
    f->stream = (hipStream_t)stream;  // as given: NULL is the default (null) stream
    f->a.cost = d_cost;
    f->a.T = d_T;
    f->a.iter = 0;
    f->a.max_rounds = c->max_rounds;
    f->a.keep = (float)(1.0 - c->tol);
    f->a.delta = c->delta > 0 ? (float)c->delta : __builtin_inff();
    // persistent mode needs 32-bit byte offsets per map (buffer resources) and no ordering window
    const bool fits = f->H * f->W * (f->f64 ? 8 : 4) < (int64_t)UINT32_MAX;
    f->a.mode = (c->mode == kModePersistent && fits && !(c->delta > 0)) ? kModePersistent : kModeList;
    f->a.qtimeout = (unsigned long long)(c->qtimeout_s * 1e8);  // s_memrealtime: 100 MHz
    // in-place passes: a single map's solve is front-latency-bound (long in-place refinement of
    // the front tiles pays), a batch is throughput-bound (hand the workgroup to tiles with fresher
    // halos early): C2 2.07-2.09 ms at 8-16 vs 2.23 at 2; C3 6.86 ms at 2 vs 8.0 at 8.  Single map
    // 24 (profiles/r01g_passes_8_16_24.log): C2 2.03-2.04 ms vs 2.05-2.08 at 16 (within noise),
    // C4 at one GPU 16.4-16.6 vs 16.3-16.4 at 16 (within noise); 8 is clearly slower on both.
    // A single map large enough for the 4-waves-per-SIMD kernel (>= kWideTiles tiles, 16384^2) is
    // throughput-bound: 16 passes, 17.1-17.3 -> 18.3-18.9 Gcells/s (profiles/r02w_passes_wide.log).
    // A few large maps (biComputeTmap's two fronts: B = 2 of 4096^2) are latency-bound like one map.
    const bool batch = f->B > 4 || (f->B > 1 && f->a.tiles_per_map < 1024);
    // One map (round 3, profiles/r03v_passes_f64_c2_ab.log): 40 -- C2 fp64 2.461-2.468 ms at 24,
    // 2.394-2.420 at 40; fp32 1.733-1.748 at 24, 1.723-1.726 at 40.
    f->a.max_passes = c->passes > 0 ? c->passes
                      : batch                                             ? 2
                      : (!f->f64 && f->a.tiles_per_map >= kWideTiles)     ? 16
                                                                          : 40;
    f->a.qbudget = c->max_visits ? c->max_visits : 1024ull * (unsigned long long)(f->B * f->a.tiles_per_map) + (1ull << 20);
    f->iterations = 0;
    f->host_syncs = 0;
    f->sweep_ms = 0.0;
    f->solve_ms = 0.0;
    f->ev_used = 0;
    HIPCHK(c, hipEventRecord(f->ev_start, f->stream));
    // (the previous solve on this solver synchronised before returning: h_goals is free)
    memcpy(f->h_goals, goals, sizeof(int64_t) * 2 * f->B);
    HIPCHK(c, hipMemcpyAsync(f->goals.p, f->h_goals, sizeof(int64_t) * 2 * f->B, hipMemcpyHostToDevice, f->stream));
    // priority bands (persistent mode): kBands rings of twice the tiles each (a pending tile has at
    // most one live entry per band it was pushed to plus stale ones, dropped when taken), cleared
    // with the queue before the seed kernel pushes the goal's tile
    f->a.bctl = nullptr;
    // (one map or a few: a batch of independent maps keeps the FIFO -- their keys do not compare)
    // (a domain-decomposition block -- ghost strips bound -- keeps the bands at any size, at width >= 1:
    // they order the ghosts' arrivals, whose T spans the whole raster's range, not the block's.  The
    // 16384^2 4 x 2 rehearsal: FIFO 3.7x the single domain's visits, width 1 0.96x (22 ms), the
    // block-sized 0.35 2.96x (61 ms), profiles/r05d_c4_rehearsal_n8_*.json, r05h_c4_rehearsal_n8.log)
    const bool dd_block = f->a.ghost[0] || f->a.ghost[1] || f->a.ghost[2] || f->a.ghost[3];
    // fp32 keeps the FIFO below kWideTiles tiles (its passes are twice as fast and the one dispatcher held
    // it back: C2 fp32 1.6 -> 1.9 ms with bands, round 5); one map of >= kWideTiles tiles takes the bands
    // since the 128-entry dispatches (round 6: C4 at one GPU fp32 18.4 -> 19.5 Gcells/s mean of 5 same-box
    // alternations, 145 k -> 108 k visits, profiles/r06s7/r06s7_c4f32_prio_ab{,2}.log)
    const bool f32_wide = !f->f64 && f->B == 1 && f->a.tiles_per_map >= kWideTiles && !dd_block;
    const double prio = c->prio >= 0 ? c->prio
                        : f32_wide ? default_prio(f->H, f->W, 4096.0)
                        : !f->f64  ? 0.0
                        : dd_block ? std::max(1.0, default_prio(f->H, f->W, 0.0))
                                   : default_prio(f->H, f->W, 4096.0);
    if (prio > 0 && f->a.mode == kModePersistent && f->B <= 2 && !f->no_bands && f->a.capacity < (1 << kBandTagShift) - 1) {
        // (a decomposition block's launch lives through many halo rounds: the band-membership bits
        // bound every band to one entry per tile however many pending episodes its tiles go through;
        // round 5 gave blocks 16 x the tiles per ring instead, which only moved the threshold)
        HIPCHK(c, setup_bands(c, f->bslot, f->bctl, f->a.capacity, f->a, f->stream));
        float* pd = (float*)((char*)f->bctl.p + 128 * kBands);
        HIPCHK(c, fim2d_prio_delta(d_cost, f->f64, f->H * f->W, (float)prio, pd, f->stream));
        f->a.pdelta = pd;
        f->a.disp = c->prio_dispatch > 0 ? (unsigned)c->prio_dispatch
                                         : f->a.tiles_per_map >= kWideTiles ? 128u : 16u;  // (fim_engine.hpp band_dispatch)
    }
    HIPCHK(c, fim2d_init(f->a, f->f64, (int)f->B, (const int64_t*)f->goals.p, (unsigned*)f->edge.p, f->stream));
    f->started = true;
    f->need_rewind = false;  // the init cleared the queue words
    return EIK_OK;
}

// the persistent launch's queue words (h_q, read back after it): errors and the active count
static int persist_result(eik_fim2d* f, int64_t* active) {
    eik_ctx* c = f->ctx;
    const unsigned err = f->h_q[192 / 4];
    f->band_overflow = (err & 4u) != 0u;
    if (f->band_overflow)
        return set_err(c, EIK_ERR_HIP, "persistent solver: a priority band's ring is full (EIK_OPT_PRIO=0 "
                                       "uses the FIFO; eik_fim2d_solve falls back by itself)");
    if (err & 1u)
        return set_err(c, EIK_ERR_HIP, "persistent solver: a queue wait exceeded %.1f s (EIK_OPT_QTIMEOUT)",
                       c->qtimeout_s);
    if (err & 2u)
        return set_err(c, EIK_ERR_NOCONVERGE, "no convergence within %llu tile visits (negative costs?)",
                       (unsigned long long)f->a.qbudget);
    if (active) *active = f->h_q[128 / 4];
    return EIK_OK;
}

static int drain_timing(eik_fim2d* f) {
    // events were recorded in (start, stop) pairs; the stream has been synchronised
    for (size_t i = 0; i + 1 < f->ev_used; i += 2) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, f->ev_pool[i], f->ev_pool[i + 1]) == hipSuccess) f->sweep_ms += ms;
    }
    f->ev_used = 0;
    return EIK_OK;
}

// A persistent launch's idle waiters take tickets past the tail; eik_fim2d_solve skips the rewind
// kernel after its launch, so before anything appends to the same queue again (merge_ghost, the
// next iterate) the ticket counter is restarted at the tail.
static hipError_t rewind_if_needed(eik_fim2d* f) {
    if (!f->need_rewind) return hipSuccess;
    f->need_rewind = false;
    return fim2d_qrewind(f->a, f->stream);
}

// ---- a layered volume's block in a domain decomposition (split in x-y, the
// layers stay together): the layered solver (fim2dl.hip) with ghost strips of nl values per edge
// cell, driven by the relaunch schedule (eikonal/dd.py solve: iterate to local convergence, pack,
// exchange, merge)
int eik_fim3dl_create(eik_ctx* c, int64_t H, int64_t W, int64_t L, int z0, int nl, int dtype, eik_fim2d** out) {
    if (!c || !out) return EIK_ERR_ARG;
    const int kmax = dtype == EIK_F64 ? 3 : 4;
    if (nl < 1 || nl > kmax || z0 < 0 || z0 + nl > L)
        return set_err(c, EIK_ERR_ARG, "layered block: nl=%d z0=%d L=%ld (nl <= %d)", nl, z0, (long)L, kmax);
    // the layered kernel addresses T through one buffer resource per tile row band and layer: 32-bit
    // byte offsets over (rows + 2) raster rows of W cells of L values (fim3d_solve_one's gate)
    const int64_t esz = dtype == EIK_F64 ? 8 : 4;
    if (W < 1 || L < 1 || (fim2dl_rows(dtype == EIK_F64) + 2) * W * L * esz >= (int64_t)UINT32_MAX)
        return set_err(c, EIK_ERR_ARG, "layered block: a tile row band of W=%ld x L=%ld exceeds 4 GiB", (long)W, (long)L);
    const int rc = fim2d_create_rows(c, 1, H, W, dtype, fim2dl_rows(dtype == EIK_F64), out);
    if (rc) return rc;
    (*out)->lnl = nl;
    (*out)->lz0 = z0;
    (*out)->lL = L;
    return EIK_OK;
}

int eik_fim3dl_start(eik_fim2d* f, const void* d_cost, void* d_T, const int64_t goal[3], void* stream) {
    if (!f || !f->lnl || !d_cost || !d_T || !goal) return EIK_ERR_ARG;
    eik_ctx* c = f->ctx;
    HIPCHK(c, hipSetDevice(c->device));
    f->stream = (hipStream_t)stream;
    Fim2dArgs& a = f->a;
    a.cost = d_cost;
    a.T = d_T;
    a.ls = f->lL;
    a.z0 = f->lz0;
    a.lzs = 1;
    a.mode = kModePersistent;
    a.max_rounds = 1;
    a.keep = (float)(1.0 - c->tol);
    a.delta = __builtin_inff();
    a.edge_dirty = nullptr;
    a.bctl = nullptr;
    a.qhold = nullptr;
    a.live = nullptr;
    a.qtimeout = (unsigned long long)(c->qtimeout_s * 1e8);
    a.max_passes = c->passes > 0 ? c->passes : 24;  // the layered solver's (solve_layered)
    a.qbudget = c->max_visits ? c->max_visits : 1024ull * (unsigned long long)a.tiles_per_map + (1ull << 20);
    a.fresh_first = c->fresh_first;
    f->iterations = 0;
    f->host_syncs = 0;
    f->sweep_ms = f->solve_ms = 0.0;
    HIPCHK(c, hipMemsetAsync((void*)a.visits, 0, 3 * sizeof(unsigned long long), f->stream));
    // (the FIFO: priority bands on these blocks were measured slower -- 2048^2 x 3 in 2 x 2 blocks, fp64
    // 99 -> 108 ms, fp32 40 -> 44 ms, the same visits; the relaunch schedule has no work inflation for
    // them to remove, profiles/r05as_dd_layered_prio_probe.log)
    const bool in = goal[0] >= 0 && goal[1] >= 0 && goal[0] < f->W && goal[1] < f->H;
    if (in && (goal[2] < f->lz0 || goal[2] >= f->lz0 + f->lnl))
        return set_err(c, EIK_ERR_ARG, "goal layer %ld outside the solved layers", (long)goal[2]);
    // (a block without the goal: no seed -- its first launch ends at once, its ghosts bring the front)
    HIPCHK(c, fim2dl_init(a, f->f64, in ? goal[0] : -1, goal[1], goal[2] - f->lz0, f->H * f->W * f->lL, f->stream));
    f->started = true;
    f->need_rewind = false;
    return EIK_OK;
}

int eik_fim2d_iterate(eik_fim2d* f, int64_t max_iters, int64_t* active) {
    if (!f || !f->started) return EIK_ERR_ARG;
    eik_ctx* c = f->ctx;
    HIPCHK(c, hipSetDevice(c->device));
    if (f->lnl) {  // a layered block: one persistent launch to local convergence (fim2dl.hip)
        if (max_iters < 1) {
            if (active) *active = -1;
            return EIK_OK;
        }
        int& res = c->resident_l[f->f64 ? 1 : 0][f->lnl];
        if (res == 0) res = fim2dl_persist_resident(f->lnl, f->f64, c->cu_count);
        const int g = std::min(c->grid > 0 ? c->grid : 4 * c->cu_count, res);
        HIPCHK(c, hipEventRecord(f->ev_start, f->stream));
        HIPCHK(c, fim2dl_persist(f->a, f->lnl, f->f64, g, f->stream));  // (+ the queue rewind)
        HIPCHK(c, hipEventRecord(f->ev_stop, f->stream));
        ++f->iterations;
        HIPCHK(c, hipMemcpyAsync(f->h_q, f->qctl.p, kQueueCtlBytes, hipMemcpyDeviceToHost, f->stream));
        HIPCHK(c, hipStreamSynchronize(f->stream));
        ++f->host_syncs;
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, f->ev_start, f->ev_stop) == hipSuccess) f->solve_ms += ms;
        memcpy(f->h_visits, (const char*)f->h_q + kVisitsOff, 3 * sizeof(unsigned long long));
        return persist_result(f, active);
    }
    int64_t done = 0;
    int h = 1;
    const int grid = c->grid > 0 ? c->grid : 4 * c->cu_count;
    if (f->a.mode == kModePersistent) {  // one launch runs the local solve to its fixed point
        if (max_iters < 1) {
            if (active) *active = -1;
            return EIK_OK;
        }
        if (c->timing) {
            while (f->ev_pool.size() < f->ev_used + 2) {
                hipEvent_t ev;
                HIPCHK(c, hipEventCreate(&ev));
                f->ev_pool.push_back(ev);
            }
            HIPCHK(c, hipEventRecord(f->ev_pool[f->ev_used++], f->stream));
        }
        const bool wide = !f->f64 && f->a.tiles_per_map >= kWideTiles;  // one large raster (a batch of small maps: no gain)
        if (f->persist_grid == 0) f->persist_grid = fim2d_persist_resident(f->f64, c->cu_count, wide);
        const int g = std::min(grid, f->persist_grid);
        f->a.fresh_first = c->fresh_first;
        f->a.sched = c->sched;
        f->a.live_pack = c->live_pack;
        // eik_fim2d_solve launches without the queue rewind (the next solve's init clears the
        // queue); a later merge_ghost / iterate on the same solve issues it first (need_rewind)
        HIPCHK(c, rewind_if_needed(f));
        HIPCHK(c, fim2d_persist(f->a, f->f64, g, f->stream, wide, !f->defer_sync));
        f->need_rewind = f->defer_sync;
        if (c->timing) HIPCHK(c, hipEventRecord(f->ev_pool[f->ev_used++], f->stream));
        ++f->iterations;
        HIPCHK(c, hipMemcpyAsync(f->h_q, f->qctl.p, kQueueCtlBytes, hipMemcpyDeviceToHost, f->stream));
        if (f->defer_sync) return EIK_OK;  // eik_fim2d_solve: one synchronisation for the whole solve
        HIPCHK(c, hipStreamSynchronize(f->stream));
        ++f->host_syncs;
        if (c->timing) drain_timing(f);
        return persist_result(f, active);
    }
    while (done < max_iters) {
        const int64_t K = std::min<int64_t>(c->sync_every, max_iters - done);
        for (int64_t k = 0; k < K; ++k) {
            f->a.iter = (unsigned)f->iterations;
            if (c->timing) {
                while (f->ev_pool.size() < f->ev_used + 2) {
                    hipEvent_t ev;
                    HIPCHK(c, hipEventCreate(&ev));
                    f->ev_pool.push_back(ev);
                }
                HIPCHK(c, hipEventRecord(f->ev_pool[f->ev_used++], f->stream));
            }
            HIPCHK(c, fim2d_sweep(f->a, f->f64, grid, f->stream));
            if (c->timing) HIPCHK(c, hipEventRecord(f->ev_pool[f->ev_used++], f->stream));
            ++f->iterations;
        }
        done += K;
        HIPCHK(c, hipMemcpyAsync(f->h_counts, (int*)f->counts.p + (f->iterations % 3), sizeof(int),
                                 hipMemcpyDeviceToHost, f->stream));
        HIPCHK(c, hipStreamSynchronize(f->stream));
        ++f->host_syncs;
        if (c->timing) drain_timing(f);
        h = f->h_counts[0];
        if (h == 0) break;
    }
    if (active) *active = h;
    return EIK_OK;
}

int eik_fim2d_active(eik_fim2d* f, int64_t* active) {
    if (!f || !active) return EIK_ERR_ARG;
    eik_ctx* c = f->ctx;
    if (f->a.mode == kModePersistent) {
        HIPCHK(c, hipMemcpyAsync(f->h_q, f->qctl.p, kQueueCtlBytes, hipMemcpyDeviceToHost, f->stream));
        HIPCHK(c, hipStreamSynchronize(f->stream));
        *active = f->h_q[128 / 4];
        return EIK_OK;
    }
    HIPCHK(c, hipMemcpyAsync(f->h_counts, (int*)f->counts.p + (f->iterations % 3), sizeof(int), hipMemcpyDeviceToHost,
                             f->stream));
    HIPCHK(c, hipStreamSynchronize(f->stream));
    *active = f->h_counts[0];
    return EIK_OK;
}

static void fill_stats(const eik_fim2d* f, eik_stats* out);

// Wait for a solve's stream: poll first (a blocking wait's wake-up cost ~20 us per solve on the
// C2 raster, ~1 % of it), then block for long solves.
static hipError_t wait_stream(hipStream_t st) {
    static const int spin_on = [] {
        const char* v = getenv("EIK_WAIT_SPIN");
        return v ? atoi(v) : 1;
    }();
    if (!spin_on) return hipStreamSynchronize(st);
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spin = 0;; ++spin) {
        const hipError_t e = hipStreamQuery(st);
        if (e != hipErrorNotReady) return e;
        if ((spin & 63u) == 63u &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 0.02)
            return hipStreamSynchronize(st);
        __builtin_ia32_pause();
    }
}

// the stop event and the visit counters after the solve's launches, then ONE synchronisation
// (the persistent launch's queue words were queued for read-back behind it)
static int finish_solve(eik_fim2d* f, int64_t* active) {
    eik_ctx* c = f->ctx;
    HIPCHK(c, hipEventRecord(f->ev_stop, f->stream));
    const bool persist = f->a.mode == kModePersistent;  // h_q (queued after the launch) holds the counters
    if (!persist)
        HIPCHK(c, hipMemcpyAsync(f->h_visits, (void*)f->a.visits, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                                 f->stream));
    HIPCHK(c, wait_stream(f->stream));
    ++f->host_syncs;
    if (persist) memcpy(f->h_visits, (const char*)f->h_q + kVisitsOff, 3 * sizeof(unsigned long long));
    if (c->timing) drain_timing(f);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, f->ev_start, f->ev_stop);
    f->solve_ms = ms;
    fill_stats(f, &c->last);
    return f->a.mode == kModePersistent ? persist_result(f, active) : EIK_OK;
}

int eik_fim2d_solve(eik_fim2d* f, const void* d_cost, void* d_T, const int64_t* goals, void* stream) {
    int64_t active = 0;
    int rc = EIK_OK;
    for (int attempt = 0; attempt < 2; ++attempt) {
        rc = eik_fim2d_start(f, d_cost, d_T, goals, stream);
        if (rc) return rc;
        f->defer_sync = f->a.mode == kModePersistent;
        rc = eik_fim2d_iterate(f, f->max_iters, &active);
        f->defer_sync = false;
        if (!rc) rc = finish_solve(f, &active);  // (the persistent launch's error word is read here)
        if (!(rc && f->band_overflow)) break;
        // a priority band's ring was full: solve again from the start with the FIFO (this solver
        // keeps it); finish_solve waited for the stream
        f->band_overflow = false;
        f->no_bands = true;
    }
    if (rc) return rc;
    if (active != 0)
        return set_err(f->ctx, EIK_ERR_NOCONVERGE, "no convergence after %ld iterations (negative costs?)",
                       (long)f->iterations);
    return EIK_OK;
}

int eik_fim2d_pack_edges(eik_fim2d* f, void* n, void* s, void* w, void* e) {
    if (!f || !f->started) return EIK_ERR_ARG;
    if (f->lnl)  // a layered block: nl values per edge cell
        HIPCHK(f->ctx, fim2dl_pack_edges(f->a, f->lnl, f->f64, n, s, w, e, f->stream));
    else
        HIPCHK(f->ctx, fim2d_pack_edges(f->a, f->f64, n, s, w, e, f->stream));
    return EIK_OK;
}

int eik_fim2d_merge_ghost(eik_fim2d* f, int side, const void* recv) {
    if (!f || !f->started || side < 0 || side > 3 || !recv || !f->a.ghost[side]) return EIK_ERR_ARG;
    if (f->lnl) {  // a layered block (its launches rewind their queue themselves)
        HIPCHK(f->ctx, fim2dl_merge_ghost(f->a, f->lnl, f->f64, side, recv, f->stream));
        return EIK_OK;
    }
    f->a.iter = (unsigned)f->iterations;  // enqueue for the next sweep launch
    HIPCHK(f->ctx, rewind_if_needed(f));
    HIPCHK(f->ctx, fim2d_merge_ghost(f->a, f->f64, side, recv, side < 2 ? f->W : f->H, f->stream));
    return EIK_OK;
}

// ------------------------------------------------------------- live domain decomposition
static int live_box(eik_fim2d* f) {
    if (f->box) return EIK_OK;
    const hipError_t e = hipHostMalloc((void**)&f->box, sizeof(LiveBox), hipHostMallocCoherent);
    if (e != hipSuccess) {
        f->box = nullptr;
        return set_err(f->ctx, EIK_ERR_NOMEM, "live mailbox: %s", hipGetErrorString(e));
    }
    memset(f->box, 0, sizeof(LiveBox));
    return EIK_OK;
}

int eik_fim2d_live_bind(eik_fim2d* f, void* const send[8], void* const recv[8]) {
    if (!f || !send || !recv) return EIK_ERR_ARG;
    if (f->live_on) return set_err(f->ctx, EIK_ERR_ARG, "cannot rebind strips during a live launch");
    int rc = live_box(f);
    if (rc) return rc;
    for (int p = 0; p < 2; ++p)
        for (int s = 0; s < 4; ++s) {
            f->box->send[p][s] = send[p * 4 + s];
            f->box->recv[p][s] = recv[p * 4 + s];
        }
    return EIK_OK;
}

// post one command to the halo agent and wait for it (bounded by the queue timeout)
static int live_cmd(eik_fim2d* f, unsigned op, unsigned par) {
    eik_ctx* c = f->ctx;
    LiveBox* b = f->box;
    const unsigned seq = __atomic_load_n(&b->seq, __ATOMIC_RELAXED) + 1u;
    __atomic_store_n(&b->cmd, op | (par & 1u) << 8, __ATOMIC_RELAXED);
    __atomic_store_n(&b->seq, seq, __ATOMIC_RELEASE);
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spin = 0; __atomic_load_n(&b->done, __ATOMIC_ACQUIRE) != seq; ++spin) {
        if ((spin & 1023u) == 1023u) {
            const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (el > c->qtimeout_s + 1.0)
                return set_err(c, EIK_ERR_HIP, "live solve: the halo agent did not answer within %.1f s", el);
            if (__atomic_load_n(&b->error, __ATOMIC_RELAXED) & 1u) break;
            // the launch ended early (fault, or every workgroup left): nothing will answer
            if (hipStreamQuery(f->stream) == hipSuccess) {
                // the queue's words (error bits: 1 a wait timed out, 2 the visit budget, 4 a priority
                // band's ring lapped), the visit counters and the fullest band (tail - head)
                unsigned q[kQueueCtlBytes / 4] = {};
                (void)hipMemcpy(q, f->qctl.p, kQueueCtlBytes, hipMemcpyDeviceToHost);
                unsigned long long vis[2] = {};
                memcpy(vis, (const char*)q + kVisitsOff, sizeof vis);
                long long band_max = -1;
                if (f->a.bctl) {
                    std::vector<unsigned long long> bw(16 * kBands);
                    if (hipMemcpy(bw.data(), f->a.bctl, 128 * kBands, hipMemcpyDeviceToHost) == hipSuccess)
                        for (int b = 0; b < kBands; ++b)
                            band_max = std::max(band_max, (long long)(bw[16 * b + 8] - bw[16 * b]));
                }
                unsigned long long qh = 0, qt = 0;
                memcpy(&qh, q, 8);
                memcpy(&qt, (const char*)q + 64, 8);
                return set_err(c, EIK_ERR_HIP,
                               "live solve: the persistent launch is no longer running (queue error %u, active %d, "
                               "visits %llu, passes %llu, fifo head-tail %lld, fullest band %lld of %u slots)",
                               q[192 / 4], (int)q[128 / 4], vis[0], vis[1], (long long)(qh - qt), band_max,
                               f->a.bctl ? f->a.bmask + 1u : 0u);
            }
        }
        __builtin_ia32_pause();
    }
    const unsigned err = __atomic_load_n(&b->error, __ATOMIC_RELAXED);
    if (err & 4u)
        return set_err(c, EIK_ERR_HIP, "live solve: a priority band's ring is full (EIK_OPT_PRIO=0 or a larger "
                                       "EIK_OPT_PRIO_RING)");
    if (err & 1u)
        return set_err(c, EIK_ERR_HIP, "live solve: a queue wait exceeded %.1f s (EIK_OPT_QTIMEOUT)", c->qtimeout_s);
    if (err & 2u)
        return set_err(c, EIK_ERR_NOCONVERGE, "no convergence within %llu tile visits (negative costs?)",
                       (unsigned long long)f->a.qbudget);
    return EIK_OK;
}

int eik_fim2d_launch(eik_fim2d* f, int live) {
    if (!f || !f->started) return EIK_ERR_ARG;
    eik_ctx* c = f->ctx;
    if (f->live_on) return set_err(c, EIK_ERR_ARG, "a live launch is still running (eik_fim2d_release)");
    if (f->a.mode != kModePersistent)
        return set_err(c, EIK_ERR_ARG, "eik_fim2d_launch needs the persistent mode (EIK_OPT_MODE)");
    HIPCHK(c, hipSetDevice(c->device));
    const int grid = c->grid > 0 ? c->grid : 4 * c->cu_count;
    const bool wide = !f->f64 && f->a.tiles_per_map >= kWideTiles;  // one large raster (a batch of small maps: no gain)
    if (f->lnl) {  // a layered block (eik_fim3dl_create): the layered kernel's co-resident count
        int& res = c->resident_l[f->f64 ? 1 : 0][f->lnl];
        if (res == 0) res = fim2dl_persist_resident(f->lnl, f->f64, c->cu_count);
        f->persist_grid = res;
    } else if (f->persist_grid == 0) {
        f->persist_grid = fim2d_persist_resident(f->f64, c->cu_count, wide);
    }
    Fim2dArgs a = f->a;
    if (live) {
        int rc = live_box(f);
        if (rc) return rc;
        hipError_t e = f->hold.ensure(64);
        if (e != hipSuccess) return set_err(c, EIK_ERR_NOMEM, "live hold word: %s", hipGetErrorString(e));
        HIPCHK(c, hipMemsetAsync(f->hold.p, 0, 64, f->stream));
        f->box->seq = f->box->done = 0;
        f->box->error = 0;
        a.qhold = (unsigned*)f->hold.p;
        a.live = f->box;
    }
    if (c->timing) {
        while (f->ev_pool.size() < f->ev_used + 2) {
            hipEvent_t ev;
            HIPCHK(c, hipEventCreate(&ev));
            f->ev_pool.push_back(ev);
        }
        HIPCHK(c, hipEventRecord(f->ev_pool[f->ev_used++], f->stream));
    }
    // live: workgroup 0 is the halo agent (dispatched first); the others should be co-resident (grid <= resident)
    const int g = std::max(live ? 2 : 1, std::min(grid, f->persist_grid));
    a.fresh_first = c->fresh_first;
    a.sched = c->sched;
    if (f->lnl) {  // (its launches rewind their queue themselves)
        // a live layered block orders its waiting tiles on the priority bands at width >= 1, as the 2D
        // blocks do (§3.2): on the FIFO the blocks re-solved their interiors as the ghosts' corrections
        // arrived (C5 split 4 x 2: 4.5 x the single domain's visits, profiles/r06i_c4_rehearsal_n8.log).
        // (The relaunch schedule keeps the FIFO: its launches run to local convergence either way.)
        const double prio = c->prio >= 0 ? c->prio : std::max(1.0, default_prio(f->H, f->W, 0.0));
        a.bctl = nullptr;
        if (live && prio > 0 && a.capacity < (1 << kBandTagShift) - 1) {
            HIPCHK(c, setup_bands(c, f->bslot, f->bctl, a.capacity, a, f->stream));
            HIPCHK(c, hipMemsetD32Async((hipDeviceptr_t)a.key, 0x7f800000u, (size_t)a.capacity, f->stream));  // keys: +inf
            float* pd = (float*)((char*)f->bctl.p + 128 * kBands);
            HIPCHK(c, fim2d_prio_delta(a.cost, f->f64, f->H * f->W * f->lL, (float)prio, pd, f->stream));
            a.pdelta = pd;
            a.disp = c->prio_dispatch > 0 ? (unsigned)c->prio_dispatch : 32u;
        }
        HIPCHK(c, fim2dl_persist(a, f->lnl, f->f64, g, f->stream));
    } else {
        HIPCHK(c, rewind_if_needed(f));
        HIPCHK(c, fim2d_persist(a, f->f64, g, f->stream, wide));
    }
    if (c->timing) HIPCHK(c, hipEventRecord(f->ev_pool[f->ev_used++], f->stream));
    f->live_on = live != 0;
    ++f->iterations;
    return EIK_OK;
}

int eik_fim2d_live_pack(eik_fim2d* f, int par) {
    if (!f || !f->live_on) return EIK_ERR_ARG;
    return live_cmd(f, kLivePack, (unsigned)par);
}

int eik_fim2d_live_merge(eik_fim2d* f, int par, int64_t* active, int64_t* changed) {
    if (!f || !f->live_on) return EIK_ERR_ARG;
    int rc = live_cmd(f, kLiveMerge, (unsigned)par);
    if (rc) return rc;
    ++f->host_syncs;
    if (active) *active = __atomic_load_n(&f->box->active, __ATOMIC_RELAXED);
    if (changed) *changed = __atomic_load_n(&f->box->changed, __ATOMIC_RELAXED);
    return EIK_OK;
}

int eik_fim2d_release(eik_fim2d* f, int64_t* active) {
    if (!f || !f->live_on) return EIK_ERR_ARG;
    eik_ctx* c = f->ctx;
    f->live_on = false;
    const int rc_cmd = live_cmd(f, kLiveRelease, 0);
    HIPCHK(c, hipMemcpyAsync(f->h_q, f->qctl.p, kQueueCtlBytes, hipMemcpyDeviceToHost, f->stream));
    HIPCHK(c, hipStreamSynchronize(f->stream));
    ++f->host_syncs;
    if (c->timing) drain_timing(f);
    if (rc_cmd) return rc_cmd;
    const unsigned err = f->h_q[192 / 4];
    if (err & 4u)
        return set_err(c, EIK_ERR_HIP, "live solve: a priority band's ring is full (EIK_OPT_PRIO=0 or a larger "
                                       "EIK_OPT_PRIO_RING)");
    if (err & 1u)
        return set_err(c, EIK_ERR_HIP, "live solve: a queue wait exceeded %.1f s (EIK_OPT_QTIMEOUT)", c->qtimeout_s);
    if (err & 2u)
        return set_err(c, EIK_ERR_NOCONVERGE, "no convergence within %llu tile visits (negative costs?)",
                       (unsigned long long)f->a.qbudget);
    if (active) *active = f->h_q[128 / 4];
    return EIK_OK;
}

// ---------------------------------------------------------------- inter-process buffers
int eik_host_alloc(int64_t bytes, void** out) {
    if (!out || bytes <= 0) return EIK_ERR_ARG;
    *out = nullptr;
    void* p = nullptr;
    const hipError_t e = hipHostMalloc(&p, (size_t)bytes, hipHostMallocDefault);
    if (e != hipSuccess) return set_err(nullptr, EIK_ERR_NOMEM, "pinned host allocation of %lld bytes: %s",
                                        (long long)bytes, hipGetErrorString(e));
    std::lock_guard<std::mutex> lk(g_pin_mu);
    g_pinned.emplace_back(reinterpret_cast<uintptr_t>(p), (size_t)bytes);
    *out = p;
    return EIK_OK;
}

int eik_host_free(void* p) {
    if (!p) return EIK_OK;
    {
        std::lock_guard<std::mutex> lk(g_pin_mu);
        auto it = std::find_if(g_pinned.begin(), g_pinned.end(),
                               [&](const std::pair<uintptr_t, size_t>& b) { return b.first == reinterpret_cast<uintptr_t>(p); });
        if (it == g_pinned.end()) return EIK_ERR_ARG;
        g_pinned.erase(it);
    }
    return hipHostFree(p) == hipSuccess ? EIK_OK : EIK_ERR_HIP;
}

int eik_ipc_alloc(eik_ctx* c, int64_t bytes, void** d_ptr, unsigned char handle[64]) {
    if (!c || !d_ptr || !handle || bytes <= 0) return EIK_ERR_ARG;
    static_assert(sizeof(hipIpcMemHandle_t) <= 64, "IPC handle size");
    HIPCHK(c, hipSetDevice(c->device));
    void* p = nullptr;
    HIPCHK(c, hipMalloc(&p, (size_t)bytes));
    hipIpcMemHandle_t h;
    const hipError_t e = hipIpcGetMemHandle(&h, p);
    if (e != hipSuccess) {
        (void)hipFree(p);
        return set_err(c, EIK_ERR_HIP, "hipIpcGetMemHandle: %s", hipGetErrorString(e));
    }
    memset(handle, 0, 64);
    memcpy(handle, &h, sizeof h);
    *d_ptr = p;
    return EIK_OK;
}

int eik_ipc_free(eik_ctx* c, void* d_ptr) {
    if (!c) return EIK_ERR_ARG;
    if (d_ptr) HIPCHK(c, hipFree(d_ptr));
    return EIK_OK;
}

int eik_ipc_open(eik_ctx* c, const unsigned char handle[64], void** d_ptr) {
    if (!c || !handle || !d_ptr) return EIK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    hipIpcMemHandle_t h;
    memcpy(&h, handle, sizeof h);
    HIPCHK(c, hipIpcOpenMemHandle(d_ptr, h, hipIpcMemLazyEnablePeerAccess));
    return EIK_OK;
}

int eik_ipc_close(eik_ctx* c, void* d_ptr) {
    if (!c) return EIK_ERR_ARG;
    if (d_ptr) HIPCHK(c, hipIpcCloseMemHandle(d_ptr));
    return EIK_OK;
}

int eik_fim2d_stats(eik_fim2d* f, eik_stats* out) {
    if (!f || !out) return EIK_ERR_ARG;
    if (f->started) {
        eik_ctx* c = f->ctx;
        HIPCHK(c, hipMemcpyAsync(f->h_visits, (void*)f->a.visits, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                                 f->stream));
        HIPCHK(c, hipStreamSynchronize(f->stream));
    }
    fill_stats(f, out);
    return EIK_OK;
}

static void fill_stats(const eik_fim2d* f, eik_stats* out) {
    out->iterations = f->iterations;
    out->tile_visits = (int64_t)f->h_visits[0];
    out->inplace_passes = (int64_t)f->h_visits[1];
    out->host_syncs = f->host_syncs;
    out->solve_ms = f->solve_ms;
    out->sweep_ms = f->sweep_ms;
    out->fresh_visits = (int64_t)f->h_visits[2];
    out->bytes_alg = (double)out->tile_visits * bytes_per_visit(f->f64) -
                     (double)out->fresh_visits * kTile * kTile * (f->f64 ? 8 : 4) +
                     (double)out->inplace_passes * bytes_per_pass(f->f64) +
                     (double)f->B * f->H * f->W * (f->f64 ? 8 : 4);
}

}  // extern "C"

// ------------------------------------------------------------------- host-buffer drop-ins
static int get_solver(eik_ctx* c, int64_t B, int64_t H, int64_t W, int dtype, eik_fim2d** out) {
    eik_fim2d* f = c->cached;
    if (f && f->B == B && f->H == H && f->W == W && (int)f->f64 == (dtype == EIK_F64)) {
        *out = f;
        return EIK_OK;
    }
    if (f) eik_fim2d_destroy(f);
    c->cached = nullptr;
    int rc = eik_fim2d_create(c, B, H, W, dtype, &f);
    if (rc) return rc;
    c->cached = f;
    *out = f;
    return EIK_OK;
}

// Costs must be >= 0 or +inf (negative or NaN: EIK_ERR_ARG).  Checked on the device copy `dev`
// of the host array `cost` (a host scan of a 4096^2 f64 raster took ~19 ms at one core's memory
// bandwidth): one short kernel and an 8-byte read-back, before anything is solved.
template <typename R>
static int check_cost(eik_ctx* c, const R* cost, const void* dev, int64_t n, hipStream_t st) {
    HIPCHK(c, c->misc.ensure(64));
    unsigned long long* first = (unsigned long long*)c->misc.p + 7;  // (words 0..: the join's)
    HIPCHK(c, cost_check(dev, n, sizeof(R) == 8, first, st));
    unsigned long long i = 0;
    HIPCHK(c, hipMemcpyAsync(&i, first, sizeof i, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    if (i != ~0ull)
        return set_err(c, EIK_ERR_ARG, "cost[%ld] = %g: costs must be >= 0 or +inf", (long)i, (double)cost[i]);
    return EIK_OK;
}

template <typename R>
static int tmap_host(eik_ctx* c, const R* cost, int64_t B, int64_t H, int64_t W, const int64_t* goals, R* T) {
    if (!c || !cost || !T || !goals || B < 1 || H < 1 || W < 1) return c ? set_err(c, EIK_ERR_ARG, "bad arguments") : EIK_ERR_ARG;
    for (int64_t b = 0; b < B; ++b)
        if (goals[2 * b] < 0 || goals[2 * b + 1] < 0 || goals[2 * b] >= W || goals[2 * b + 1] >= H)
            return set_err(c, EIK_ERR_ARG, "goal (%ld, %ld) of map %ld outside %ldx%ld", (long)goals[2 * b],
                           (long)goals[2 * b + 1], (long)b, (long)H, (long)W);
    const int64_t n = B * H * W;
    HIPCHK(c, hipSetDevice(c->device));
    eik_fim2d* f = nullptr;
    int rc = get_solver(c, B, H, W, sizeof(R) == 8 ? EIK_F64 : EIK_F32, &f);
    if (rc) return rc;
    HIPCHK(c, c->cost.ensure(sizeof(R) * n));
    HIPCHK(c, c->T.ensure(sizeof(R) * n));
    HIPCHK(c, host_to_dev(c, c->cost.p, cost, sizeof(R) * n, c->stream));
    rc = check_cost(c, cost, c->cost.p, n, c->stream);
    if (rc) return rc;
    rc = eik_fim2d_solve(f, c->cost.p, c->T.p, goals, c->stream);
    if (rc) return rc;
    HIPCHK(c, dev_to_host(c, T, c->T.p, sizeof(R) * n, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return EIK_OK;
}

extern "C" {

int eik_tmap2d_f32(eik_ctx* c, const float* cost, int64_t H, int64_t W, int64_t gx, int64_t gy, float* T) {
    const int64_t g[2] = {gx, gy};
    return tmap_host<float>(c, cost, 1, H, W, g, T);
}

int eik_tmap2d_f64(eik_ctx* c, const double* cost, int64_t H, int64_t W, int64_t gx, int64_t gy, double* T) {
    const int64_t g[2] = {gx, gy};
    return tmap_host<double>(c, cost, 1, H, W, g, T);
}

int eik_tmap2d_batch_f32(eik_ctx* c, const float* cost, int64_t B, int64_t H, int64_t W, const int64_t* goals,
                         float* T) {
    return tmap_host<float>(c, cost, B, H, W, goals, T);
}

// nodeJoin + partial fields from the two device-resident full fields dT[0:n] (goal front) and
// dT[n:2n] (start front), in place; *best = the packed join (~0: the fronts never meet).  d_cost
// (the fronts' raster): band cells by the band relaxation (bidir.hip), else at their full-field
// values; d_chk: the capped fronts' check.  Ends with the stream synchronised on *best.
// src (with d_cost): the goal's and the start's linear index, for EIK_OPT_EXACT_BAND's replay.
static int join_and_partial(eik_ctx* c, double* dT, int64_t n, int64_t H, int64_t W, unsigned long long* best,
                            int64_t members[2], const double* d_cost = nullptr, FrontsCheck* d_chk = nullptr,
                            FrontsCheck* h_chk = nullptr, const int64_t* src = nullptr) {
    hipStream_t st = c->stream;
    HIPCHK(c, c->work.ensure(bidir_join_work_bytes(n)));
    HIPCHK(c, c->misc.ensure(64));
    HIPCHK(c, bidir_join(dT, dT + n, n, c->work.p, c->work.bytes, (unsigned long long*)c->misc.p, st, members));
    if (d_cost && src && c->exact_band && members[0] > 0 && members[1] > 0) {
        // the reference's own band values, LIFO ties and nodeJoin, replayed from the join's ranks
        const unsigned *rg = nullptr, *rs = nullptr;
        bidir_join_ranks(c->work.p, n, &rg, &rs);
        HIPCHK(c, c->exact.ensure(bidir_exact_work_bytes(n, members[0], members[1])));
        hipEvent_t e0 = nullptr, e1 = nullptr;
        HIPCHK(c, hipEventCreate(&e0));
        HIPCHK(c, hipEventCreate(&e1));
        HIPCHK(c, hipEventRecord(e0, st));
        unsigned long long info[4] = {0, 0, 0, 0};
        const hipError_t e = bidir_exact(dT, dT + n, d_cost, H, W, src[0], src[1], rg, rs, members, c->exact.p,
                                         c->exact.bytes, (unsigned long long*)c->misc.p, st, info);
        if (e == hipErrorNotReady || e == hipErrorNotSupported || e == hipErrorIllegalState) {
            (void)hipEventDestroy(e0);
            (void)hipEventDestroy(e1);
            return set_err(c, EIK_ERR_NOCONVERGE,
                           e == hipErrorNotReady      ? "biComputeTmap: the exact band replay did not settle"
                           : e == hipErrorNotSupported ? "biComputeTmap: the exact band replay met a run of more than "
                                                         "4096 cells of exactly equal T (a zero-cost region)"
                                                       : "biComputeTmap: the exact meeting is not clear of the ranked "
                                                         "cells' bound");
        }
        HIPCHK(c, e);
        HIPCHK(c, hipEventRecord(e1, st));
        HIPCHK(c, hipMemcpyAsync(best, c->misc.p, sizeof *best, hipMemcpyDeviceToHost, st));
        HIPCHK(c, hipStreamSynchronize(st));
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        for (int q = 0; q < 4; ++q) c->exact_info[q] = info[q];
        c->exact_info[4] = (unsigned long long)(ms * 1000.0f);
        for (int q = 0; q < 4; ++q) c->fronts_info[6 + q] = 0;
        if (d_chk) {
            HIPCHK(c, hipMemcpyAsync(h_chk, d_chk, sizeof *h_chk, hipMemcpyDeviceToHost, st));
            HIPCHK(c, hipStreamSynchronize(st));
            h_chk->viol = 0;  // band values come from the replay's events, not from the capped field
        }
        return EIK_OK;
    }
    {
        const hipError_t e = bidir_partial(dT, dT + n, H, W, c->work.p, (const unsigned long long*)c->misc.p, st, d_cost,
                                           d_chk ? &d_chk->viol : nullptr);
        if (e == hipErrorNotReady)
            return set_err(c, EIK_ERR_NOCONVERGE, "biComputeTmap: the band relaxation of the partial fields did not settle");
        HIPCHK(c, e);
    }
    if (d_cost) {
        unsigned bs[4] = {0, 0, 0, 0};
        HIPCHK(c, bidir_band_stats(c->work.p, n, bs, st));
        for (int q = 0; q < 4; ++q) c->fronts_info[6 + q] = bs[q];
    }
    HIPCHK(c, hipMemcpyAsync(best, c->misc.p, sizeof *best, hipMemcpyDeviceToHost, st));
    if (d_chk) HIPCHK(c, hipMemcpyAsync(h_chk, d_chk, sizeof *h_chk, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    return EIK_OK;
}

// Capped fronts: rasters of at least kFrontsCapCells cells, F x F coarse blocks with F =
// max(4, ceil(max(H, W) / 512)), cap = F x (coarse T at the join bound's rank K0, bidir.hip
// fronts_estimate) x margin (kFrontsMargin, EIK_OPT_FRONTS_CAP) + the largest finite cost
constexpr int64_t kFrontsCapCells = 1 << 20;

// biComputeTmap's two fronts (FastMarching.py:114-162) as one B = 2 batch -- map 0 from the goal
// (g[0], g[1]), map 1 from the start (g[2], g[3]) -- over the device cost dcost (both maps), into
// dT, then nodeJoin (*best) and the partial fields.  The fronts only matter up to their meeting,
// so by default (EIK_OPT_FRONTS_CAP) each is solved only up to a cap on T estimated from a coarse
// copy of the raster (bidir.hip "capped fronts"); a capped result that cannot be shown equal to
// the full one (meeting rank at or above a front's kept cells, a band cell cut off, no meeting)
// is replaced by the uncapped solve.
static int solve_fronts(eik_ctx* c, eik_fim2d* f, double* dcost, double* dT, const int64_t g[4], int64_t H, int64_t W,
                        unsigned long long* best) {
    hipStream_t st = c->stream;
    const int64_t n = H * W;
    const int64_t src[2] = {g[1] * W + g[0], g[3] * W + g[2]};
    for (int64_t& v : c->fronts_info) v = 0;  // (join_and_partial fills the band entries)
    for (auto& v : c->exact_info) v = 0;
    // exact band: the fronts in the reference's arithmetic, so the replay mostly confirms their values
    struct RefArith {
        eik_fim2d* f;
        RefArith(eik_fim2d* f_, bool on) : f(f_) { f->a.ref_arith = on ? 1 : 0; }
        ~RefArith() { f->a.ref_arith = 0; }
    } ref_guard(f, c->exact_band);
    HIPCHK(c, c->work.ensure(bidir_join_work_bytes(n)));
    const bool capped = c->fronts_cap > 0 && n >= kFrontsCapCells && std::min(H, W) >= 256;
    if (capped) {
        // coarse side 512 (EIK_FRONTS_COARSE, diagnostics): 256 / 1024 were slower at 4096^2
        // (profiles/r04t_fronts_coarse_side.log: looser caps / a longer coarse chain)
        static const int64_t cside = getenv("EIK_FRONTS_COARSE") ? std::max(64, atoi(getenv("EIK_FRONTS_COARSE"))) : 512;
        const int64_t F = std::max<int64_t>(4, (std::max(H, W) + cside - 1) / cside);
        const int64_t Hc = (H + F - 1) / F, Wc = (W + F - 1) / F, nc = Hc * Wc;
        const size_t cb = sizeof(double) * 2 * nc;
        HIPCHK(c, c->fronts.ensure(2 * cb + 256));
        double* ccost = (double*)c->fronts.p;
        double* cT = ccost + 2 * nc;
        FrontsCheck* chk = (FrontsCheck*)((char*)c->fronts.p + 2 * cb);
        HIPCHK(c, fronts_coarse_cost(dcost, H, W, (int)F, ccost, Hc, Wc, chk, st));
        HIPCHK(c, hipMemcpyAsync(ccost + nc, ccost, sizeof(double) * nc, hipMemcpyDeviceToDevice, st));
        eik_fim2d* fc = c->cached_fronts;
        if (!fc || fc->H != Hc || fc->W != Wc) {
            if (fc) eik_fim2d_destroy(fc);
            c->cached_fronts = nullptr;
            int rc = eik_fim2d_create(c, 2, Hc, Wc, EIK_F64, &fc);
            if (rc) return rc;
            c->cached_fronts = fc;
        }
        const int64_t gc[4] = {g[0] / F, g[1] / F, g[2] / F, g[3] / F};
        const eik_stats keep = c->last;  // the coarse estimate's solve is not the caller's
        int rc = eik_fim2d_solve(fc, ccost, cT, gc, st);
        c->last = keep;
        if (rc) return rc;
        HIPCHK(c, fronts_estimate(cT, cT + nc, nc, c->work.p, (double)F, c->fronts_cap, chk, st));
        f->a.tcap = chk->caps;
        rc = eik_fim2d_solve(f, dcost, dT, g, st);
        f->a.tcap = nullptr;
        if (rc) return rc;
        HIPCHK(c, fronts_clean(dT, n, chk, st));
        FrontsCheck h{};
        int64_t mem[2] = {0, 0};
        rc = join_and_partial(c, dT, n, H, W, best, mem, dcost, chk, &h, src);
        if (rc) return rc;
        const unsigned long long k = *best >> 30;
        const bool ok = *best != ~0ull && h.viol == 0 && k < h.kept[0] && k < h.kept[1];
        c->fronts_info[0] = std::isfinite(h.caps[0]) || std::isfinite(h.caps[1]);
        c->fronts_info[2] = h.kept[0];
        c->fronts_info[3] = h.kept[1];
        c->fronts_info[4] = mem[0];
        c->fronts_info[5] = mem[1];
        if (ok || !c->fronts_info[0]) return EIK_OK;  // (no finite cap: that was the full solve)
        c->fronts_info[1] = 1;  // the capped fronts did not settle the join: solve them in full
    }
    int rc = eik_fim2d_solve(f, dcost, dT, g, st);
    if (rc) return rc;
    int64_t mem[2] = {0, 0};
    rc = join_and_partial(c, dT, n, H, W, best, mem, dcost, nullptr, nullptr, src);
    if (!capped) {
        c->fronts_info[4] = mem[0];
        c->fronts_info[5] = mem[1];
    }
    return rc;
}

int eik_exact_info(const eik_ctx* c, int64_t out[5]) {
    if (!c || !out) return EIK_ERR_ARG;
    for (int i = 0; i < 5; ++i) out[i] = (int64_t)c->exact_info[i];
    return EIK_OK;
}

int eik_fronts_info(const eik_ctx* c, int64_t out[10]) {
    if (!c || !out) return EIK_ERR_ARG;
    for (int i = 0; i < 10; ++i) out[i] = c->fronts_info[i];
    return EIK_OK;
}

int eik_tmap2d_bidir_f64(eik_ctx* c, const double* cost, int64_t H, int64_t W, int64_t gx, int64_t gy, int64_t sx,
                         int64_t sy, double* TG, double* TS, uint32_t join[2]) {
    if (!c || !cost || !TG || !TS || !join) return c ? set_err(c, EIK_ERR_ARG, "NULL argument") : EIK_ERR_ARG;
    const int64_t n = H * W;
    if (n >= (1ll << 29)) return set_err(c, EIK_ERR_ARG, "bidirectional join supports < 2^29 cells");
    // both fronts as one 2-map batch: map 0 from the goal, map 1 from the start.  The raster goes up
    // once and is duplicated on the device; the fields come back straight into TG / TS (no host
    // staging copies: the drop-in's biComputeTmap spent ~200 ms in them for a 4096^2 raster)
    const int64_t goals[4] = {gx, gy, sx, sy};
    for (int b = 0; b < 2; ++b)
        if (goals[2 * b] < 0 || goals[2 * b + 1] < 0 || goals[2 * b] >= W || goals[2 * b + 1] >= H)
            return set_err(c, EIK_ERR_ARG, "node (%ld, %ld) outside %ldx%ld", (long)goals[2 * b], (long)goals[2 * b + 1],
                           (long)H, (long)W);
    HIPCHK(c, hipSetDevice(c->device));
    eik_fim2d* f = nullptr;
    int rc = get_solver(c, 2, H, W, EIK_F64, &f);
    if (rc) return rc;
    HIPCHK(c, c->cost.ensure(sizeof(double) * 2 * n));
    HIPCHK(c, c->T.ensure(sizeof(double) * 2 * n));
    double* dcost = (double*)c->cost.p;
    HIPCHK(c, host_to_dev(c, dcost, cost, sizeof(double) * n, c->stream));
    rc = check_cost(c, cost, dcost, n, c->stream);
    if (rc) return rc;
    HIPCHK(c, hipMemcpyAsync(dcost + n, dcost, sizeof(double) * n, hipMemcpyDeviceToDevice, c->stream));
    // the fronts (c->T holds both maps back to back), nodeJoin and the partial fields at the
    // meeting iteration (FastMarching.py:141-162)
    unsigned long long best = 0;
    rc = solve_fronts(c, f, dcost, (double*)c->T.p, goals, H, W, &best);
    if (rc) return rc;
    HIPCHK(c, dev_to_host(c, TG, c->T.p, sizeof(double) * n, c->stream));
    HIPCHK(c, dev_to_host(c, TS, (double*)c->T.p + n, sizeof(double) * n, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (best == ~0ull) return set_err(c, EIK_ERR_UNREACHABLE, "goal and start are not connected");
    const int64_t node = (int64_t)(best & ((1ull << 29) - 1));
    join[0] = (uint32_t)(node % W);
    join[1] = (uint32_t)(node / W);
    return EIK_OK;
}

int eik_bidir_join_f64(eik_ctx* c, const double* TG, const double* TS, int64_t H, int64_t W, double* TGp,
                       double* TSp, uint32_t join[2], int64_t members[2]) {
    if (!c || !TG || !TS || !TGp || !TSp || !join) return c ? set_err(c, EIK_ERR_ARG, "NULL argument") : EIK_ERR_ARG;
    if (H < 1 || W < 1) return set_err(c, EIK_ERR_ARG, "empty field");
    const int64_t n = H * W;
    if (n >= (1ll << 29)) return set_err(c, EIK_ERR_ARG, "bidirectional join supports < 2^29 cells");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, c->T.ensure(sizeof(double) * 2 * n));
    double* dT = (double*)c->T.p;
    HIPCHK(c, host_to_dev(c, dT, TG, sizeof(double) * n, c->stream));
    HIPCHK(c, host_to_dev(c, dT + n, TS, sizeof(double) * n, c->stream));
    unsigned long long best = 0;
    int64_t mem[2] = {0, 0};
    int rc = join_and_partial(c, dT, n, H, W, &best, mem);
    if (rc) return rc;
    if (members) {
        members[0] = mem[0];
        members[1] = mem[1];
    }
    if (best == ~0ull) return set_err(c, EIK_ERR_UNREACHABLE, "the fields share no finite cell");
    HIPCHK(c, dev_to_host(c, TGp, dT, sizeof(double) * n, c->stream));
    HIPCHK(c, dev_to_host(c, TSp, dT + n, sizeof(double) * n, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const int64_t node = (int64_t)(best & ((1ull << 29) - 1));
    join[0] = (uint32_t)(node % W);
    join[1] = (uint32_t)(node / W);
    return EIK_OK;
}

int eik_selftest_walker_math(eik_ctx* c, int64_t n, uint64_t seed, int64_t mismatches[6]) {
    if (!c || !mismatches || n < 1) return EIK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, c->misc.ensure(64));
    unsigned long long* d = (unsigned long long*)c->misc.p;
    HIPCHK(c, hipMemsetAsync(d, 0, 6 * sizeof(unsigned long long), c->stream));
    HIPCHK(c, walker_math_selftest((long long)n, (unsigned long long)seed, d, c->stream));
    unsigned long long h[6];
    HIPCHK(c, hipMemcpyAsync(h, d, sizeof h, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (int k = 0; k < 6; ++k) mismatches[k] = (int64_t)h[k];
    return EIK_OK;
}

int eik_path2d_dev(eik_ctx* c, const void* d_T, int dtype, int64_t H, int64_t W, const double init[2],
                   const double end[2], double tau, double* d_out, int64_t cap, int64_t* d_n_out, int* d_status,
                   void* stream) {
    if (!c || !d_T || !init || !end || !d_out || !d_n_out || !d_status || cap < 2 || H < 3 || W < 3 || !(tau > 0))
        return c ? set_err(c, EIK_ERR_ARG, "bad path arguments") : EIK_ERR_ARG;
    Gdm2dArgs a;
    a.T = d_T;
    a.H = H;
    a.W = W;
    a.ix = init[0];
    a.iy = init[1];
    a.ex = end[0];
    a.ey = end[1];
    a.tau = tau;
    a.steps = (long)std::nearbyint(15000.0 / tau);  // round(15000/tau), FastMarching.py:173
    a.out = d_out;
    a.cap = cap;
    a.n_out = d_n_out;
    a.status = d_status;
    a.fused = c->path_loop;
    HIPCHK(c, gdm2d(a, dtype == EIK_F64, (hipStream_t)stream));
    return EIK_OK;
}

int eik_path2d_f64(eik_ctx* c, const double* T, int64_t H, int64_t W, const double init[2], const double end[2],
                   double tau, double* out, int64_t cap, int64_t* n_out, int* status) {
    if (!c || !T || !out || !n_out || !status) return c ? set_err(c, EIK_ERR_ARG, "NULL argument") : EIK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t n = H * W;
    HIPCHK(c, c->T2.ensure(sizeof(double) * n));
    HIPCHK(c, c->work.ensure(sizeof(double) * 2 * cap + 64));
    HIPCHK(c, host_to_dev(c, c->T2.p, T, sizeof(double) * n, c->stream));
    double* d_out = (double*)c->work.p;
    int64_t* d_n = (int64_t*)(d_out + 2 * cap);
    int* d_st = (int*)(d_n + 1);
    int rc = eik_path2d_dev(c, c->T2.p, EIK_F64, H, W, init, end, tau, d_out, cap, d_n, d_st, c->stream);
    if (rc) return rc;
    int64_t nn = 0;
    int st = 0;
    HIPCHK(c, hipMemcpyAsync(&nn, d_n, sizeof nn, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(&st, d_st, sizeof st, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (nn > cap) nn = cap;
    HIPCHK(c, hipMemcpy(out, d_out, sizeof(double) * 2 * nn, hipMemcpyDeviceToHost));
    *n_out = nn;
    *status = st;
    return EIK_OK;
}

// ------------------------------------------------------------------------------ 3D
// Few-layer fp32 volumes (the rover's (x, y, mode) costmaps) on the layered 2D-tile solver:
// layers z0 .. z0+nl-1 of a [H][W][L] volume, one persistent launch.
static int solve_layered(eik_ctx* c, const void* d_cost, void* d_T, int64_t H, int64_t W, int64_t L, int z0, int nl,
                         const int64_t goal[3], int dtype, hipStream_t st) {
    const bool f64 = dtype == EIK_F64;
    const int th = fim2dl_rows(f64);
    eik_fim2d*& slot = f64 ? c->cached_l64 : c->cached_l;
    eik_fim2d* f = slot;
    if (!f || f->H != H || f->W != W) {
        if (f) eik_fim2d_destroy(f);
        slot = nullptr;
        int rc = fim2d_create_rows(c, 1, H, W, dtype, th, &f);
        if (rc) return rc;
        slot = f;
    }
    Fim2dArgs a = f->a;
    a.cost = d_cost;
    a.T = d_T;
    a.ls = L;
    a.z0 = z0;
    a.lzs = 1;
    int64_t nT = H * W * L;  // T's elements (the init's +inf)
    const bool planar = c->layer_planar != 0;
    const size_t esz = f64 ? 8 : 4;
    if (planar) {  // the solve on layer-planar copies (fim2dl.hip layer_planar_in_kernel)
        HIPCHK(c, c->lp_cost.ensure(esz * nl * H * W));
        HIPCHK(c, c->lp_T.ensure(esz * nl * H * W));
        a.cost = c->lp_cost.p;
        a.T = c->lp_T.p;
        a.ls = 1;
        a.z0 = 0;
        a.lzs = H * W;
        nT = (int64_t)nl * H * W;
    }
    a.mode = kModePersistent;
    a.max_rounds = 1;
    a.keep = (float)(1.0 - c->tol);
    a.delta = __builtin_inff();
    a.edge_dirty = nullptr;
    for (auto& g : a.ghost) g = nullptr;
    a.qtimeout = (unsigned long long)(c->qtimeout_s * 1e8);
    // C5 A/B (profiles/r02a_c5_passes.log): 8 / 16 / 24 passes 15.5-16.3 / 13.9 / 12.9 ms
    a.max_passes = c->passes > 0 ? c->passes : 24;
    a.qbudget = c->max_visits ? c->max_visits : 1024ull * (unsigned long long)a.tiles_per_map + (1ull << 20);
    int& res = c->resident_l[f64 ? 1 : 0][nl];
    if (res == 0) res = fim2dl_persist_resident(nl, f64, c->cu_count);
    const int grid = std::min(c->grid > 0 ? c->grid : 4 * c->cu_count, res);
    a.fresh_first = c->fresh_first;
    unsigned err = 0;
    // attempt 1 without bands when attempt 0's band ring overflowed (qerror bit 4, as eik_fim2d_solve)
    for (int attempt = 0; attempt < 2; ++attempt) {
    HIPCHK(c, hipEventRecord(f->ev_start, st));
    HIPCHK(c, hipMemsetAsync((void*)f->a.visits, 0, 3 * sizeof(unsigned long long), st));
    if (planar) HIPCHK(c, layer_planar(d_cost, c->lp_cost.p, f64, H * W, L, z0, nl, true, st));
    // priority bands (fim_engine.hpp), as eik_fim2d_start sets them up: on an explicit EIK_OPT_PRIO
    a.bctl = nullptr;
    const double prio = c->prio < 0 ? default_prio(H, W, 3072.0) : c->prio;
    if (prio > 0 && attempt == 0 && a.capacity < (1 << kBandTagShift) - 1) {
        HIPCHK(c, setup_bands(c, f->bslot, f->bctl, a.capacity, a, st));
        HIPCHK(c, hipMemsetD32Async((hipDeviceptr_t)a.key, 0x7f800000u, (size_t)a.capacity, st));  // keys: +inf
        float* pd = (float*)((char*)f->bctl.p + 128 * kBands);
        HIPCHK(c, fim2d_prio_delta(a.cost, f64, planar ? (int64_t)nl * H * W : H * W * L, (float)prio, pd, st));
        a.pdelta = pd;
        // the dispatch batch: 32 below kWideTiles tiles (C5 16 / 32 / 48 / 64: fp64 3.61 / 3.67-3.69 / 3.65 /
        // 3.58, fp32 6.30-6.33 / 6.37-6.38 / 6.27 / 6.08-6.12 Gcells/s, profiles/r05ak_layered_dispatch_ab.log)
        a.disp = c->prio_dispatch > 0 ? (unsigned)c->prio_dispatch : a.tiles_per_map >= kWideTiles ? 64u : 32u;
    }
    HIPCHK(c, fim2dl_init(a, f64, goal[0], goal[1], goal[2] - z0, nT, st));
    HIPCHK(c, fim2dl_persist(a, nl, f64, grid, st));
    if (planar) HIPCHK(c, layer_planar(c->lp_T.p, d_T, f64, H * W, L, z0, nl, false, st));
    HIPCHK(c, hipEventRecord(f->ev_stop, st));
    HIPCHK(c, hipMemcpyAsync(f->h_q, f->qctl.p, kQueueCtlBytes, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(f->h_visits, (void*)f->a.visits, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    err = f->h_q[192 / 4];
    if (!(err & 4u) || (err & 3u)) break;
    }
    if (err & 1u)
        return set_err(c, EIK_ERR_HIP, "layered solver: a queue wait exceeded %.1f s (EIK_OPT_QTIMEOUT)", c->qtimeout_s);
    if (err & 2u)
        return set_err(c, EIK_ERR_NOCONVERGE, "no convergence within %llu tile visits (negative costs?)",
                       (unsigned long long)a.qbudget);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, f->ev_start, f->ev_stop);
    c->last = eik_stats{};
    c->last.iterations = 1;
    c->last.tile_visits = (int64_t)f->h_visits[0];
    c->last.inplace_passes = (int64_t)f->h_visits[1];
    c->last.fresh_visits = (int64_t)f->h_visits[2];
    c->last.host_syncs = 1;
    c->last.solve_ms = ms;
    // per visit: cost + T read and T write of the tile's nl layers plus the halo ring (a first
    // visit reads no T); per in-place pass: T write + halo
    // (esz: the element size above)
    // (+ the init's T store; planar: + the copies, cost in (L read, nl written) and field out (nl
    // read, L written) per cell, instead of the init's L)
    c->last.bytes_alg = (double)esz * nl *
                            ((double)c->last.tile_visits * (3.0 * kTile * th + 2.0 * (kTile + th)) -
                             (double)c->last.fresh_visits * kTile * th +
                             (double)c->last.inplace_passes * (1.0 * kTile * th + 2.0 * (kTile + th))) +
                        (double)esz * H * W * (planar ? 2.0 * (L + nl) + nl : (double)L);
    return EIK_OK;
}

// Layers [z0, z0 + nl) of a volume the layered solver can take, or nl = 0: L <= kmax layers (fp32 4,
// fp64 3), or L <= kmax + 2 whose first and last layers are entirely +inf (the reference's z padding).
static int layered_plan(eik_ctx* c, const void* d_cost, int64_t H, int64_t W, int64_t L, int dtype, hipStream_t st,
                        int* z0, int* nl) {
    const bool f64 = dtype == EIK_F64;
    const int kmax = f64 ? 3 : 4;
    *z0 = 0;
    *nl = 0;
    if (L <= kmax) {
        *nl = (int)L;
        return EIK_OK;
    }
    if (L > kmax + 2) return EIK_OK;
    HIPCHK(c, c->misc.ensure(64));
    int* d_flag = (int*)c->misc.p;
    int h_flag = 0;
    HIPCHK(c, hipMemsetAsync(d_flag, 0, sizeof(int), st));
    HIPCHK(c, layer_finite(d_cost, f64, H * W, L, 0, d_flag, st));
    HIPCHK(c, layer_finite(d_cost, f64, H * W, L, L - 1, d_flag, st));
    HIPCHK(c, hipMemcpyAsync(&h_flag, d_flag, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    if (h_flag == 0) {
        *z0 = 1;
        *nl = (int)L - 2;
    }
    return EIK_OK;
}

// Persistent driver of the 3D solver (fim3d_persist_kernel): one launch per solve, the tiles of
// all B volumes share one device FIFO (fim_engine.hpp), a visit's face activations queue the
// neighbours into the running launch -- no per-iteration launches or host syncs (the list driver
// took 16-32 launches of ~41 us on the planner's 60 x 60 x 41 end-effector volume).
static int fim3d_solve_persist(eik_ctx* c, Fim3dArgs a, int64_t B, int dtype, const int64_t* goals, hipStream_t st) {
    const int64_t tiles = a.capacity;
    uint64_t nq = 4096;
    while (nq < 8 * (uint64_t)tiles) nq <<= 1;
    HIPCHK(c, c->q3ctl.ensure(kQueueCtlBytes));
    HIPCHK(c, c->q3slot.ensure(sizeof(unsigned) * nq));
    HIPCHK(c, c->q3state.ensure(sizeof(unsigned) * tiles));
    HIPCHK(c, c->q3vis.ensure(3 * sizeof(unsigned long long)));  // visits, (unused) in-place, relaxation passes
    if (!c->h_q3) HIPCHK(c, hipHostMalloc((void**)&c->h_q3, kQueueCtlBytes + 3 * sizeof(unsigned long long)));
    for (hipEvent_t& e : c->e3)
        if (!e) HIPCHK(c, hipEventCreate(&e));
    Fim2dArgs q{};
    q.mode = kModePersistent;
    q.qhead = (unsigned long long*)c->q3ctl.p;
    q.qtail = (unsigned long long*)((char*)c->q3ctl.p + 64);
    q.qactive = (int*)((char*)c->q3ctl.p + 128);
    q.qerror = (unsigned*)((char*)c->q3ctl.p + 192);
    q.qslot = (unsigned*)c->q3slot.p;
    q.qmask = (unsigned)(nq - 1);
    q.qstate = (unsigned*)c->q3state.p;
    q.visits = (unsigned long long*)c->q3vis.p;
    q.qtimeout = (unsigned long long)(c->qtimeout_s * 1e8);
    q.qbudget = c->max_visits ? c->max_visits : 1024ull * (unsigned long long)tiles + (1ull << 20);
    q.fresh_first = 0;
    q.qhold = nullptr;
    a.visits = (unsigned long long*)c->q3vis.p + 2;
    const bool f64 = dtype == EIK_F64;
    int& res = c->resident3[f64 ? 1 : 0];
    if (res == 0) res = fim3d_persist_resident(f64, c->cu_count);
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(std::min(c->grid > 0 ? c->grid : res, res), tiles));
    hipEvent_t e0 = c->e3[0], e1 = c->e3[1];
    HIPCHK(c, hipEventRecord(e0, st));
    HIPCHK(c, hipMemsetAsync(c->q3vis.p, 0, 3 * sizeof(unsigned long long), st));
    HIPCHK(c, c->goals.ensure(sizeof(int64_t) * 3 * B));
    HIPCHK(c, hipMemcpyAsync(c->goals.p, goals, sizeof(int64_t) * 3 * B, hipMemcpyHostToDevice, st));
    HIPCHK(c, fim3d_persist_init(a, q, f64, (const int64_t*)c->goals.p, (int)B, st));
    HIPCHK(c, fim3d_persist(a, q, f64, grid, st));
    HIPCHK(c, hipEventRecord(e1, st));
    unsigned* hq = c->h_q3;
    unsigned long long* hv = (unsigned long long*)((char*)hq + kQueueCtlBytes);
    HIPCHK(c, hipMemcpyAsync(hq, c->q3ctl.p, kQueueCtlBytes, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(hv, c->q3vis.p, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    const unsigned err = hq[192 / 4];
    if (err & 1u)
        return set_err(c, EIK_ERR_HIP, "3D solver: a queue wait exceeded %.1f s (EIK_OPT_QTIMEOUT)", c->qtimeout_s);
    if (err & 2u)
        return set_err(c, EIK_ERR_NOCONVERGE, "3D solve: no convergence within %llu tile visits (negative costs?)",
                       (unsigned long long)q.qbudget);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    c->last = eik_stats{};
    c->last.iterations = 1;
    c->last.host_syncs = 1;
    c->last.tile_visits = (int64_t)hv[0];
    c->last.inplace_passes = (int64_t)hv[2];  // 3D: relaxation passes summed over the visits
    c->last.solve_ms = ms;
    c->last.bytes_alg = (double)hv[0] * (f64 ? 8 : 4) * 3.0 * a.tx * a.ty * a.tz;
    return EIK_OK;
}

// B independent volumes of one shape (list mode; the tiles of all volumes share the lists).
// goals: B x (x, y, z), host memory.
// stop_off >= 0 (B = 1): FastMarching3D.computeTmap's early exit at that cell follows, so cells are
// only lowered to values the early-exit field keeps (Fim3dArgs::stop_off)
static int fim3d_solve_batch(eik_ctx* c, const void* d_cost, void* d_T, int64_t B, int64_t H, int64_t W, int64_t L,
                             int dtype, const int64_t* goals, hipStream_t st, int64_t stop_off = -1) {
    Fim3dArgs a{};
    a.cost = d_cost;
    a.T = d_T;
    a.H = H;
    a.W = W;
    a.L = L;
    a.stop_off = -1;
    if (stop_off >= 0 && B == 1) {
        HIPCHK(c, c->misc.ensure(64));
        HIPCHK(c, max_finite(d_cost, H * W * L, dtype == EIK_F64, (char*)c->misc.p + 32, st));
        a.stop_off = stop_off;
        a.stop_slack = (char*)c->misc.p + 32;
    }
    fim3d_tile_shape(L, &a.tx, &a.ty, &a.tz);
    a.ntx = (int)((W + a.tx - 1) / a.tx);
    a.nty = (int)((H + a.ty - 1) / a.ty);
    a.ntz = (int)((L + a.tz - 1) / a.tz);
    const int64_t tpv = (int64_t)a.ntx * a.nty * a.ntz;
    const int64_t tiles = B * tpv;
    if (tiles >= (1ll << 31) - 8) return set_err(c, EIK_ERR_ARG, "too many 3D tiles");
    a.tpv = (int)tpv;
    a.capacity = (int)tiles;
    a.max_passes = c->passes > 0 ? c->passes : c->max_passes3;
    if (c->mode == kModePersistent && H * W * L * (dtype == EIK_F64 ? 8 : 4) < (int64_t)UINT32_MAX)
        return fim3d_solve_persist(c, a, B, dtype, goals, st);
    HIPCHK(c, c->l3.ensure(sizeof(int) * 3 * tiles));
    HIPCHK(c, c->c3.ensure(sizeof(int) * 64));
    HIPCHK(c, c->m3.ensure(sizeof(unsigned) * tiles));
    HIPCHK(c, c->v3.ensure(sizeof(unsigned long long)));
    a.lists = (int*)c->l3.p;
    a.counts = (int*)c->c3.p;
    a.mark = (unsigned*)c->m3.p;
    a.visits = (unsigned long long*)c->v3.p;
    // pinned words and events live in the context: a solve of a small volume (the planner's
    // end-effector volumes) is ~1 ms, so per-call hipHostMalloc / event creation would show
    if (!c->h3) HIPCHK(c, hipHostMalloc((void**)&c->h3, sizeof(int) * 2 + sizeof(unsigned long long)));
    for (hipEvent_t& e : c->e3)
        if (!e) HIPCHK(c, hipEventCreate(&e));
    hipEvent_t e0 = c->e3[0], e1 = c->e3[1];
    HIPCHK(c, hipEventRecord(e0, st));
    HIPCHK(c, hipMemsetAsync(c->v3.p, 0, sizeof(unsigned long long), st));
    HIPCHK(c, c->goals.ensure(sizeof(int64_t) * 3 * B));
    HIPCHK(c, hipMemcpyAsync(c->goals.p, goals, sizeof(int64_t) * 3 * B, hipMemcpyHostToDevice, st));
    HIPCHK(c, fim3d_init(a, dtype == EIK_F64, (const int64_t*)c->goals.p, (int)B, st));
    int* h = c->h3;
    const int grid = c->grid > 0 ? c->grid : 4 * c->cu_count;
    const int64_t max_iters = 64 * ((int64_t)a.ntx + a.nty + a.ntz) + 8 * tiles + 4096;
    int64_t it = 0;
    int rc = EIK_OK;
    for (;;) {
        for (int k = 0; k < c->sync_every; ++k, ++it) {
            a.iter = (unsigned)it;
            hipError_t e = fim3d_sweep(a, dtype == EIK_F64, grid, st);
            if (e != hipSuccess) { rc = set_err(c, EIK_ERR_HIP, "fim3d_sweep: %s", hipGetErrorString(e)); break; }
        }
        if (rc) break;
        hipError_t e = hipMemcpyAsync(h, (int*)c->c3.p + (it % 3), sizeof(int), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) { rc = set_err(c, EIK_ERR_HIP, "fim3d sync: %s", hipGetErrorString(e)); break; }
        if (h[0] == 0) break;
        if (it >= max_iters) { rc = set_err(c, EIK_ERR_NOCONVERGE, "3D solve did not converge"); break; }
    }
    if (rc == EIK_OK) {
        unsigned long long* hv = (unsigned long long*)(h + 2);
        (void)hipEventRecord(e1, st);
        (void)hipMemcpyAsync(hv, c->v3.p, sizeof(unsigned long long), hipMemcpyDeviceToHost, st);
        (void)hipStreamSynchronize(st);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        c->last = eik_stats{};
        c->last.iterations = it;
        c->last.tile_visits = (int64_t)*hv;
        c->last.solve_ms = ms;
        c->last.bytes_alg = (double)*hv * (dtype == EIK_F64 ? 8 : 4) * 3.0 * a.tx * a.ty * a.tz;
    }
    return rc;
}

static int fim3d_solve_one(eik_ctx* c, const void* d_cost, void* d_T, int64_t H, int64_t W, int64_t L, int dtype,
                           const int64_t goal[3], hipStream_t st, int64_t stop_off);

int eik_fim3d_solve(eik_ctx* c, const void* d_cost, void* d_T, int64_t H, int64_t W, int64_t L, int dtype,
                    const int64_t goal[3], void* stream) {
    return fim3d_solve_one(c, d_cost, d_T, H, W, L, dtype, goal, (hipStream_t)stream, -1);
}

// one volume; stop_off >= 0: the caller applies the early exit at that cell afterwards
static int fim3d_solve_one(eik_ctx* c, const void* d_cost, void* d_T, int64_t H, int64_t W, int64_t L, int dtype,
                           const int64_t goal[3], hipStream_t st, int64_t stop_off) {
    if (!c || !d_cost || !d_T || !goal || H < 1 || W < 1 || L < 1)
        return c ? set_err(c, EIK_ERR_ARG, "bad 3D arguments") : EIK_ERR_ARG;
    if (goal[0] < 0 || goal[1] < 0 || goal[2] < 0 || goal[0] >= W || goal[1] >= H || goal[2] >= L)
        return set_err(c, EIK_ERR_ARG, "goal (%ld,%ld,%ld) outside %ldx%ldx%ld", (long)goal[0], (long)goal[1],
                       (long)goal[2], (long)H, (long)W, (long)L);
    HIPCHK(c, hipSetDevice(c->device));
    // few-layer volumes (the rover's (x, y, mode) costmaps, C5): the layered solver, fp32 and fp64
    const int64_t esz = dtype == EIK_F64 ? 8 : 4;
    // (an fp64 early-exit solve stays on fim3d.hip: its solve3_ref keeps the reference's exact ties,
    // which decide FM3D's closed set)
    // (the layered kernel addresses T per tile and layer: (rows + 2) x W x L elements under 4 GiB)
    if (c->mode == kModePersistent && c->max_rounds == 1 &&
        (fim2dl_rows(dtype == EIK_F64) + 2) * W * L * esz < (int64_t)UINT32_MAX && !(stop_off >= 0 && dtype == EIK_F64)) {
        int z0 = 0, nl = 0;
        int rc = layered_plan(c, d_cost, H, W, L, dtype, st, &z0, &nl);
        if (rc) return rc;
        if (nl > 0 && goal[2] >= z0 && goal[2] < z0 + nl) {
            return solve_layered(c, d_cost, d_T, H, W, L, z0, nl, goal, dtype, st);
        }
    }
    return fim3d_solve_batch(c, d_cost, d_T, 1, H, W, L, dtype, goal, st, stop_off);
}

}  // extern "C"

// Linear index of `start` for the early exit of FastMarching3D.computeTmap (:141), or -1 when the
// reference never pops it: start == goal (the goal is closed without a pop, :132-134) or outside
// the volume.  A start on +inf cost is never popped either; the kernel sees T[start] = +inf then.
static int64_t early_offset(const int64_t goal[3], const int64_t start[3], int64_t H, int64_t W, int64_t L) {
    if (!start) return -1;
    if (start[0] < 0 || start[1] < 0 || start[2] < 0 || start[0] >= W || start[1] >= H || start[2] >= L) return -1;
    if (start[0] == goal[0] && start[1] == goal[1] && start[2] == goal[2]) return -1;
    return (start[1] * W + start[0]) * L + start[2];
}

template <typename R>
static int tmap3d_host(eik_ctx* c, const R* cost, int64_t H, int64_t W, int64_t L, const int64_t goal[3],
                       const int64_t* start, R* T) {
    if (!c || !cost || !T || !goal) return c ? set_err(c, EIK_ERR_ARG, "NULL argument") : EIK_ERR_ARG;
    const int64_t n = H * W * L;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, c->cost.ensure(sizeof(R) * n));
    HIPCHK(c, c->T.ensure(sizeof(R) * n));
    HIPCHK(c, host_to_dev(c, c->cost.p, cost, sizeof(R) * n, c->stream));
    int rc = check_cost(c, cost, c->cost.p, n, c->stream);
    if (rc) return rc;
    const int dt = sizeof(R) == 8 ? EIK_F64 : EIK_F32;
    rc = fim3d_solve_one(c, c->cost.p, c->T.p, H, W, L, dt, goal, c->stream, early_offset(goal, start, H, W, L));
    if (rc) return rc;
    const void* src = c->T.p;
    if (start) {
        HIPCHK(c, c->T2.ensure(sizeof(R) * n));
        rc = eik_fim3d_early_exit(c, c->cost.p, c->T.p, c->T2.p, H, W, L, dt, goal, start, c->stream);
        if (rc) return rc;
        src = c->T2.p;
    }
    HIPCHK(c, dev_to_host(c, T, src, sizeof(R) * n, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return EIK_OK;
}

extern "C" {

int eik_fim3d_early_exit(eik_ctx* c, const void* d_cost, const void* d_T, void* d_Te, int64_t H, int64_t W, int64_t L,
                         int dtype, const int64_t goal[3], const int64_t start[3], void* stream) {
    if (!c || !d_cost || !d_T || !d_Te || !goal || !start || H < 1 || W < 1 || L < 1 || d_T == d_Te)
        return c ? set_err(c, EIK_ERR_ARG, "bad early-exit arguments") : EIK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t ts_off = early_offset(goal, start, H, W, L);
    for (auto& v : c->exact_info) v = 0;
    if (c->exact_band && dtype == EIK_F64 && ts_off >= 0) {
        // the reference's own band values and LIFO ties (bidir_exact.hip fm3d_exact)
        const int64_t n = H * W * L;
        if (n >= (1ll << 29)) return set_err(c, EIK_ERR_ARG, "exact band replay: volumes of < 2^29 cells");
        HIPCHK(c, c->exact.ensure(fm3d_exact_work_bytes(n)));
        hipStream_t st = (hipStream_t)stream;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        HIPCHK(c, hipEventCreate(&e0));
        HIPCHK(c, hipEventCreate(&e1));
        HIPCHK(c, hipEventRecord(e0, st));
        unsigned long long info[4] = {0, 0, 0, 0};
        const int64_t goal_off = (goal[1] * W + goal[0]) * L + goal[2];
        const hipError_t e = fm3d_exact(static_cast<const double*>(d_cost), static_cast<const double*>(d_T),
                                        static_cast<double*>(d_Te), H, W, L, goal_off, ts_off, c->exact.p,
                                        c->exact.bytes, st, info);
        if (e == hipErrorNotReady || e == hipErrorNotSupported) {
            (void)hipEventDestroy(e0);
            (void)hipEventDestroy(e1);
            return set_err(c, EIK_ERR_NOCONVERGE, e == hipErrorNotReady
                                                      ? "FM3D early exit: the exact band replay did not settle"
                                                      : "FM3D early exit: the exact band replay met a run of more "
                                                        "than 4096 cells of exactly equal T (a zero-cost region)");
        }
        HIPCHK(c, e);
        HIPCHK(c, hipEventRecord(e1, st));
        HIPCHK(c, hipEventSynchronize(e1));
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        for (int q = 0; q < 4; ++q) c->exact_info[q] = info[q];
        c->exact_info[4] = (unsigned long long)(ms * 1000.0f);
        return EIK_OK;
    }
    HIPCHK(c, fim3d_early(d_cost, d_T, d_Te, H, W, L, ts_off, dtype == EIK_F64, (hipStream_t)stream));
    return EIK_OK;
}

int eik_tmap3d_f32(eik_ctx* c, const float* cost, int64_t H, int64_t W, int64_t L, const int64_t goal[3], float* T) {
    return tmap3d_host<float>(c, cost, H, W, L, goal, nullptr, T);
}

int eik_tmap3d_f64(eik_ctx* c, const double* cost, int64_t H, int64_t W, int64_t L, const int64_t goal[3],
                   double* T) {
    return tmap3d_host<double>(c, cost, H, W, L, goal, nullptr, T);
}

int eik_tmap3d_early_f32(eik_ctx* c, const float* cost, int64_t H, int64_t W, int64_t L, const int64_t goal[3],
                         const int64_t start[3], float* T) {
    if (!start) return c ? set_err(c, EIK_ERR_ARG, "NULL start") : EIK_ERR_ARG;
    return tmap3d_host<float>(c, cost, H, W, L, goal, start, T);
}

int eik_tmap3d_early_f64(eik_ctx* c, const double* cost, int64_t H, int64_t W, int64_t L, const int64_t goal[3],
                         const int64_t start[3], double* T) {
    if (!start) return c ? set_err(c, EIK_ERR_ARG, "NULL start") : EIK_ERR_ARG;
    return tmap3d_host<double>(c, cost, H, W, L, goal, start, T);
}

int eik_path3d_dev(eik_ctx* c, const void* d_T, int dtype, int64_t H, int64_t W, int64_t L, const double init[3],
                   const double end[3], double tau, double* d_out, int64_t cap, int64_t* d_n_out, int* d_status,
                   void* stream) {
    if (!c || !d_T || !init || !end || !d_out || !d_n_out || !d_status || cap < 2 || !(tau > 0) || H < 1 || W < 1 ||
        L < 1)
        return c ? set_err(c, EIK_ERR_ARG, "bad 3D path arguments") : EIK_ERR_ARG;
    Gdm3dArgs a;
    a.T = d_T;
    a.H = H;
    a.W = W;
    a.L = L;
    for (int i = 0; i < 3; ++i) {
        a.init[i] = init[i];
        a.end[i] = end[i];
    }
    a.tau = tau;
    a.steps = (long)std::nearbyint(15000.0 / tau);  // int(round(15000/tau)), FastMarching3D.py:207
    a.out = d_out;
    a.cap = cap;
    a.n_out = d_n_out;
    a.status = d_status;
    HIPCHK(c, gdm3d(a, dtype == EIK_F64, (hipStream_t)stream));
    return EIK_OK;
}

int eik_path3d_f64(eik_ctx* c, const double* T, int64_t H, int64_t W, int64_t L, const double init[3],
                   const double end[3], double tau, double* out, int64_t cap, int64_t* n_out, int* status) {
    if (!c || !T || !out || !n_out || !status) return c ? set_err(c, EIK_ERR_ARG, "NULL argument") : EIK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t n = H * W * L;
    HIPCHK(c, c->T2.ensure(sizeof(double) * n));
    HIPCHK(c, c->work.ensure(sizeof(double) * 3 * cap + 64));
    HIPCHK(c, host_to_dev(c, c->T2.p, T, sizeof(double) * n, c->stream));
    double* d_out = (double*)c->work.p;
    int64_t* d_n = (int64_t*)(d_out + 3 * cap);
    int* d_st = (int*)(d_n + 1);
    int rc = eik_path3d_dev(c, c->T2.p, EIK_F64, H, W, L, init, end, tau, d_out, cap, d_n, d_st, c->stream);
    if (rc) return rc;
    int64_t nn = 0;
    int st = 0;
    HIPCHK(c, hipMemcpyAsync(&nn, d_n, sizeof nn, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(&st, d_st, sizeof st, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (nn > cap) nn = cap;
    HIPCHK(c, hipMemcpy(out, d_out, sizeof(double) * 3 * nn, hipMemcpyDeviceToHost));
    *n_out = nn;
    *status = st;
    return EIK_OK;
}

int eik_gradient2d_f64(eik_ctx* c, const double* T, int64_t H, int64_t W, double* gnx, double* gny) {
    if (!c || !T || !gnx || !gny || H < 2 || W < 2) return c ? set_err(c, EIK_ERR_ARG, "bad arguments") : EIK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t n = H * W;
    HIPCHK(c, c->T2.ensure(sizeof(double) * n));
    HIPCHK(c, c->work.ensure(sizeof(double) * 2 * n));
    HIPCHK(c, host_to_dev(c, c->T2.p, T, sizeof(double) * n, c->stream));
    double* gx = (double*)c->work.p;
    HIPCHK(c, gradient2d((const double*)c->T2.p, H, W, gx, gx + n, c->stream));
    HIPCHK(c, dev_to_host(c, gnx, gx, sizeof(double) * n, c->stream));
    HIPCHK(c, dev_to_host(c, gny, gx + n, sizeof(double) * n, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return EIK_OK;
}

}  // extern "C"

// ------------------------------------------------------------------ cost-raster builder
// image_filling (:82-94) of the device mask m in place: the pixels equal to m[0] that the
// 4-connected flood fill from (0, 0) reaches.  Default: connected components (cm_fill_ccl,
// union-find); EIK_FILL_FIM=1 in the build: reachability by the block-FIM solver on cost 0 / +inf.
#ifndef EIK_FILL_FIM
#define EIK_FILL_FIM 0
#endif
static int cm_fill(eik_ctx* c, unsigned char* m, int64_t H, int64_t W, float* fcost, float* fT, hipStream_t st) {
#if EIK_FILL_FIM
    eik_fim2d* f = c->cached_fill;
    if (!f || f->H != H || f->W != W) {
        if (f) eik_fim2d_destroy(f);
        c->cached_fill = nullptr;
        int rc = eik_fim2d_create(c, 1, H, W, EIK_F32, &f);
        if (rc) return rc;
        c->cached_fill = f;
    }
    HIPCHK(c, cm_fill_cost(m, H * W, fcost, st));
    const int64_t goal[2] = {0, 0};
    const eik_stats keep = c->last;  // the builder's internal solves do not count as the caller's
    int rc = eik_fim2d_solve(f, fcost, fT, goal, st);
    c->last = keep;
    if (rc) return rc;
    HIPCHK(c, cm_fill_apply(m, fT, H * W, st));
#else
    // the two f32 scratch planes serve as the int32 lroot / parent arrays
    HIPCHK(c, cm_fill_ccl(m, H, W, reinterpret_cast<int*>(fcost), reinterpret_cast<int*>(fT), st));
#endif
    return EIK_OK;
}

extern "C" {

int eik_costmap_dev(eik_ctx* c, const double* d_Z, int64_t H, int64_t W, double res, double size,
                    const eik_costmap_params* params, double* d_cost, uint8_t* d_obst, void* stream) {
    if (!c || !d_Z || !d_cost || H < 3 || W < 3 || !(res > 0) || !(size > 0))
        return c ? set_err(c, EIK_ERR_ARG, "bad cost-map arguments") : EIK_ERR_ARG;
    const eik_costmap_params p = params ? *params : eik_costmap_params{0.20, 0.9, 1.0, 10.0, 300.0};
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t st = (hipStream_t)stream;
    const int64_t n = H * W;
    // scratch: 3 masks, 3 int planes (column distances, squared EDT, envelope apexes), 2 f32 (fill
    // cost, fill T), 2 f64 planes, reduction words
    HIPCHK(c, c->cm_u8.ensure(3 * n + 64));
    HIPCHK(c, c->cm_i32.ensure(sizeof(int) * 3 * n));
    HIPCHK(c, c->cm_f32.ensure(sizeof(float) * 2 * n));
    HIPCHK(c, c->cm_f64.ensure(sizeof(double) * 2 * n + 64));
    unsigned char* obst = d_obst ? d_obst : (unsigned char*)c->cm_u8.p;
    unsigned char* tmp = (unsigned char*)c->cm_u8.p + n;
    unsigned char* dil = (unsigned char*)c->cm_u8.p + 2 * n;
    int* g = (int*)c->cm_i32.p;
    int* D = g + n;
    int* vbuf = g + 2 * n;
    float* fcost = (float*)c->cm_f32.p;
    float* fT = fcost + n;
    double* work = (double*)c->cm_f64.p;
    double* tmpd = work + n;
    unsigned long long* red = (unsigned long long*)(tmpd + n);
    const int r1 = 10;                                              // :1167
    const int r2 = (int)std::nearbyint((p.diagonal / 2) / res);     // :1172-1173
    const int r3 = (int)std::nearbyint(p.expansion / res);          // :1190-1191
    HIPCHK(c, cm_normals(d_Z, H, W, size, red, p.slope_max, obst, nullptr, nullptr, nullptr, st));  // :1104-1160
    // min(Z)'s key (red is reused below) for the rover path's z lookup (:1101, :1246): misc word 5
    HIPCHK(c, c->misc.ensure(64));
    HIPCHK(c, hipMemcpyAsync((unsigned long long*)c->misc.p + 5, red, sizeof(unsigned long long),
                             hipMemcpyDeviceToDevice, st));
    int rc = cm_fill(c, obst, H, W, fcost, fT, st);                 // :1163-1164
    if (rc) return rc;
    HIPCHK(c, cm_morph(obst, H, W, r1, true, tmp, g, D, vbuf, st));  // :1168
    HIPCHK(c, cm_morph(tmp, H, W, r1, false, obst, g, D, vbuf, st)); // :1169
    HIPCHK(c, cm_morph(obst, H, W, r2, false, tmp, g, D, vbuf, st)); // :1175
    rc = cm_fill(c, tmp, H, W, fcost, fT, st);                      // :1176
    if (rc) return rc;
    HIPCHK(c, cm_morph(tmp, H, W, r2, true, obst, g, D, vbuf, st));  // :1177
    HIPCHK(c, cm_border(obst, H, W, 1, st));                         // :1180-1184
    HIPCHK(c, cm_morph(obst, H, W, r3, false, dil, g, D, vbuf, st)); // :1192
    HIPCHK(c, cm_edt_ramp(obst, H, W, r3, g, D, vbuf, st));          // :1194 (distance to obstacles, as :1196 uses it)
    HIPCHK(c, cm_cost(obst, dil, D, H, W, res, p.high, p.gradient, work, tmpd, d_cost, red, st));  // :1187-1216
    return EIK_OK;
}

int eik_costmap_f64(eik_ctx* c, const double* Z, int64_t H, int64_t W, double res, double size,
                    const eik_costmap_params* params, double* cost_out, uint8_t* obst_out) {
    if (!c || !Z || !cost_out) return c ? set_err(c, EIK_ERR_ARG, "NULL argument") : EIK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t n = H * W;
    HIPCHK(c, c->T2.ensure(sizeof(double) * 2 * n + n));
    double* dZ = (double*)c->T2.p;
    double* dC = dZ + n;
    uint8_t* dO = (uint8_t*)(dC + n);
    HIPCHK(c, host_to_dev(c, dZ, Z, sizeof(double) * n, c->stream));
    int rc = eik_costmap_dev(c, dZ, H, W, res, size, params, dC, dO, c->stream);
    if (rc) return rc;
    HIPCHK(c, dev_to_host(c, cost_out, dC, sizeof(double) * n, c->stream));
    if (obst_out) HIPCHK(c, dev_to_host(c, obst_out, dO, n, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return EIK_OK;
}

int eik_surface_normal_f64(eik_ctx* c, const double* Z, int64_t H, int64_t W, double size, double* Nx, double* Ny,
                           double* Nz) {
    if (!c || !Z || !Nx || !Ny || !Nz || H < 3 || W < 3 || !(size > 0))
        return c ? set_err(c, EIK_ERR_ARG, "bad surface_normal arguments") : EIK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t n = H * W;
    HIPCHK(c, c->T2.ensure(sizeof(double) * 4 * n + 64));
    double* dZ = (double*)c->T2.p;
    unsigned long long* red = (unsigned long long*)(dZ + 4 * n);
    HIPCHK(c, host_to_dev(c, dZ, Z, sizeof(double) * n, c->stream));
    HIPCHK(c, cm_normals(dZ, H, W, size, red, 0.0, nullptr, dZ + n, dZ + 2 * n, dZ + 3 * n, c->stream));
    HIPCHK(c, dev_to_host(c, Nx, dZ + n, sizeof(double) * n, c->stream));
    HIPCHK(c, dev_to_host(c, Ny, dZ + 2 * n, sizeof(double) * n, c->stream));
    HIPCHK(c, dev_to_host(c, Nz, dZ + 3 * n, sizeof(double) * n, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return EIK_OK;
}

int eik_image_fill_u8(eik_ctx* c, const uint8_t* im, int64_t H, int64_t W, uint8_t* out) {
    if (!c || !im || !out || H < 1 || W < 1) return c ? set_err(c, EIK_ERR_ARG, "bad image_filling arguments") : EIK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t n = H * W;
    HIPCHK(c, c->cm_u8.ensure(3 * n + 64));
    HIPCHK(c, c->cm_f32.ensure(sizeof(float) * 2 * n));
    unsigned char* m = (unsigned char*)c->cm_u8.p;
    HIPCHK(c, host_to_dev(c, m, im, n, c->stream));
    float* fcost = (float*)c->cm_f32.p;
    int rc = cm_fill(c, m, H, W, fcost, fcost + n, c->stream);
    if (rc) return rc;
    HIPCHK(c, dev_to_host(c, out, m, n, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return EIK_OK;
}

int eik_disk_morph_u8(eik_ctx* c, const uint8_t* im, int64_t H, int64_t W, int radius, int erode, uint8_t* out) {
    if (!c || !im || !out || H < 1 || W < 1 || radius < 0)
        return c ? set_err(c, EIK_ERR_ARG, "bad disk morphology arguments") : EIK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t n = H * W;
    HIPCHK(c, c->cm_u8.ensure(3 * n + 64));
    HIPCHK(c, c->cm_i32.ensure(sizeof(int) * 3 * n));
    unsigned char* a = (unsigned char*)c->cm_u8.p;
    unsigned char* o = a + n;
    int* g = (int*)c->cm_i32.p;
    HIPCHK(c, host_to_dev(c, a, im, n, c->stream));
    HIPCHK(c, cm_morph(a, H, W, radius, erode != 0, o, g, g + n, g + 2 * n, c->stream));
    HIPCHK(c, dev_to_host(c, out, o, n, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return EIK_OK;
}

// ------------------------------------------------------- rover path (planner step 1, :1097-1258)
int eik_rover_path_f64(eik_ctx* c, const double* Z, int64_t H, int64_t W, const eik_rover_query* q,
                       const eik_costmap_params* params, double* path_xyz, double* heading, int64_t cap,
                       int64_t* n_out, uint32_t join[2], double* cost_out) {
    if (!c || !Z || !q || !path_xyz || !heading || !n_out || H < 3 || W < 3 || !(q->resolution > 0) ||
        !(q->size > 0) || !(q->tau > 0))
        return c ? set_err(c, EIK_ERR_ARG, "bad rover-path arguments") : EIK_ERR_ARG;
    const int64_t n = H * W;
    if (n >= (1ll << 29)) return set_err(c, EIK_ERR_ARG, "bidirectional join supports < 2^29 cells");
    // nodes: int(round(v / res - 1)), Python's round = half to even   :1107-1117
    const double res = q->resolution;
    const int64_t g[4] = {(int64_t)std::nearbyint(q->xm / res - 1), (int64_t)std::nearbyint(q->ym / res - 1),
                          (int64_t)std::nearbyint(q->xr / res - 1), (int64_t)std::nearbyint(q->yr / res - 1)};
    for (int k = 0; k < 2; ++k)
        if (g[2 * k] < 0 || g[2 * k + 1] < 0 || g[2 * k] >= W || g[2 * k + 1] >= H)
            return set_err(c, EIK_ERR_ARG, "%s node (%ld, %ld) outside the %ldx%ld DEM", k ? "rover" : "sample",
                           (long)g[2 * k], (long)g[2 * k + 1], (long)H, (long)W);
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t st = c->stream;
    const int64_t steps = (int64_t)std::nearbyint(15000.0 / q->tau);  // FastMarching.py:173
    const int64_t pcap = steps + 4;
    const size_t pbytes = sizeof(double) * 2 * 2 * pcap + 64;
    HIPCHK(c, c->T2.ensure(std::max(sizeof(double) * n, pbytes)));  // Z, then (Z consumed) the paths
    HIPCHK(c, c->cost.ensure(sizeof(double) * 2 * n));
    HIPCHK(c, c->T.ensure(sizeof(double) * 2 * n));
    double* dZ = (double*)c->T2.p;
    double* dcost = (double*)c->cost.p;
    double* dT = (double*)c->T.p;
    // EIK_ROVER_PHASES=1 (diagnostics): synchronise after each phase and print its wall time
    static const bool phases = getenv("EIK_ROVER_PHASES") != nullptr;
    auto tp = std::chrono::steady_clock::now();
    auto phase = [&](const char* name) {
        if (!phases) return;
        (void)hipStreamSynchronize(st);
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[rover] %-10s %8.3f ms\n", name, std::chrono::duration<double, std::milli>(now - tp).count());
        tp = now;
    };
    phase("setup");
    HIPCHK(c, host_to_dev(c, dZ, Z, sizeof(double) * n, st));
    phase("dem_h2d");
    int rc = eik_costmap_dev(c, dZ, H, W, res, q->size, params, dcost, nullptr, st);  // :1101-1216
    if (rc) return rc;
    phase("costmap");
    // biComputeTmap(cMap.T, goal = sample node, start = rover node)   :1222; both fronts, one batch
    HIPCHK(c, hipMemcpyAsync(dcost + n, dcost, sizeof(double) * n, hipMemcpyDeviceToDevice, st));
    if (cost_out) HIPCHK(c, dev_to_host(c, cost_out, dcost, sizeof(double) * n, st));
    eik_fim2d* f = nullptr;
    rc = get_solver(c, 2, H, W, EIK_F64, &f);
    if (rc) return rc;
    unsigned long long best = 0;
    rc = solve_fronts(c, f, dcost, dT, g, H, W, &best);  // :114-162
    if (rc) return rc;
    phase("fronts");
    if (best == ~0ull) return set_err(c, EIK_ERR_UNREACHABLE, "the rover cannot reach the sample");
    const int64_t node = (int64_t)(best & ((1ull << 29) - 1));
    const double jn[2] = {(double)(node % W), (double)(node / W)};
    if (join) {
        join[0] = (uint32_t)(node % W);
        join[1] = (uint32_t)(node / W);
    }
    // pathG = getPathGDM(TmapG, nodeJoin, goal, tau), pathS = getPathGDM(TmapS, nodeJoin, start, tau)   :1225-1226
    double* dP = (double*)c->T2.p;  // [pathG | pathS], then n_out[2], status[2]
    int64_t* dn = (int64_t*)(dP + 2 * 2 * pcap);
    int* dst = (int*)(dn + 2);
    const double eg[2] = {(double)g[0], (double)g[1]}, es[2] = {(double)g[2], (double)g[3]};
    // the two walks are independent one-workgroup kernels: pathS runs on a second stream beside
    // pathG (each walk is one dependent chain of steps, ~0.4 us each)
    if (!c->stream2) HIPCHK(c, hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking));
    if (!c->ev_fork) HIPCHK(c, hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
    if (!c->ev_join) HIPCHK(c, hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
    HIPCHK(c, hipEventRecord(c->ev_fork, st));
    HIPCHK(c, hipStreamWaitEvent(c->stream2, c->ev_fork, 0));
    rc = eik_path2d_dev(c, dT, EIK_F64, H, W, jn, eg, q->tau, dP, pcap, dn, dst, st);
    if (rc) return rc;
    rc = eik_path2d_dev(c, dT + n, EIK_F64, H, W, jn, es, q->tau, dP + 2 * pcap, pcap, dn + 1, dst + 1, c->stream2);
    if (rc) return rc;
    HIPCHK(c, hipEventRecord(c->ev_join, c->stream2));
    HIPCHK(c, hipStreamWaitEvent(st, c->ev_join, 0));
    phase("walks");
    int64_t hn[2];
    int hs[2];
    unsigned long long zkey = 0;
    HIPCHK(c, hipMemcpyAsync(hn, dn, sizeof hn, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(hs, dst, sizeof hs, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(&zkey, (unsigned long long*)c->misc.p + 5, sizeof zkey, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    if (hs[0] == EIK_PATH_ERROR || hs[1] == EIK_PATH_ERROR)
        return set_err(c, EIK_ERR_ARG, "getPathGDM failed (the reference raises): NaN point or out of range");
    std::vector<double> pg((size_t)(2 * hn[0])), ps((size_t)(2 * hn[1]));
    HIPCHK(c, hipMemcpyAsync(pg.data(), dP, sizeof(double) * 2 * hn[0], hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(ps.data(), dP + 2 * pcap, sizeof(double) * 2 * hn[1], hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    phase("paths_d2h");
    // the cost builder's min(Z), from its order-preserving key (costmap.hip dkey)
    const unsigned long long zb = (zkey >> 63) ? (zkey & ~(1ull << 63)) : ~zkey;
    double zmin;
    memcpy(&zmin, &zb, sizeof zmin);
    rc = rover_assemble(ps.data(), hn[1], pg.data(), hn[0], Z, H, W, q, path_xyz, heading, cap, n_out, zmin);
    phase("assemble");
    if (rc) return set_err(c, rc, *n_out > cap ? "path buffer too small (%ld rows needed)" : "waypoint outside the DEM",
                           (long)*n_out);
    return EIK_OK;
}

}  // extern "C"

// ------------------------------------------- end-effector cost volume (planner step 3, :1462-1593)
namespace {

// The host side of arm.hip: the tables TunnelCost forms in Python floats (:515-519, :527-546,
// :571-590, :621-631, :655-668, :683-703), in the reference's evaluation order.
struct ArmTables {
    std::vector<double> buf;  // toaA | toaB | toaC | I | K | norm | valA | ct | st | cs | ss | ks | valC
    size_t oA = 0, oB = 0, oC = 0, oI = 0, oK = 0, oN = 0, oV = 0, oct = 0, ost = 0, ocs = 0, oss = 0, oks = 0, ovc = 0;
    int nX = 0, nZ = 0, nK = 0;
    double rad = 0;
};

void np_linspace(double a, double b, int64_t n, double* out) {
#pragma clang fp contract(off)
    if (n == 1) {
        out[0] = a;
        return;
    }
    const double div = (double)(n - 1), delta = b - a, step = delta / div;
    for (int64_t i = 0; i < n; ++i) out[i] = step == 0 ? ((double)i / div) * delta + a : (double)i * step + a;
    out[n - 1] = b;
}

void arm_toa(const double* h, const double* p, double yaw_off, double* t) {
#pragma clang fp contract(off)
    const double alpha = h[2] - yaw_off, beta = h[1], gamma = h[0];
    const double ca = std::cos(alpha), cb = std::cos(beta), cg = std::cos(gamma);
    const double sa = std::sin(alpha), sb = std::sin(beta), sg = std::sin(gamma);
    const double r[12] = {ca * cb, ca * sb * sg - sa * cg, ca * sb * cg + sa * sg, p[0],
                          sa * cb, sa * sb * sg + ca * cg, sa * sb * cg - ca * sg, p[1],
                          -sb,     cb * sg,                cb * cg,                p[2]};
    for (int i = 0; i < 12; ++i) t[i] = r[i];
}

void arm_tables(const double* gamma2D, const double* heading, int64_t npts, const eik_arm_volume& v, ArmTables& T) {
#pragma clang fp contract(off)
    const double gradient = 15.0;                                              // :512
    const double tunnelRad = v.rlim + 2 * v.resX;                              // :515
    T.nX = (int)(std::nearbyint(2 * tunnelRad / v.resX) + 1);                  // :516
    T.nZ = (int)(std::nearbyint(2 * tunnelRad / v.resZ) + 1);                  // :517
    T.nK = (int)std::nearbyint(T.nZ / 2.0) + 1;                                // :671
    T.rad = v.rlim + 2 * v.resZ;                                               // :688-690
    const size_t nik = (size_t)T.nX * T.nZ;
    size_t o = 0;
    T.oA = o; o += 12 * (size_t)npts;
    T.oB = o; o += 12;
    T.oC = o; o += 12;
    T.oI = o; o += T.nX;
    T.oK = o; o += T.nZ;
    T.oN = o; o += nik;
    T.oV = o; o += nik;
    T.oct = o; o += 100;
    T.ost = o; o += 100;
    T.ocs = o; o += 90;
    T.oss = o; o += 90;
    T.oks = o; o += T.nK;
    T.ovc = o; o += T.nK;
    T.buf.assign(o, 0.0);
    double* b = T.buf.data();
    const double half_pi = 3.141592653589793 / 2;  // math.pi / 2
    for (int64_t j = 0; j < npts; ++j) arm_toa(heading + 3 * j, gamma2D + 3 * j, half_pi, b + T.oA + 12 * j);
    arm_toa(heading, gamma2D, half_pi, b + T.oB);                                          // :617-631
    arm_toa(heading + 3 * (npts - 1), gamma2D + 3 * (npts - 1), 0.0, b + T.oC);            // :655-668
    np_linspace(-tunnelRad, tunnelRad, T.nX, b + T.oI);                                     // :563
    np_linspace(-tunnelRad, tunnelRad, T.nZ, b + T.oK);                                     // :564
    const double c = (v.rO + v.rm) / 2;
    for (int i = 0; i < T.nX; ++i)
        for (int k = 0; k < T.nZ; ++k) {
            const double I = b[T.oI + i], K = b[T.oK + k];
            const double i2 = I * I, k2 = K * K;
            const double norm = std::sqrt(i2 + k2);                                         // :578
            const double d = norm - c;
            const double t1 = gradient * (d * d) + 2;
            const double u = ((I + v.rlim) + 2 * v.resZ);
            b[T.oN + (size_t)i * T.nZ + k] = norm;
            b[T.oV + (size_t)i * T.nZ + k] = t1 + 4 * u;                                   // :590
        }
    for (int ti = 0; ti < 100; ++ti) {                                                      // :674-676
        const double theta = 3.141592653589793 * (-100 + 2 * ti) / 180;
        b[T.oct + ti] = std::cos(theta);
        b[T.ost + ti] = std::sin(theta);
    }
    for (int si = 0; si < 90; ++si) {                                                       // :679-681
        const double sigma = 3.141592653589793 * (-90 + 2 * si) / 180;
        b[T.ocs + si] = std::cos(sigma);
        b[T.oss + si] = std::sin(sigma);
    }
    np_linspace(0.0, tunnelRad, T.nK, b + T.oks);                                           // :684
    for (int k = 0; k < T.nK; ++k) {
        const double d = b[T.oks + k] - c;
        b[T.ovc + k] = gradient * (d * d) + 2;                                              // :703
    }
}

}  // namespace

// Build the volume on the device into d_cost (fmap * tunnel) and/or return the pieces.  d_fmap:
// GetObstMap's finalMap (computed here when d_Z != nullptr); d_tunnel: TunnelCost's map.
static int arm_volume_dev(eik_ctx* c, const double* d_Z, const double* d_obst, int64_t m, int64_t n,
                          const double* gamma2D, const double* heading, int64_t npts, const eik_arm_volume* v,
                          double* d_fmap, double* d_omap, double* d_gmap, double* d_tunnel, double* d_cost,
                          hipStream_t st) {
    const int64_t nc = v->sX * v->sY * v->sZ;
    if (d_Z) {
        HIPCHK(c, c->misc.ensure(64));
        HIPCHK(c, hipMemsetAsync(c->misc.p, 0, sizeof(unsigned), st));
        HIPCHK(c, arm_obst_map(d_Z, d_obst, m, n, v->resX, v->resY, v->resZ, v->sX, v->sY, v->sZ, v->xm, v->ym, d_fmap,
                               d_omap, d_gmap, (unsigned*)c->misc.p, st));
    }
    if (!d_tunnel) return EIK_OK;
    ArmTables T;
    arm_tables(gamma2D, heading, npts, *v, T);
    ArmArgs a{};
    a.sX = v->sX;
    a.sY = v->sY;
    a.sZ = v->sZ;
    a.resX = v->resX;
    a.resY = v->resY;
    a.resZ = v->resZ;
    a.rlim = v->rlim;
    a.rad = T.rad;
    a.nX = T.nX;
    a.nZ = T.nZ;
    a.nK = T.nK;
    a.nA = 2ull * (unsigned long long)npts * T.nX * T.nZ;
    a.nB = (unsigned long long)T.nX * T.nZ;
    a.nC = 100ull * 90ull * (unsigned long long)(T.nK + 1);
    if (a.nA + a.nB + a.nC >= 0xffffffffull) return set_err(c, EIK_ERR_ARG, "too many tunnel events");
    for (int k = 0; k < 3; ++k) {
        a.fw[k] = v->final_wp[k];
        a.iw[k] = v->initial_wp[k];
    }
    // scratch: tables | first (u32) | closed (u8)
    const size_t tb = sizeof(double) * T.buf.size();
    const size_t need = tb + sizeof(unsigned) * nc + nc + 256;
    HIPCHK(c, c->arm.ensure(need));
    char* p = (char*)c->arm.p;
    HIPCHK(c, hipMemcpyAsync(p, T.buf.data(), tb, hipMemcpyHostToDevice, st));
    const double* d = (const double*)p;
    a.toaA = d + T.oA;
    a.toaB = d + T.oB;
    a.toaC = d + T.oC;
    a.tabI = d + T.oI;
    a.tabK = d + T.oK;
    a.norm = d + T.oN;
    a.valA = d + T.oV;
    a.ct = d + T.oct;
    a.st = d + T.ost;
    a.cs = d + T.ocs;
    a.ss = d + T.oss;
    a.ks = d + T.oks;
    a.valC = d + T.ovc;
    a.first = (unsigned*)(p + ((tb + 255) & ~(size_t)255));
    a.closed = (unsigned char*)(a.first + nc);
    a.tunnel = d_tunnel;
    a.fmap = d_fmap;
    a.out = d_cost;
    HIPCHK(c, arm_tunnel(a, st));
    // the tables must outlive the kernels: T.buf is host memory copied above; wait before return
    HIPCHK(c, hipStreamSynchronize(st));
    if (d_Z) {
        unsigned bad = 0;
        HIPCHK(c, hipMemcpy(&bad, c->misc.p, sizeof bad, hipMemcpyDeviceToHost));
        if (bad) return set_err(c, EIK_ERR_ARG, "GetObstMap: a surface index below -sZ (the reference raises IndexError)");
    }
    return EIK_OK;
}

static int arm_check(eik_ctx* c, const eik_arm_volume* v) {
    if (!v || v->sX < 1 || v->sY < 1 || v->sZ < 1 || !(v->resX > 0) || !(v->resY > 0) || !(v->resZ > 0))
        return set_err(c, EIK_ERR_ARG, "bad arm volume");
    if (v->sX != v->sY) return set_err(c, EIK_ERR_ARG, "arm volume must be square in x, y (sX %ld != sY %ld)",
                                       (long)v->sX, (long)v->sY);
    return EIK_OK;
}

extern "C" {

int eik_arm_obst_map_f64(eik_ctx* c, const double* Z, const double* obst, int64_t m, int64_t n,
                         const eik_arm_volume* v, double* fmap, double* omap, double* gmap) {
    if (!c || !Z || !obst || !fmap || m < 1 || n < 1) return c ? set_err(c, EIK_ERR_ARG, "NULL argument") : EIK_ERR_ARG;
    int rc = arm_check(c, v);
    if (rc) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t st = c->stream;
    const int64_t nc = v->sX * v->sY * v->sZ, nz = m * n;
    HIPCHK(c, c->T2.ensure(sizeof(double) * (2 * nz + 3 * nc)));
    double* dZ = (double*)c->T2.p;
    double* dO = dZ + nz;
    double* dF = dO + nz;
    double* dOm = omap ? dF + nc : nullptr;
    double* dGm = gmap ? dF + 2 * nc : nullptr;
    HIPCHK(c, host_to_dev(c, dZ, Z, sizeof(double) * nz, st));
    HIPCHK(c, host_to_dev(c, dO, obst, sizeof(double) * nz, st));
    rc = arm_volume_dev(c, dZ, dO, m, n, nullptr, nullptr, 0, v, dF, dOm, dGm, nullptr, nullptr, st);
    if (rc) return rc;
    unsigned bad = 0;
    HIPCHK(c, hipMemcpyAsync(&bad, c->misc.p, sizeof bad, hipMemcpyDeviceToHost, st));
    HIPCHK(c, dev_to_host(c, fmap, dF, sizeof(double) * nc, st));
    if (omap) HIPCHK(c, dev_to_host(c, omap, dOm, sizeof(double) * nc, st));
    if (gmap) HIPCHK(c, dev_to_host(c, gmap, dGm, sizeof(double) * nc, st));
    HIPCHK(c, hipStreamSynchronize(st));
    if (bad) return set_err(c, EIK_ERR_ARG, "GetObstMap: a surface index below -sZ (the reference raises IndexError)");
    return EIK_OK;
}

int eik_arm_tunnel_cost_f64(eik_ctx* c, const double* gamma2D, const double* heading, int64_t npts,
                            const eik_arm_volume* v, double* Cmap) {
    if (!c || !gamma2D || !heading || !Cmap || npts < 1) return c ? set_err(c, EIK_ERR_ARG, "NULL argument") : EIK_ERR_ARG;
    int rc = arm_check(c, v);
    if (rc) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t nc = v->sX * v->sY * v->sZ;
    HIPCHK(c, c->T2.ensure(sizeof(double) * nc));
    double* dT = (double*)c->T2.p;
    rc = arm_volume_dev(c, nullptr, nullptr, 0, 0, gamma2D, heading, npts, v, nullptr, nullptr, nullptr, dT, nullptr,
                        c->stream);
    if (rc) return rc;
    HIPCHK(c, dev_to_host(c, Cmap, dT, sizeof(double) * nc, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return EIK_OK;
}

int eik_arm_path_f64(eik_ctx* c, const double* Z, const double* obst, int64_t m, int64_t n, const double* gamma2D,
                     const double* heading, int64_t npts, const eik_arm_volume* v, double tau, double* path,
                     int64_t cap, int64_t* n_out, int* status, double* cost_out, double* T_out) {
    if (!c || !Z || !obst || !gamma2D || !heading || !path || !n_out || !status || npts < 1 || m < 1 || n < 1 ||
        !(tau > 0) || cap < 2)
        return c ? set_err(c, EIK_ERR_ARG, "bad arm-path arguments") : EIK_ERR_ARG;
    int rc = arm_check(c, v);
    if (rc) return rc;
    for (int k = 0; k < 3; ++k) {
        const int64_t lim = k == 0 ? v->sX : k == 1 ? v->sY : v->sZ;
        if ((int64_t)v->final_wp[k] >= lim || (int64_t)v->initial_wp[k] >= lim)
            return set_err(c, EIK_ERR_ARG, "waypoint outside the %ldx%ldx%ld volume", (long)v->sX, (long)v->sY,
                           (long)v->sZ);
    }
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t st = c->stream;
    const int64_t nc = v->sX * v->sY * v->sZ, nz = m * n;
    const int64_t steps = (int64_t)std::nearbyint(15000.0 / tau);
    const int64_t pcap = std::min<int64_t>(cap, steps + 4);
    // Z | obst | fmap | tunnel | cost | T (full) | T (early exit) | path | n_out | status
    HIPCHK(c, c->T2.ensure(sizeof(double) * (2 * nz + 5 * nc + 3 * pcap) + 64));
    double* dZ = (double*)c->T2.p;
    double* dO = dZ + nz;
    double* dF = dO + nz;
    double* dTun = dF + nc;
    double* dC = dTun + nc;
    double* dTf = dC + nc;
    double* dT = dTf + nc;
    double* dP = dT + nc;
    int64_t* dn = (int64_t*)(dP + 3 * pcap);
    int* dst = (int*)(dn + 1);
    HIPCHK(c, host_to_dev(c, dZ, Z, sizeof(double) * nz, st));
    HIPCHK(c, host_to_dev(c, dO, obst, sizeof(double) * nz, st));
    rc = arm_volume_dev(c, dZ, dO, m, n, gamma2D, heading, npts, v, dF, nullptr, nullptr, dTun, dC, st);
    if (rc) return rc;
    // FM3D.computeTmap(Cmap, finalWayPointArm, initialWayPointArm) :1585; H = sY rows, W = sX columns
    // with its early exit once initialWayPointArm is popped (FastMarching3D.py:141)
    const int64_t goal[3] = {v->final_wp[0], v->final_wp[1], v->final_wp[2]};
    const int64_t start[3] = {v->initial_wp[0], v->initial_wp[1], v->initial_wp[2]};
    rc = fim3d_solve_one(c, dC, dTf, v->sY, v->sX, v->sZ, EIK_F64, goal, st,
                         early_offset(goal, start, v->sY, v->sX, v->sZ));
    if (rc) return rc;
    rc = eik_fim3d_early_exit(c, dC, dTf, dT, v->sY, v->sX, v->sZ, EIK_F64, goal, start, st);
    if (rc) return rc;
    // FM3D.getPathGDM(Tmap3D, initialWayPointArm, finalWayPointArm, 0.5) :1588
    const double init[3] = {(double)v->initial_wp[0], (double)v->initial_wp[1], (double)v->initial_wp[2]};
    const double end[3] = {(double)v->final_wp[0], (double)v->final_wp[1], (double)v->final_wp[2]};
    rc = eik_path3d_dev(c, dT, EIK_F64, v->sY, v->sX, v->sZ, init, end, tau, dP, pcap, dn, dst, st);
    if (rc) return rc;
    int64_t hn = 0;
    HIPCHK(c, hipMemcpyAsync(&hn, dn, sizeof hn, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(status, dst, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    *n_out = hn;
    HIPCHK(c, hipMemcpyAsync(path, dP, sizeof(double) * 3 * hn, hipMemcpyDeviceToHost, st));
    if (cost_out) HIPCHK(c, dev_to_host(c, cost_out, dC, sizeof(double) * nc, st));
    if (T_out) HIPCHK(c, dev_to_host(c, T_out, dT, sizeof(double) * nc, st));
    HIPCHK(c, hipStreamSynchronize(st));
    return EIK_OK;
}

int eik_tmap3d_batch_f64(eik_ctx* c, const double* cost, int64_t B, int64_t H, int64_t W, int64_t L,
                         const int64_t* goals, double* T) {
    if (!c || !cost || !T || !goals || B < 1 || H < 1 || W < 1 || L < 1)
        return c ? set_err(c, EIK_ERR_ARG, "bad 3D batch arguments") : EIK_ERR_ARG;
    for (int64_t b = 0; b < B; ++b)
        if (goals[3 * b] < 0 || goals[3 * b + 1] < 0 || goals[3 * b + 2] < 0 || goals[3 * b] >= W ||
            goals[3 * b + 1] >= H || goals[3 * b + 2] >= L)
            return set_err(c, EIK_ERR_ARG, "goal of volume %ld outside %ldx%ldx%ld", (long)b, (long)H, (long)W, (long)L);
    const int64_t n = B * H * W * L;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, c->cost.ensure(sizeof(double) * n));
    HIPCHK(c, c->T.ensure(sizeof(double) * n));
    HIPCHK(c, host_to_dev(c, c->cost.p, cost, sizeof(double) * n, c->stream));
    int rc = check_cost(c, cost, c->cost.p, n, c->stream);
    if (rc) return rc;
    rc = fim3d_solve_batch(c, c->cost.p, c->T.p, B, H, W, L, EIK_F64, goals, c->stream);
    if (rc) return rc;
    HIPCHK(c, dev_to_host(c, T, c->T.p, sizeof(double) * n, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return EIK_OK;
}

}  // extern "C"
