// eik_kernels.hpp -- device-side argument blocks and host launchers of the HIP kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace eik {

// One FIM solve over B maps of H x W (or one subdomain of a decomposed raster).
struct Fim2dArgs {
    const void* cost;      // [B][H][W] R, device
    void* T;               // [B][H][W] R, device
    int64_t H, W;
    int ntx, nty, tiles_per_map;
    const void* ghost[4];  // N (W), S (W), W (H), E (H) ghost strips, device; nullptr = +inf
    int* lists;            // 3 x capacity active-tile lists (triple-buffered by iteration)
    int* counts;           // [4] list lengths
    unsigned* mark;        // per tile: last iteration+1 it was enqueued for (dedup)
    int capacity;          // B * tiles_per_map
    unsigned iter;         // outer iteration index of this launch
    int max_rounds;        // sweep rounds per tile visit
    float keep;            // 1 - tol: a change counts for (re)activation only if new < old * keep
    unsigned* key;         // per tile: smallest T entering it since its last visit (f32 bits)
    unsigned* minkey;      // [3] per list: min key of the tiles enqueued in it (f32 bits)
    float delta;           // process a listed tile only if key <= minkey + delta (inf: always)
    unsigned long long* visits;  // tile-visit counter (stats / roofline bytes)
    unsigned* edge_dirty;  // DD: bit per subdomain side whose edge row/column changed
    // persistent mode (one launch per solve, device FIFO of tiles)
    int mode;              // kModeList / kModePersistent
    unsigned long long* qhead;  // ticket counter (consumers)      -- qctl + 0
    unsigned long long* qtail;  // append counter (producers)      -- qctl + 64
    int* qactive;          // tiles pending or busy               -- qctl + 128
    unsigned* qerror;      // nonzero: a spin timed out           -- qctl + 192
    unsigned* qslot;       // [qmask + 1] FIFO slots: tile + 1, 0 = empty
    unsigned qmask;        // power of two >= tiles, minus one
    unsigned* qstate;      // per tile: kPending | kBusy | trigger bits | kVisited
    int fresh_first;       // nonzero: a tile's first activation jumps a backlog (qslot_put_front)
    int sched;             // persistent visits: bit 0 consume activations in place, bit 1 defer in-place activations
    unsigned long long qtimeout;  // spin limit, s_memrealtime ticks (100 MHz)
    unsigned long long qbudget;   // tile-visit cap (negative costs never converge)
    int max_passes;        // in-place sweep passes per persistent visit (EIK_OPT_PASSES)
    // bidirectional fronts (eikonal_api.cpp solve_fronts): per map, an edge value above tcap[map]
    // activates no neighbour -- every cell whose converged T is <= tcap depends only on cells below
    // it, so it still converges exactly; nullptr: no cap (honoured by the fp64 persistent kernel only)
    const double* tcap;
    // EIK_OPT_EXACT_BAND's fronts (eikonal_api.cpp solve_fronts): fp64 persistent solves step in the
    // reference's getEikonal arithmetic (fim2d.hip sweep_quadrant REF)
    int ref_arith;
    // every tile's west / east edge column, [tile][2][kTile] R, kept equal to T's (fim2d.hip kEcol): the
    // west / east halo of a tile visit is one contiguous 64-cell read instead of 64 rows' lines
    void* ecol;
    // layered solver (fim2dl.hip): cell (y, x) holds ls consecutive values, layers z0.. solved
    int64_t ls;            // cell stride (the [y][x][L] volume: L; 1 for the 2D solver and layer-planar copies)
    int z0;                // offset of the first solved layer in a cell (the volume: its index; planar: 0)
    int64_t lzs;           // layer stride: 1 in the [y][x][L] volume, H * W in a layer-planar copy
    // live domain decomposition (eik_fim2d_launch with live != 0): the persistent launch stays up
    // -- its workgroup 0 is the halo agent serving the host's commands -- and ends when
    // *qhold != 0
    unsigned* qhold;       // nullptr: end when no tile is pending or busy
    struct LiveBox* live;  // pinned host mailbox of the halo agent (live launches only)
    int live_pack;         // EIK_OPT_LIVE_PACK: 1 = the agent packs only cells of idle tiles
    // priority bands (EIK_OPT_PRIO, fim_engine.hpp): pending tiles wait in kBands FIFOs by entering T
    // (band = T / pdelta, the last band open-ended) and are taken lowest band first; nullptr bctl: off
    unsigned* bslot;            // [kBands][bmask + 1]: tile + 1, 0 = empty
    unsigned bmask;
    // per tile: bit b set while an entry of the tile sits in band b's ring or on its way from there
    // through the FIFO (fim_engine.hpp band_put): at most one entry per (tile, band), so a ring of
    // >= tiles slots can never lap
    unsigned long long* bmem;
    unsigned long long* bctl;   // band b: head at bctl[16 b], tail at bctl[16 b + 8] (own 64-B lines)
    const float* pdelta;        // band width in units of T (device word: prio_delta_kernel sets it per solve)
    unsigned disp;              // band entries moved per dispatch (fim_engine.hpp band_dispatch; 0: kDispatch)
};

// Host <-> halo-agent mailbox (pinned, coherent host memory).  The host writes cmd, then seq
// (release); the agent runs the command and writes its results, then done = seq (release).
constexpr unsigned kLivePack = 1, kLiveMerge = 2, kLiveRelease = 3;
struct LiveBox {
    unsigned seq;        // host: sequence number of the posted command
    unsigned cmd;        // host: op | parity << 8
    unsigned done;       // agent: seq of the last completed command
    unsigned active;     // agent: tiles pending or busy at the last pack (snapshot BEFORE reading T)
    unsigned changed;    // agent: ghost cells the last merge lowered
    unsigned error;      // agent: queue error bits
    unsigned pad[2];
    void* send[2][4];    // host: edge targets by parity and side (a neighbour's receive strips)
    const void* recv[2][4];  // host: this block's receive strips by parity and side
};
constexpr int kModeList = 0, kModePersistent = 1;
// queue words: head @0, tail @64, active @128, error @192; the 2D solver's two visit counters
// @kVisitsOff, on a 128-B line of their own (sharing the error word's line -- polled by every
// grab -- with the in-place passes' atomics cost C2 ~20 %)
constexpr size_t kQueueCtlBytes = 384;
constexpr int kBands = 64;  // priority bands (EIK_OPT_PRIO): one band per lane of the grabbing wave
// a FIFO entry moved there from band b carries b + 1 in its top bits (the claimer clears the tile's
// band-membership bit); the low bits hold tile + 1
constexpr unsigned kBandTagShift = 25;
constexpr unsigned kSlotTileMask = (1u << kBandTagShift) - 1u;
constexpr size_t kVisitsOff = 256;

// T = inf, queue / list / visit / edge words cleared, goals seeded
hipError_t fim2d_init(const Fim2dArgs& a, bool f64, int nmaps, const int64_t* d_goals, unsigned* edge, hipStream_t st);
hipError_t fim2d_sweep(const Fim2dArgs& a, bool f64, int grid, hipStream_t st);
// wide: the 4-waves-per-SIMD form of the fp32 kernel, for maps of >= kWideTiles tiles
constexpr int64_t kWideTiles = 16384;
hipError_t fim2d_persist(const Fim2dArgs& a, bool f64, int grid, hipStream_t st, bool wide = false, bool rewind = true);
hipError_t fim2d_qrewind(const Fim2dArgs& a, hipStream_t st);
hipError_t fim2d_prio_delta(const void* cost, bool f64, int64_t n, float mult, float* out, hipStream_t st);
int fim2d_persist_resident(bool f64, int cus, bool wide = false);
hipError_t fim2d_merge_ghost(const Fim2dArgs& a, bool f64, int side, const void* recv, int64_t len, hipStream_t st);
hipError_t fim2d_pack_edges(const Fim2dArgs& a, bool f64, void* n, void* s, void* w, void* e, hipStream_t st);

// Layered solver (fim2dl.hip): a [H][W][ls] volume, layers z0 .. z0+nl-1 (fp32: nl <= 4, tiles of
// 64 x 64; fp64: nl <= 3, tiles of fim2dl_rows(true) = 40 rows x 64 columns), on the 2D tile engine
// (persistent mode only; a.ls / a.z0 set, no ghosts, no ordering window; a.nty counts tiles of
// fim2dl_rows(f64) rows).
int fim2dl_rows(bool f64);
hipError_t fim2dl_init(const Fim2dArgs& a, bool f64, int64_t gx, int64_t gy, int64_t gz, int64_t n, hipStream_t st);
// [y][x][L] volume <-> layer-planar copy [nl][H][W] of layers z0 .. z0+nl-1 (in: volume -> copy;
// out: copy -> volume, the other layers of every cell set to +inf)
hipError_t layer_planar(const void* src, void* dst, bool f64, int64_t hw, int64_t L, int z0, int nl, bool in,
                        hipStream_t st);
// layered domain decomposition: edges of nl values per cell into strips; strips min-merged into ghosts
hipError_t fim2dl_pack_edges(const Fim2dArgs& a, int nl, bool f64, void* n, void* s, void* w, void* e, hipStream_t st);
hipError_t fim2dl_merge_ghost(const Fim2dArgs& a, int nl, bool f64, int side, const void* recv, hipStream_t st);
hipError_t fim2dl_persist(const Fim2dArgs& a, int nl, bool f64, int grid, hipStream_t st);
int fim2dl_persist_resident(int nl, bool f64, int cus);
hipError_t layer_finite(const void* cost, bool f64, int64_t hw, int64_t L, int64_t z, int* d_flag, hipStream_t st);

// 3D FIM over one H x W x L volume ([y][x][z], FastMarching3D.py layout).
struct Fim3dArgs {
    const void* cost;
    void* T;
    int64_t H, W, L;
    int tx, ty, tz;        // tile shape
    int ntx, nty, ntz;
    int* lists;
    int* counts;
    unsigned* mark;
    int capacity;
    unsigned iter;
    int max_passes;        // relaxation passes per tile visit
    unsigned long long* visits;
    int tpv;               // tiles per volume (B volumes: tile = volume * tpv + tile in volume)
    // early exit at `start` (FastMarching3D.py:141; one volume): a cell is lowered only to values
    // <= T[stop_off] + *stop_slack (the largest finite cost), the bound of every value the
    // early-exit field keeps (fim3d_early_kernel).  stop_off = -1: no bound.
    int64_t stop_off;
    const void* stop_slack;  // device R
};
// the largest finite cost of n values (non-negative or +inf) -> *d_max (device R, zeroed here)
hipError_t max_finite(const void* cost, int64_t n, bool f64, void* d_max, hipStream_t st);
// T = inf for B volumes, goal cell of volume b = d_goals[3b..3b+2] (x, y, z) set to 0 and listed
hipError_t fim3d_init(const Fim3dArgs& a, bool f64, const int64_t* d_goals, int B, hipStream_t st);
hipError_t fim3d_sweep(const Fim3dArgs& a, bool f64, int grid, hipStream_t st);
void fim3d_tile_shape(int64_t L, int* tx, int* ty, int* tz);
// persistent driver of the 3D solver (one launch per solve): q carries the tile FIFO of
// fim_engine.hpp (qhead .. qstate, qtimeout, qbudget, visits[2]) sized for a.capacity tiles
hipError_t fim3d_persist_init(const Fim3dArgs& a, const Fim2dArgs& q, bool f64, const int64_t* d_goals, int B,
                              hipStream_t st);
hipError_t fim3d_persist(const Fim3dArgs& a, const Fim2dArgs& q, bool f64, int grid, hipStream_t st);
int fim3d_persist_resident(bool f64, int cus);
// FastMarching3D.computeTmap's early exit at `start` (:141) from a converged field Tf into Te
// (a separate buffer); ts_off = start's linear index, or -1 for no early exit (fim3d.hip).
hipError_t fim3d_early(const void* cost, const void* Tf, void* Te, int64_t H, int64_t W, int64_t L, int64_t ts_off,
                       bool f64, hipStream_t st);

// Gradient-descent path extraction (getPathGDM, FastMarching.py:164-236), one wave.
struct Gdm2dArgs {
    const void* T;         // [H][W] field (R), device
    int64_t H, W;
    double ix, iy, ex, ey, tau;
    long steps;            // round(15000 / tau)
    double* out;           // [cap][2], device
    int64_t cap;
    int64_t* n_out;        // device
    int* status;           // device
    int fused;             // EIK_OPT_PATH_LOOP: 2 single-exit loop + range-free sqrt/div, 1 single-exit loop,
                           // 0 reference-structured loop (same path bits)
};
hipError_t gdm2d(const Gdm2dArgs& a, bool f64, hipStream_t st);
// fast-path arithmetic of the 2D walker vs the exact forms (gdm.hip): mismatch counts [3] + samples, device
hipError_t walker_math_selftest(long long n, unsigned long long seed, unsigned long long* d_counts, hipStream_t st);

// FastMarching3D.getPathGDM (:198-271): np.gradient field, trilinear (a7 as in :290), integer
// 6-neighbour fallback, unnormalised step.
struct Gdm3dArgs {
    const void* T;         // [H][W][L] field (R), device
    int64_t H, W, L;
    double init[3], end[3], tau;
    long steps;
    double* out;           // [cap][3]
    int64_t cap;
    int64_t* n_out;
    int* status;
};
hipError_t gdm3d(const Gdm3dArgs& a, bool f64, hipStream_t st);

// Cost-raster builder (costmap.hip), f64 DEM -> f64 cost, uint8 obstacle masks.
hipError_t cm_normals(const double* Z, int64_t H, int64_t W, double size, unsigned long long* zmin, double slope_max,
                      unsigned char* obst, double* Nx, double* Ny, double* Nz, hipStream_t st);
hipError_t cm_morph(const unsigned char* A, int64_t H, int64_t W, int r, bool erode, unsigned char* out, int* g, int* D,
                    int* vbuf, hipStream_t st);
// :1194's transform as od (:1196) uses it: exact where D <= r^2 (r = :1192's dil radius) and at its maximum
hipError_t cm_edt_ramp(const unsigned char* m, int64_t H, int64_t W, int r, int* g, int* D, int* vbuf, hipStream_t st);
hipError_t cm_edt(const unsigned char* m, unsigned char val, int64_t H, int64_t W, int* g, int* D, int* vbuf,
                  hipStream_t st);
hipError_t cm_fill_cost(const unsigned char* m, int64_t n, float* c, hipStream_t st);
hipError_t cm_fill_apply(unsigned char* m, const float* T, int64_t n, hipStream_t st);
// the same fill by connected components (union-find; lroot, parent: n ints of scratch)
hipError_t cm_fill_ccl(unsigned char* m, int64_t H, int64_t W, int* lroot, int* parent, hipStream_t st);
// first index with cost < 0 or NaN into *first (~0: none); costmap.hip
hipError_t cost_check(const void* cost, int64_t n, bool f64, unsigned long long* first, hipStream_t st);
hipError_t cm_border(unsigned char* m, int64_t H, int64_t W, unsigned char v, hipStream_t st);
hipError_t cm_cost(const unsigned char* obst, const unsigned char* dil, const int* Dobst, int64_t H, int64_t W,
                   double res, double high, double gradient, double* work, double* tmp, double* cost,
                   unsigned long long* red, hipStream_t st);

// Full-field inf-aware normalised gradient (computeGradient(T, point=[]), FastMarching.py:242-300)
hipError_t gradient2d(const double* T, int64_t H, int64_t W, double* gnx, double* gny, hipStream_t st);

// End-effector cost volume (arm.hip): GetObstMap + TunnelCost event painting.
struct ArmArgs {
    long long sX, sY, sZ;       // volume [iy][ix][iz], sY x sX x sZ (the planner's area is square)
    double resX, resY, resZ, rlim, rad;
    int nX, nZ, nK;
    unsigned long long nA, nB, nC;  // events of the tunnel, the closing step, the half sphere
    const double* toaA;         // [points][12]: rows 0..2 of the base transform (yaw - pi/2)
    const double* toaB;         // [12] first point (closing step)
    const double* toaC;         // [12] last point, no yaw offset (half sphere)
    const double *tabI, *tabK, *norm, *valA;      // linspaces, per (i, k) norm and value
    const double *ct, *st, *cs, *ss, *ks, *valC;  // half-sphere tables
    long long fw[3], iw[3];     // sample / start nodes (x, y, z)
    unsigned* first;            // [cells] lowest assign sequence number
    unsigned char* closed;      // [cells]
    double* tunnel;             // [cells] TunnelCost's Cmap
    const double* fmap;         // [cells] GetObstMap's finalMap (for out)
    double* out;                // nullable: fmap * tunnel
};
hipError_t arm_obst_map(const double* Zs, const double* obst, int64_t m, int64_t n, double resX, double resY,
                        double resZ, int64_t sX, int64_t sY, int64_t sZ, double xm, double ym, double* fmap,
                        double* omap, double* gmap, unsigned* bad, hipStream_t st);
hipError_t arm_tunnel(const ArmArgs& a, hipStream_t st);

// ---- biComputeTmap's join (bidir.hip) -------------------------------------------------------
// nodeJoin from two full fields (d_best: the packed join, ~0 = the fronts never meet); one host
// synchronisation; members (optional, host): the cells ranked per front
hipError_t bidir_join(const double* d_TG, const double* d_TS, int64_t n, void* d_work, size_t work_bytes,
                      unsigned long long* d_best, hipStream_t st, int64_t* members = nullptr);
size_t bidir_join_work_bytes(int64_t n);
hipError_t bidir_band_stats(const void* d_work, int64_t n, unsigned out[4], hipStream_t st);
// after bidir_join on the same work buffer: the two fields -> biComputeTmap's partial fields;
// d_cost / d_viol (optional): flag a band cell of finite cost left +inf (capped fronts)
hipError_t bidir_partial(double* d_TG, double* d_TS, int64_t H, int64_t W, const void* d_work,
                         const unsigned long long* d_best, hipStream_t st, const double* d_cost = nullptr,
                         unsigned* d_viol = nullptr);
void bidir_join_ranks(const void* d_work, int64_t n, const unsigned** rg, const unsigned** rs);
hipError_t bidir_join_min(const unsigned* d_rg, const unsigned* d_rs, int64_t n, unsigned long long* d_best,
                          hipStream_t st);
// EIK_OPT_EXACT_BAND (bidir_exact.hip): the reference's own partial fields and nodeJoin, replayed in pop
// order from the join's ranks d_rg / d_rs (members[f] cells ranked per front) over the device cost;
// d_TG / d_TS (the converged fields) become the partial fields, *d_best the exact join.  info
// (accumulated): passes, relaxation sweeps G, S, tie-run launches.  hipErrorNotReady: no fixed point
// within the caps; hipErrorNotSupported: a run of more than 4096 exactly equal T (a zero-cost region);
// hipErrorIllegalState: the exact meeting is not clear of the ranked prefix's bound (never expected).
size_t bidir_exact_work_bytes(int64_t n, int64_t m0, int64_t m1);
hipError_t bidir_exact(double* d_TG, double* d_TS, const double* d_cost, int64_t H, int64_t W, int64_t gnode,
                       int64_t snode, const unsigned* d_rg, const unsigned* d_rs, const int64_t members[2],
                       void* d_work, size_t work_bytes, unsigned long long* d_best, hipStream_t st,
                       unsigned long long info[4]);
// ... and FastMarching3D.computeTmap's early exit (:137-142) in the same replay: d_T the converged fp64
// field from goal_off, d_Te the reference's own partial field after popping start_off (its band's
// tentative values, its LIFO ties)
size_t fm3d_exact_work_bytes(int64_t n);
hipError_t fm3d_exact(const double* d_cost, const double* d_T, double* d_Te, int64_t H, int64_t W, int64_t L,
                      int64_t goal_off, int64_t start_off, void* d_work, size_t work_bytes, hipStream_t st,
                      unsigned long long info[4]);
// the capped fronts' device block (eikonal_api.cpp solve_fronts)
struct FrontsCheck {
    double caps[2];                   // per front: activation cap of the full-resolution solve
    unsigned long long maxcost_bits;  // largest finite cost of the raster (double bits)
    unsigned kept[2];                 // cells at or below the cap per front
    unsigned viol;                    // a band cell was cut off by the cap
    unsigned pad;
    unsigned long long best_c;        // the coarse fields' seed (~0: they never meet)
};
hipError_t fronts_coarse_cost(const double* d_cost, int64_t H, int64_t W, int F, double* d_out, int64_t Hc, int64_t Wc,
                              FrontsCheck* chk, hipStream_t st);
hipError_t fronts_estimate(const double* d_TG, const double* d_TS, int64_t n, void* d_work, double F, double margin,
                           FrontsCheck* chk, hipStream_t st);
hipError_t fronts_clean(double* d_T, int64_t n, FrontsCheck* chk, hipStream_t st);

}  // namespace eik
