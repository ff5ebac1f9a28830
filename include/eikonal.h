/*
 * eikonal.h -- C ABI of the MI355X-native Eikonal cost-to-go solver (libeikonal.so).
 *
 * The drop-in boundary for the hot path of esa-prl/planning-motion_planning:
 *   src/FastMarching/FastMarching.py   (2D FMM + gradient-descent path)
 *   src/FastMarching/FastMarching3D.py (3D FMM + path)
 * reached from Python through ctypes (planning-motion_planning_amd/FastMarching/, same module
 * and function names as the reference) and from C++ directly (include/MotionPlanning.hpp
 * users, Rock components).  Plain C: pointers + sizes, no exceptions, no torch types.
 *
 * Conventions (identical to the reference):
 *   - rasters are row-major [y][x] (3D: [y][x][z]); nodes are (x, y(, z));
 *   - cost = +inf marks an impassable cell (FastMarching.py:93-94); costs must be >= 0;
 *   - T = +inf marks an unreached cell;
 *   - out-of-range neighbours read as +inf (the reference instead relies on an inf border,
 *     Coupled_motion_planner.py:1213-1216, and wraps/raises without one).
 * Every function returns an eik_status (0 = OK); on error eik_last_error() describes it.
 * One context per host thread; a context owns its device buffers and HIP stream.
 * Host-buffer entry points (eik_tmap*, eik_path*, eik_gradient*) are synchronous.
 * Device entry points (eik_fim2d_*, eik_path2d_dev) take device pointers and a hipStream_t
 * (passed as void*, used as given: NULL is the default null stream, as in HIP) and are
 * asynchronous unless noted.
 */
#ifndef EIKONAL_H_
#define EIKONAL_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    EIK_OK = 0,
    EIK_ERR_ARG = -1,         /* bad argument (shape, index, negative cost, NULL pointer)     */
    EIK_ERR_HIP = -2,         /* HIP runtime / launch failure                                  */
    EIK_ERR_NOMEM = -3,       /* device or host allocation failed                               */
    EIK_ERR_NOCONVERGE = -4,  /* iteration cap reached (e.g. negative cost on a device buffer)  */
    EIK_ERR_UNREACHABLE = -5, /* bidirectional fronts never meet (reference: UnboundLocalError) */
    EIK_ERR_NODEVICE = -6     /* no HIP device / library built without one                       */
} eik_status;

typedef enum { EIK_F32 = 0, EIK_F64 = 1 } eik_dtype;

/* path status (eik_path2d / eik_path3d), mirrors the reference's exits */
typedef enum {
    EIK_PATH_DONE = 0,     /* stop radius (< 1.5 cells) or step budget hit; end appended (:231-234) */
    EIK_PATH_FALLBACK = 1, /* NaN gradient: the reference's fallback returns a truncated path
                              (numpy-2 behaviour of FastMarching.py:178-218)                       */
    EIK_PATH_ERROR = 2     /* the reference raises out of getPathGDM (NaN point / out of range)     */
} eik_path_status;

typedef struct eik_ctx eik_ctx;
typedef struct eik_fim2d eik_fim2d;

typedef struct {
    int64_t iterations;   /* solver launches of the last solve (list mode: outer iterations) */
    int64_t tile_visits;  /* 64x64 tile visits of the last solve                                */
    int64_t host_syncs;   /* active-count read-backs                                            */
    double solve_ms;      /* device time of the last solve (hipEvents, init..converged)         */
    double sweep_ms;      /* summed device time of the sweep launches (timing option on)        */
    double bytes_alg;     /* algorithmic bytes of the sweep launches (tile_visits x bytes/visit) */
    int64_t inplace_passes; /* persistent mode: extra in-place passes of busy tiles (halo refresh
                               + sweep + write-back of the tile already in LDS)                 */
    int64_t fresh_visits; /* persistent mode: tile visits (among tile_visits) that read no T --
                             the tile's first visit, T still +inf (bytes_alg counts them so)    */
} eik_stats;

/* options (eik_set_option) */
typedef enum {
    EIK_OPT_MAX_ROUNDS = 0,  /* sweep rounds per tile visit before re-enqueueing (default 1)   */
    EIK_OPT_SYNC_EVERY = 1,  /* sweep launches between active-count read-backs (default 8)     */
    EIK_OPT_TIMING = 2,      /* 1: time each sweep launch with hipEvents (for the roofline)     */
    EIK_OPT_GRID = 3,        /* workgroups per sweep launch (default 4 x CUs)                   */
    EIK_OPT_TOL = 4,         /* relative change below which a cell does not (re)activate tiles  */
    EIK_OPT_DELTA = 5,       /* ordered mode: per launch, only tiles whose entering T is within
                                delta of the smallest pending one are swept (0: off; > 0 forces
                                EIK_MODE_LIST)                                                  */
    EIK_OPT_MODE = 6,        /* EIK_MODE_PERSISTENT (default): one launch per solve over a device
                                FIFO of tiles; EIK_MODE_LIST: one launch per outer iteration   */
    EIK_OPT_QTIMEOUT = 7,    /* persistent mode: seconds a workgroup may wait on the FIFO before
                                the solve fails with EIK_ERR_HIP instead of hanging (default 30) */
    EIK_OPT_MAX_VISITS = 8,  /* persistent mode: tile visits after which a solve fails with
                                EIK_ERR_NOCONVERGE (0: default 1024 x tiles + 2^20)            */
    EIK_OPT_PASSES = 9,      /* persistent mode: sweep passes a visit may run in place while its
                                tile keeps changing before it is re-queued (0, the default:
                                24 for a single map, 16 for a single fp32 map of >= 16384
                                tiles, 2 for a batch of maps)                                  */
    EIK_OPT_FRESH_FIRST = 10,/* persistent mode: 1 queues a tile's first activation ahead of
                                re-visits while the queue has a backlog (default 0: one FIFO)  */
    EIK_OPT_SCHED = 11,      /* persistent mode, bit mask: 1 = a busy tile serves activations that
                                reach it in place (no re-queued visit); 2 = after a visit's first
                                pass, neighbour activations wait for the visit's end (default 1:
                                profiles/r02d_grab_sched_ab.log)                                 */
    EIK_OPT_PATH_LOOP = 12,  /* 2D path kernel: 2 = one exit branch per step (the step is
                                computed before its special cases are tested) with the f64 sqrt /
                                division free of range handling inside their safe domain; 1 = the
                                same loop with the compiler's sqrt / division; 0 = the loop in
                                the reference's statement order; 3 = form 2 with both divisions
                                taken from the square roots' reciprocals (gdm.hip div_rs, checked
                                by eik_selftest_walker_math); 4 (default) = form 3 on lane pairs,
                                x on even lanes, y on odd, one-correction square roots.  Same
                                path bits in all five.                                          */
    EIK_OPT_FRONTS_CAP = 13, /* biComputeTmap / rover path, rasters >= 2^20 cells: 1 (default) solves
                                each front only up to a cap on T estimated from a coarse copy of
                                the raster (x 1.25) and falls back to the full solve when the
                                capped fields cannot be shown to give the full fields' join; a
                                value v > 1: the same with margin v; 0 = full fronts            */
    EIK_OPT_LIVE_PACK = 14,  /* live domain decomposition (eik_fim2d_live_pack): 0 (default) = the
                                halo agent stores every edge cell each round; 1 = only the cells
                                of tiles that are neither pending nor busy (converged edges), so a
                                neighbour is not re-activated by every intermediate refinement
                                (a round whose snapshot had no tile pending or busy packs all)   */
    EIK_OPT_PRIO = 15,       /* 2D persistent solves of one or two maps and the layered 3D solver:
                                v > 0 serves waiting tiles lowest entering T first, in 64 bands of
                                width v x 64 x the geometric mean of the finite costs
                                (fim_engine.hpp "priority bands"); 0 = the FIFO; < 0 (default) =
                                0.25 x max(1, sqrt(H W) / 4096) for fp64 2D solves of rasters
                                of >= 4096^2 cells (any size for a decomposition block), one
                                fp32 2D map of >= 16384 tiles and layered solves of >= 3072^2
                                in either dtype; else the FIFO                                   */
    EIK_OPT_LAYER_PLANAR = 16, /* few-layer 3D volumes (the layered solver): 1 (default) solves on
                                layer-planar copies [nl][H][W] of the solved layers (one copy in,
                                one out per solve; every tile-row access one contiguous run per
                                layer); 0 = in the volume's [y][x][L] layout                     */
    EIK_OPT_PRIO_RING = 17,  /* slots per priority band (rounded up to a power of two; 0, the
                                default: >= 2 x the tiles).  A band whose ring fills stops the
                                launch; eik_fim2d_solve then solves again with the FIFO.         */
    EIK_OPT_PRIO_DISPATCH = 18, /* band entries moved to the FIFO per dispatch, 1..128 (0, the
                                default: 128 on maps of >= 16384 tiles, else 16)                */
    EIK_OPT_EXACT_BAND = 19  /* biComputeTmap / rover path and fp64 FM3D early exits: 1 replays the
                                reference's sequential narrow band in pop order from the converged
                                fields (csrc/bidir_exact.hip): its tentative band values, its LIFO
                                order of equal T and so its nodeJoin / closed set, bit for bit; 0
                                (default) = band cells at their final (2D: relaxed) values (GPU <=
                                reference <= 1.03 x GPU), ties by node index / strict < T[start] */
} eik_option;

typedef enum { EIK_MODE_LIST = 0, EIK_MODE_PERSISTENT = 1 } eik_mode;

/* ---- context: replaces MotionPlanning::initPython / shutDownPython (MotionPlanning.cpp:5-29,
 *      :93-100) as the owner of solver state; one per host thread -------------------------- */
int eik_create(int device, eik_ctx** out);
void eik_destroy(eik_ctx* ctx);
const char* eik_last_error(const eik_ctx* ctx);
int eik_set_option(eik_ctx* ctx, int option, double value);
int eik_get_stats(const eik_ctx* ctx, eik_stats* out);
const char* eik_version(void);

/* ---- host-buffer drop-ins of FastMarching.py ------------------------------------------- */

/* computeTmap(costMap, goal, start) FastMarching.py:92-112 -> full arrival field T (the
 * reference raises at :107; this is its intended semantics with no early exit).
 * cost, T: H*W row-major.  f32: fp32 compute; f64: fp64 compute. */
int eik_tmap2d_f32(eik_ctx* ctx, const float* cost, int64_t H, int64_t W, int64_t gx, int64_t gy, float* T);
int eik_tmap2d_f64(eik_ctx* ctx, const double* cost, int64_t H, int64_t W, int64_t gx, int64_t gy, double* T);

/* biComputeTmap(costMap, goal, start) FastMarching.py:114-162 -> (TmapG, TmapS, nodeJoin).
 * nodeJoin is the first node popped by one front that the other front had already closed,
 * evaluated on the device from the two fields' pop ranks (the meeting iteration k).  TmapG/TmapS
 * are the fronts' PARTIAL fields at that iteration, as the reference returns them: the source and
 * its k first pops (rank <= k) and the narrow band around them at their values, +inf elsewhere
 * (fp64; band values relaxed and exact ties of T ranked by node index, or with EIK_OPT_EXACT_BAND
 * the reference's own band values, LIFO ties and nodeJoin). */
int eik_tmap2d_bidir_f64(eik_ctx* ctx, const double* cost, int64_t H, int64_t W, int64_t gx, int64_t gy,
                         int64_t sx, int64_t sy, double* TG, double* TS, uint32_t join[2]);

/* The join step of biComputeTmap alone (FastMarching.py:141-162) from two given FULL fields
 * TG (goal front) and TS (start front), H*W fp64 each (+inf = unreached): nodeJoin and the two
 * partial fields TGp / TSp, exactly as eik_tmap2d_bidir_f64 forms them after its solve.  members
 * (optional): the cells ranked per front -- the join bounds the meeting iteration first and sorts
 * only the cells under the bound (csrc/bidir.hip).  EIK_ERR_UNREACHABLE when no cell is finite in
 * both fields. */
int eik_bidir_join_f64(eik_ctx* ctx, const double* TG, const double* TS, int64_t H, int64_t W, double* TGp,
                       double* TSp, uint32_t join[2], int64_t members[2]);

/* How the last biComputeTmap / rover path formed its fronts: out[0] 1 = capped fronts, out[1] 1 =
 * the capped result was replaced by the full solve, out[2..3] cells kept under the caps (goal,
 * start front), out[4..5] cells the join ranked per front, out[6..7] band cells relaxed per front,
 * out[8..9] the band relaxation's sweeps per front. */
int eik_fronts_info(const eik_ctx* ctx, int64_t out[10]);

/* The last biComputeTmap / rover path's / FM3D early exit's exact band replay (EIK_OPT_EXACT_BAND): out[0] re-ranking
 * passes, out[1..2] relaxation sweeps (goal, start front), out[3] tie-run launches, out[4] its
 * device time in microseconds; all 0 when it did not run. */
int eik_exact_info(const eik_ctx* ctx, int64_t out[5]);

/* B independent maps (goal sweep / terrain Monte-Carlo): cost, T: B*H*W; goals: B x (x, y). */
int eik_tmap2d_batch_f32(eik_ctx* ctx, const float* cost, int64_t B, int64_t H, int64_t W, const int64_t* goals,
                         float* T);

/* getPathGDM(T, init, end, tau) FastMarching.py:164-236 on an fp64 field.
 * out: cap x 2 (x, y) rows; *n_out rows written; *status an eik_path_status. */
int eik_path2d_f64(eik_ctx* ctx, const double* T, int64_t H, int64_t W, const double init[2], const double end[2],
                   double tau, double* out, int64_t cap, int64_t* n_out, int* status);

/* computeGradient(T) FastMarching.py:242-300 (point = [] -> whole field): Gnx, Gny. */
int eik_gradient2d_f64(eik_ctx* ctx, const double* T, int64_t H, int64_t W, double* gnx, double* gny);

/* ---- host-buffer drop-ins of FastMarching3D.py ----------------------------------------- */

/* FastMarching3D.computeTmap :126-145 without its early exit -> the full field T (what the
 * reference returns when `start` is never popped).  cost, T: H*W*L row-major [y][x][z];
 * goal = (x, y, z). */
int eik_tmap3d_f32(eik_ctx* ctx, const float* cost, int64_t H, int64_t W, int64_t L, const int64_t goal[3], float* T);
int eik_tmap3d_f64(eik_ctx* ctx, const double* cost, int64_t H, int64_t W, int64_t L, const int64_t goal[3],
                   double* T);

/* FastMarching3D.computeTmap(costMap, goal, start) :126-145 as the planner calls it
 * (Coupled_motion_planner.py:1636): the loop breaks once `start` is popped (:141), so T is the
 * PARTIAL field -- cells popped before `start` (T < T[start]) and `start` at their final values,
 * the narrow band (finite cost, a closed 6-neighbour) at its converged full-field value -- <= the
 * reference's tentative value, which depends on its sequential update order --
 * and +inf elsewhere (eik_fim3d_early_exit).  fp64 with EIK_OPT_EXACT_BAND: the reference's own
 * closed set and band values, replayed in pop order (masks identical, values within 1e-11).
 * start == goal, a start outside the volume or an unreachable start -> the full field, as in the
 * reference (it never pops such a start). */
int eik_tmap3d_early_f32(eik_ctx* ctx, const float* cost, int64_t H, int64_t W, int64_t L, const int64_t goal[3],
                         const int64_t start[3], float* T);
int eik_tmap3d_early_f64(eik_ctx* ctx, const double* cost, int64_t H, int64_t W, int64_t L, const int64_t goal[3],
                         const int64_t start[3], double* T);

/* FastMarching3D.getPathGDM(T, init, end, tau) :198-271 on an fp64 field: out cap x 3 rows. */
int eik_path3d_f64(eik_ctx* ctx, const double* T, int64_t H, int64_t W, int64_t L, const double init[3],
                   const double end[3], double tau, double* out, int64_t cap, int64_t* n_out, int* status);

/* ---- device-resident solver (bench, multi-GPU domain decomposition, C++ hosts) ---------- */

/* A solver for B maps of H x W in `dtype`; owns the active lists, marks and counters. */
int eik_fim2d_create(eik_ctx* ctx, int64_t B, int64_t H, int64_t W, int dtype, eik_fim2d** out);
void eik_fim2d_destroy(eik_fim2d* fim);

/* Ghost strips for a subdomain of a decomposed raster (device pointers, NULL = +inf border):
 * north/south length W, west/east length H.  Values are min-merged by eik_fim2d_merge_ghost. */
/* A block of a domain-decomposed few-layer 3D volume ([H][W][L], layers z0 .. z0+nl-1 solved: the
 * layered solver; FastMarching3D.py:19-145 semantics; SURVEY §8(e) "C5: split x-y only, layers stay
 * together").  The handle is an eik_fim2d: eik_fim2d_set_ghosts (strips of nl values per edge cell,
 * [i][z]), eik_fim2d_iterate (one persistent launch to local convergence), eik_fim2d_pack_edges,
 * eik_fim2d_merge_ghost, eik_fim2d_active, eik_fim2d_stats and eik_fim2d_destroy apply; start with
 * eik_fim3dl_start (goal (x, y, z), z absolute; x < 0: the goal is in another block). */
int eik_fim3dl_create(eik_ctx* ctx, int64_t H, int64_t W, int64_t L, int z0, int nl, int dtype, eik_fim2d** out);
int eik_fim3dl_start(eik_fim2d* f, const void* d_cost, void* d_T, const int64_t goal[3], void* stream);

/* Diagnostics: the queue counters of the solver's last persistent launch (builds with -DEIK_QDEBUG=1:
 * FIFO claims, stale FIFO entries, band dispatches, decrease-key entries, band puts at out[3..7];
 * zeros otherwise).  tools/prio_probe.py. */
int eik_fim2d_qcount(const eik_fim2d* f, uint64_t out[8]);

int eik_fim2d_set_ghosts(eik_fim2d* fim, void* north, void* south, void* west, void* east);

/* Bind device cost/T (B*H*W of dtype), set T = inf, T[goal] = 0, seed the goal tiles.
 * goals: host array B x (x, y); a goal outside the map seeds nothing (subdomain w/o goal). */
int eik_fim2d_start(eik_fim2d* fim, const void* d_cost, void* d_T, const int64_t* goals, void* stream);

/* Run up to max_iters outer iterations (stops early when no tile is active); *active gets the
 * number of tiles active for the next iteration (synchronises the stream). */
int eik_fim2d_iterate(eik_fim2d* fim, int64_t max_iters, int64_t* active);

/* start + iterate to convergence (synchronous). */
int eik_fim2d_solve(eik_fim2d* fim, const void* d_cost, void* d_T, const int64_t* goals, void* stream);

/* Halo exchange helpers (async on the bound stream): copy edge rows/columns of T into send
 * strips; min-merge a received strip into ghost `side` (0 N, 1 S, 2 W, 3 E) and activate the
 * edge tiles whose ghost decreased. */
int eik_fim2d_pack_edges(eik_fim2d* fim, void* north, void* south, void* west, void* east);
int eik_fim2d_merge_ghost(eik_fim2d* fim, int side, const void* recv);
/* number of tiles active for the next iteration (synchronises the stream) */
int eik_fim2d_active(eik_fim2d* fim, int64_t* active);
/* statistics of the current/last solve (synchronises the stream to read the visit counter) */
int eik_fim2d_stats(eik_fim2d* fim, eik_stats* out);

/* Live domain decomposition (no reference counterpart: the multi-GPU split of SURVEY.md §8(e)).
 * eik_fim2d_launch(fim, 1) starts ONE persistent launch on the bound stream and returns at once.
 * Its last workgroup is a halo agent serving a pinned host mailbox while the others solve; the
 * launch keeps serving its tile FIFO -- idle included -- until eik_fim2d_release.  Per round:
 *   live_pack(p)   the agent snapshots "tiles pending or busy", then stores the four edges of T
 *                  into send[p][side] (the neighbours' receive strips, e.g. eik_ipc_open'ed)
 *   (host barrier: every rank has packed)
 *   live_merge(p)  the agent min-merges recv[p][side] into the ghosts and queues the edge tiles
 *                  whose ghost dropped; *active = the pack's snapshot, *changed = ghosts lowered
 * The raster is converged when, in one round, every rank reports active == 0 and changed == 0.
 * eik_fim2d_live_bind sets the strips (index parity * 4 + side, NULL = no neighbour) before the
 * launch.  live = 0 is one ordinary persistent launch without the trailing synchronisation. */
int eik_fim2d_live_bind(eik_fim2d* fim, void* const send[8], void* const recv[8]);
int eik_fim2d_launch(eik_fim2d* fim, int live);
int eik_fim2d_live_pack(eik_fim2d* fim, int parity);
int eik_fim2d_live_merge(eik_fim2d* fim, int parity, int64_t* active, int64_t* changed);
/* end the live launch: wait for it on the bound stream; *active = tiles left (0 when converged) */
int eik_fim2d_release(eik_fim2d* fim, int64_t* active);

/* Sum of one integer over the `world` ranks of one node, through a shared-memory segment of
 * 64 * world bytes (zeroed before first use); round = 1, 2, ... on every rank in step.  Returns
 * EIK_ERR_HIP after timeout_s without the others.  (Per-round vote of the live decomposition.) */
int eik_node_allreduce(void* shm, int rank, int world, uint64_t round, int64_t value, int64_t* sum, double timeout_s);
/* the segment: POSIX shm `name` of `bytes` (create != 0: new and zeroed), mapped at *addr */
int eik_node_shm_open(const char* name, int64_t bytes, int create, void** addr);
int eik_node_shm_close(void* addr, int64_t bytes);
int eik_node_shm_unlink(const char* name);

/* Page-locked host memory for the drop-in's returned fields (FastMarching.computeTmap, ...): the
 * host entry points copy a registered pinned buffer as ONE DMA at PCIe speed instead of through
 * their staging ring (host threads memcpy'ing 8 MiB chunks), e.g. a field returned by
 * eik_tmap2d_f64 and handed back to eik_path2d_f64.  Thread-safe; no context needed. */
int eik_host_alloc(int64_t bytes, void** out);
int eik_host_free(void* p);

/* Device buffers shared between the processes of one node (hipIpc handles, 64 bytes). */
int eik_ipc_alloc(eik_ctx* ctx, int64_t bytes, void** d_ptr, unsigned char handle[64]);
int eik_ipc_free(eik_ctx* ctx, void* d_ptr);
int eik_ipc_open(eik_ctx* ctx, const unsigned char handle[64], void** d_ptr);
int eik_ipc_close(eik_ctx* ctx, void* d_ptr);

/* Self-test (no reference counterpart): the 2D path kernel's fast-path f64 square root,
 * division and interpolation against the exact forms they replace, on n pseudo-random inputs
 * each from their domain (gdm.hip walker_math_selftest_kernel); counts[0..2] = mismatches of
 * each (0 expected), counts[3] = samples evaluated (n), counts[4] = mismatches of the division
 * taken from the square root's reciprocal (path loop forms 3-4), counts[5] = mismatches of the
 * one-correction square root (form 4); 0 expected in both. */
int eik_selftest_walker_math(eik_ctx* ctx, int64_t n, uint64_t seed, int64_t counts[6]);

/* getPathGDM on a device-resident field; out/n_out/status are device pointers. */
int eik_path2d_dev(eik_ctx* ctx, const void* d_T, int dtype, int64_t H, int64_t W, const double init[2],
                   const double end[2], double tau, double* d_out, int64_t cap, int64_t* d_n_out, int* d_status,
                   void* stream);

/* 3D solve on device buffers (synchronous: returns after convergence; stats via
 * eik_get_stats). */
int eik_fim3d_solve(eik_ctx* ctx, const void* d_cost, void* d_T, int64_t H, int64_t W, int64_t L, int dtype,
                    const int64_t goal[3], void* stream);

/* FastMarching3D.computeTmap's early exit at `start` (:141) on device buffers: d_T (a converged
 * full field from eik_fim3d_solve) -> d_Te (a different buffer), async on `stream`. */
int eik_fim3d_early_exit(eik_ctx* ctx, const void* d_cost, const void* d_T, void* d_Te, int64_t H, int64_t W,
                         int64_t L, int dtype, const int64_t goal[3], const int64_t start[3], void* stream);

/* FastMarching3D.getPathGDM on a device-resident field. */
int eik_path3d_dev(eik_ctx* ctx, const void* d_T, int dtype, int64_t H, int64_t W, int64_t L, const double init[3],
                   const double end[3], double tau, double* d_out, int64_t cap, int64_t* d_n_out, int* d_status,
                   void* stream);

/* ---- cost-raster builder (the solver's input producer) ----------
 * Coupled_motion_planner.py main(), :1101-1216: DEM -> surface normals -> slope obstacles ->
 * hole filling, disk erode/dilate -> 300 x obstacle + 10 x distance ramp -> 50 x 50 box blur ->
 * +inf border.  Constants default to the reference's (slope 0.20 rad, rover diagonal 0.9 m,
 * expansion 1 m, gradient 10, obstacle cost 300) when params is NULL. */
typedef struct {
    double slope_max;  /* rad, :1154 */
    double diagonal;   /* m, rover body diagonal (corridor erosion radius = diagonal / 2), :1172 */
    double expansion;  /* m, obstacle cost ramp radius, :1190 */
    double gradient;   /* ramp cost scale, :1202 */
    double high;       /* obstacle cost, :1187 */
} eik_costmap_params;

/* Z: H x W DEM (row-major, Zs of :1098-1101, spacing size / (n - 1) as linspace(0, size, n)).
 * cost_out: H x W, [y][x] -- the reference's cMap.T, i.e. the array it passes to
 * FM.biComputeTmap (:1222); obst_out (nullable): the final obstacle map (:1180-1184), 0/1. */
int eik_costmap_f64(eik_ctx* ctx, const double* Z, int64_t H, int64_t W, double resolution, double size,
                    const eik_costmap_params* params, double* cost_out, uint8_t* obst_out);
/* the same on device buffers, async on `stream` except the two hole-filling solves */
int eik_costmap_dev(eik_ctx* ctx, const double* d_Z, int64_t H, int64_t W, double resolution, double size,
                    const eik_costmap_params* params, double* d_cost, uint8_t* d_obst, void* stream);
/* surface_normal(resolution, size, z) :37-80 -> unit normals (H x W each) */
int eik_surface_normal_f64(eik_ctx* ctx, const double* Z, int64_t H, int64_t W, double size, double* Nx, double* Ny,
                           double* Nz);
/* image_filling(im) :82-94 (cv2.floodFill from (0, 0), 4-connected) on a 0/1 uint8 image */
int eik_image_fill_u8(eik_ctx* ctx, const uint8_t* im, int64_t H, int64_t W, uint8_t* out);
/* cv2.erode / cv2.dilate with the reference's structural_disk(radius) (Coupled_motion_planner.py:96-105,
 * :1168-1177, :1192) on a 0/1 uint8 mask: erode != 0 -> erosion; pixels outside the image take no part. */
int eik_disk_morph_u8(eik_ctx* ctx, const uint8_t* im, int64_t H, int64_t W, int radius, int erode, uint8_t* out);

/* ---- rover path of the planner -----------------------------------
 * Coupled_motion_planner.py main(), step 1 (:1097-1258): DEM -> cost raster (eik_costmap_*) ->
 * biComputeTmap(cMap.T, sample node, rover node) -> getPathGDM from nodeJoin to each end ->
 * roverPath = [flipud(pathS); pathG[1:]] in metres (res * (p + 1)), waypoints within 0.1 m of the
 * rover or the sample dropped, z = zp + Zs[round(y / res), round(x / res)], heading =
 * [initialHeading, atan2(dy, dx)...].  Nodes: pxm = int(round(xm / res - 1)) etc. (:1107-1117,
 * Python's round: half to even).  Defaults of the reference: zp 0.07 (:1132), tau 0.5 (:1225). */
typedef struct {
    double xm, ym;            /* sample position (m), :1107-1108                                 */
    double xr, yr;            /* rover position (m), :1115-1116                                  */
    double initial_heading;   /* rad, :1254                                                      */
    double resolution, size;  /* DEM spacing (m) and side (m) as main()'s arguments              */
    double zp;                /* height of the rover reference system above the floor, :1132     */
    double tau;               /* GDM step (cells), :1225-1226                                    */
} eik_rover_query;

/* Host-only tail of step 1 (no GPU, no context): from the two GDM paths (K x 2 cell coordinates,
 * pathS from nodeJoin to the rover node, pathG from nodeJoin to the sample node) and the DEM Z
 * (H x W, raw heights: the min shift of :1101 is applied here) to path_xyz (cap x 3, metres) and
 * heading (cap).  *n_out = rows written; EIK_ERR_ARG if cap is too small or a waypoint falls
 * outside Z (the reference raises IndexError there). */
int eik_rover_assemble(const double* pathS, int64_t nS, const double* pathG, int64_t nG, const double* Z, int64_t H,
                       int64_t W, const eik_rover_query* q, double* path_xyz, double* heading, int64_t cap,
                       int64_t* n_out);

/* The whole of step 1 on the GPU: cost raster, both fronts as one 2-map fp64 batch, the device
 * join, the two path kernels, then eik_rover_assemble on the host.  Z: H x W host DEM.  join
 * (nullable) receives nodeJoin; cost_out (nullable, H x W [y][x]) the cost raster.
 * EIK_ERR_UNREACHABLE when the rover cannot reach the sample. */
int eik_rover_path_f64(eik_ctx* ctx, const double* Z, int64_t H, int64_t W, const eik_rover_query* q,
                       const eik_costmap_params* params, double* path_xyz, double* heading, int64_t cap,
                       int64_t* n_out, uint32_t join[2], double* cost_out);

/* ---- end-effector cost volume of the planner ---------------------
 * Coupled_motion_planner.py main(), step 3 (:1462-1593): the arm's FM3D runs on
 * Cmap = GetObstMap(...)[0] * TunnelCost(...) over a small square area around the sample.  The
 * volume is [iy][ix][iz], sY x sX x sZ with sX == sY (the planner's area is square, :1519). */
typedef struct {
    int64_t sX, sY, sZ;              /* nodes per axis, :1528-1529                                 */
    double resX, resY, resZ;         /* m per node, :1532-1534                                     */
    double xm, ym;                   /* GetObstMap's sample test: columns with resX*i == xm or
                                        resY*j == ym are skipped (:329; the planner passes the
                                        global sample position)                                    */
    double rlim, rO, rm;             /* TunnelCost(Rlim, rO, rm, ...), :1577 (Rlim, rO, rm :1121-1124) */
    uint32_t final_wp[3];            /* sample node (x, y, z), :1574                                */
    uint32_t initial_wp[3];          /* end-effector start node (x, y, z), :1573                    */
} eik_arm_volume;

/* GetObstMap(ZsMap, resX, resY, resZ, sX, sY, sZ, newObstMap, xm, ym) :319-358.  ZsMap, newObstMap:
 * m x n (row j = y).  finalMap (2 / +inf), obstMap and groundMap (1 / +inf; nullable): sX*sY*sZ. */
int eik_arm_obst_map_f64(eik_ctx* ctx, const double* ZsMap, const double* newObstMap, int64_t m, int64_t n,
                         const eik_arm_volume* vol, double* finalMap, double* obstMap, double* groundMap);

/* TunnelCost(rlim, rO, rm, gamma2D, sX, sY, sZ, resX, resY, resZ, finalBaseHeading, finalWayPointArm,
 * initialWayPointArm) :505-725.  gamma2D, heading: npts x 3 (arm base positions in the area's frame,
 * (roll, pitch, yaw) per point).  Cmap: sY*sX*sZ (10 / tunnel cost / +inf), bit-identical to the
 * reference (tests/golden/arm.npz). */
int eik_arm_tunnel_cost_f64(eik_ctx* ctx, const double* gamma2D, const double* heading, int64_t npts,
                            const eik_arm_volume* vol, double* Cmap);

/* :1562-1593 on the GPU: Cmap = finalMap * tunnel on the device -> FM3D.computeTmap(Cmap,
 * finalWayPointArm, initialWayPointArm) -> FM3D.getPathGDM(T, initialWayPointArm, finalWayPointArm,
 * tau) -> path (cap x 3 node coordinates, before the planner's scaling and smoothing, :1588-1598).
 * The field is computeTmap's early-exit field at initialWayPointArm (eik_tmap3d_early_f64).
 * cost_out / T_out (nullable): the volume and that arrival field, sY*sX*sZ. */
int eik_arm_path_f64(eik_ctx* ctx, const double* ZsMap, const double* newObstMap, int64_t m, int64_t n,
                     const double* gamma2D, const double* heading, int64_t npts, const eik_arm_volume* vol, double tau,
                     double* path, int64_t cap, int64_t* n_out, int* status, double* cost_out, double* T_out);

/* FastMarching3D.computeTmap on B independent volumes of one shape in ONE solve (candidate fetch
 * poses): cost, T: B*H*W*L; goals: B x (x, y, z). */
int eik_tmap3d_batch_f64(eik_ctx* ctx, const double* cost, int64_t B, int64_t H, int64_t W, int64_t L,
                         const int64_t* goals, double* T);

/* ---- DEM ingest, host only: no GPU, no context --------------------
 * Coupled_motion_planner.py:1098-1099 reads PRL_DEM.txt as comma-separated rows with a Python
 * float() per value.  eik_load_dem_txt parses the same text with host threads (nthreads <= 0:
 * all cores), bit-identical values (correctly rounded parsing).  out == NULL: only H, W.
 * Errors: EIK_ERR_ARG, message from eik_io_last_error(). */
int eik_load_dem_txt(const char* path, double* out, int64_t cap, int64_t* H, int64_t* W, int nthreads);
const char* eik_io_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* EIKONAL_H_ */
