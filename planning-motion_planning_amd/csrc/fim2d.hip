// fim2d.hip -- block Fast Iterative Method for the 2D Eikonal cost-to-go (gfx950 / CDNA4).
//
// Replaces the reference's sequential Fast Marching wavefront (FastMarching.py:44-162: a
// Python narrow band kept sorted with bisect) by a tile-parallel FIM whose fixed point is the
// same discrete Godunov solution (the reference FMM equals the
// Jacobi fixed point to 1e-13):
//
//  * the raster is cut into 64x64 tiles; one workgroup (4 x wave64) per tile visit stages
//    cost + T (+1-cell halo) in LDS and runs four concurrent quadrant sweeps (one per wave).
//    Each sweep is Gauss-Seidel along skewed anti-diagonals (lane l = column, step s = row
//    s-l): the upstream x value comes from lane l-1 through a DPP wave shift, the upstream y
//    value from the lane's own previous step, so one round propagates any characteristic in
//    that quadrant across the tile;
//  * updates are monotone min-updates merged with ds_min, so racing waves and stale halos of
//    concurrently processed tiles only delay convergence;
//  * a tile whose values changed is revisited; a tile whose edge values undercut a neighbour's
//    adjacent cell activates that neighbour.
//
// Two drivers share the tile body:
//  * LIST mode (fim2d_sweep_kernel): one launch per outer iteration over a device-side active
//    list (triple-buffered, dedup by per-tile marks); kernel boundaries order all memory.
//  * PERSISTENT mode (fim2d_persist_kernel): ONE launch per solve.  Workgroups take tickets
//    from a device FIFO of tiles and process a tile as soon as it is activated -- no launch
//    gaps, no waiting for the slowest tile of an iteration.  Hand-offs follow the gfx950 recipe
//    for in-launch visibility (cdna_hip_programming.md Guideline 16, with sc1 loads): every
//    T store is write-through (sc1) and drained (s_waitcnt vmcnt(0) in every storing wave,
//    then a workgroup barrier) before the activating atomics; every T load is an sc1 load.
//    A per-tile state word (PENDING / BUSY) deduplicates the queue and defers activations of a
//    busy tile to its finish; a counter of non-idle tiles detects termination; every spin is
//    bounded by a wall-clock timeout that raises an error flag instead of hanging.
//
// The same kernels serve B independent maps (tile id = map * tiles_per_map + tile) and a
// subdomain of a domain-decomposed raster (ghost strips N/S/W/E stand in for out-of-range
// neighbours; edge activations are flagged for the halo exchange).
#include "fim_engine.hpp"

namespace eik {

// A cost as the sweep keeps it in LDS.  fp64 with EIK_CHAIN: at least 2^-500, the domain of the
// step's square root without a range clamp on its chain (eik_common.hpp sqrt_sweep); a zero-cost
// cell then rises by at most 2^-500 over its upstream value, far below the 1e-9 field tolerance.
template <typename R>
__device__ __forceinline__ R stage_cost(R c) {
    // (only finite non-negative small costs: NaN and negative costs keep their own paths -- a NaN
    // cost is never updated, i.e. blocked, as without the clamp)
    if constexpr (sizeof(R) == 8 && EIK_CHAIN) return (c >= R(0) && c < 0x1p-500) ? R(0x1p-500) : c;
    else return c;
}

// EIK_EDGE_FIRST (see the write-back in process_tile): measured and OFF -- C2 2-7 % slower in fp64
// and fp32 (profiles/r03l_edge_first_ab.log), and C3 / C4 3-8 % slower (round 4,
// profiles/r04u_edge_first_throughput_ab.log): the drain before the activations is latency, not the
// number of stores, and the extra per-visit barrier and edge-column stores cost more than it saves.
#ifndef EIK_WB_LINE
#define EIK_WB_LINE 0
#endif
#ifndef EIK_EDGE_FIRST
#define EIK_EDGE_FIRST 0
#endif

// EIK_ACT_SPLIT (persistent in-place passes, default on): the neighbour activations' state-word
// atomics are issued at the pass boundary and their queueing is finished by wave 0 when its next
// sweep reaches step kActStep (fim_engine.hpp qpush_issue / qpush_complete), so no wave waits for
// their round trips at the boundary's barrier: the other three waves start sweeping at once.
// C2 fp64 2.37-2.42 -> 2.28-2.32 ms, fp32 1.66-1.69 -> 1.56 ms; step 0 (at the sweep's start)
// ties 4 and beats 8 / 16, which delay the neighbour's queueing (profiles/r03zz_act_split_ab.log).
// (EIK_ACT_SPLIT: fim_engine.hpp)
#ifndef EIK_ACT_STEP
#define EIK_ACT_STEP 0
#endif
constexpr int kActStep = EIK_ACT_STEP;

// (EIK_LAZY_CLAIM, round 4: a grabbed tile claimed -- PENDING -> BUSY -- at its first pass boundary
// instead of before its staging, taking the grab's exchange round trip off the front's hop; the
// first boundary then has to reload the halo to tell new activations from the served ones.
// Measured and removed: C2 fp64 2.34-2.37 -> 2.38-2.39 ms, C3 / C4 within noise,
// profiles/r04f_lazy_claim_ab.log.)
// (Also measured in round 4 and removed, profiles/r04d_follow_split_ab.log: EIK_FOLLOW -- a workgroup
// whose pass made a FRESH neighbour reachable claimed it and continued with it, skipping the queue's
// round trips; and EIK_SPLIT_WB -- two waves stored the write-back without waiting while two
// reloaded the halo, the activations following the drain from inside the next sweep.  Both did 2-5x
// the tile visits (C2 fp64 2.35 -> 3.3-6.8 ms, C4 at one GPU 11 -> 0.6-4.7 Gcells/s): tiles reached
// ahead of the FIFO's order converge against incomplete halos and are revisited, and a delayed
// activation costs the same.  The FIFO's breadth-first order is worth more than the hops it costs.)
// (EIK_ASYNC_WB, round 4: the pass boundary's write-back drain moved into the next sweep -- every
// wave waiting for its own stores mid-sweep, wave 0 activating the neighbours once all four had
// drained, wave 1 consuming activations and reloading the halo ring mid-sweep.  Measured and
// removed: C2 fp64 2.36 -> 3.3-4.0 ms for every choice of steps, tile visits +40-120 %
// (profiles/r04c_async_wb_ab.log).  The drain is the front's hop either way -- a neighbour may be
// activated only once the edge it reads has landed.)

// (Round 5, measured on one box against this schedule and removed -- code in commit f3e04a5:
//  * EIK_WB_ONCE: a pass stored only the first / last rows and the edge-column copies, the interior
//    rows once when the visit ended (a 64-bit sum of the cells' bit patterns told a pass that changed
//    them).  PMC writes would fall ~8x, but C2 fp64 2.39-2.41 -> 2.52-2.58 ms, C3 -6 %, C4 -8 %
//    (profiles/r05a_wb_once_ab.log): the per-pass drain is latency, not bytes, and the interior's
//    drain moved onto the visit's finish.
//  * EIK_EARLY_AND: the activation consumption issued by wave 0 at sweep step 96 (or 64) so that the
//    halo reload could overlap the write-back's drain.  C2 fp64 2.38-2.41 -> 2.85-2.91 ms, visits
//    +20 %, in-place passes +19 % (profiles/r05b_early_and_ab.log): activations arriving in the
//    sweep's last steps were no longer served in place and came back as full visits.)

// EIK_ECOL_F64 / _F32 (kEcol): the W / E halo columns of a visit come from Fim2dArgs::ecol, a copy of every tile's two
// edge columns stored beside T by the write-back (and the init / seed kernels), instead of from T:
// a column of T spans 64 rows, i.e. 64 lines of 64-128 B for 256-512 B of data (the fp64 solve's
// reads were 1.01 GB per launch against 0.58 GB algorithmic, profiles/r03s_pmc_traffic_f64.json).
// Per dtype: on in fp64 (C2 within noise, 2.36-2.44 vs 2.37-2.41 ms; PMC traffic per launch 2.94 ->
// 2.56 GB, reads 0.88 -> 0.45 GB: profiles/r04j_ecol_ab.log), off in fp32 (C2 1.60-1.63 -> 1.65-1.66 ms:
// the 147 -> 164 VGPRs of the one-wave kernel, profiles/r04k_ecol_f32_ab.log).
#ifndef EIK_ECOL_F64
#define EIK_ECOL_F64 1
#endif
#ifndef EIK_ECOL_F32
#define EIK_ECOL_F32 0
#endif
template <typename R>
constexpr bool kEcol = sizeof(R) == 8 ? EIK_ECOL_F64 : EIK_ECOL_F32;

// EIK_FRESH_SKIP: a persistent visit of a tile no visit has written yet (its grab's exchange
// returns the state without kVisited) stages only the cost: its T is the init kernel's +inf.
// Between a solve's init and its end, the only writers of a full tile's T outside a visit are the
// init kernel and the seed kernel, and the seed kernel queues its tile as visited (the kernels that
// rewrite T afterwards -- bidir.hip's partial fields and cap clean-up -- run after the solve, and
// the next solve starts with the init).  (Cut tiles, whose ghost cells come from load_T, always
// read T.)
#ifndef EIK_FRESH_SKIP
#define EIK_FRESH_SKIP 1
#endif
constexpr bool kFreshSkip = EIK_FRESH_SKIP;

// ------------------------------------------------------------------------- quadrant sweep
// A tile cell in LDS: arrival time and cost side by side, so one ds_read_b64 (fp32) fetches both.
template <typename R>
struct alignas(2 * sizeof(R)) Cell {
    R t, c;
};

// LDS bank swizzle (EIK_SWZ, default OFF -- measured below): a cell of an LDS column with bit 4 set holds (cost, T)
// instead of (T, cost).  The sweeps' T-only accesses (ds_min, the upstream-x read, the start-row
// read) of a skewed anti-diagonal put lane l at byte -(kLds - 1) * sizeof(Cell) * l from lane 0:
// with T always the cell's first half that is bank -2l mod 32 (fp32, b32 banking) / -4l mod 64
// (fp64, b64), so lanes l and l + 16 -- in the same 32-lane group -- collide on every step (53 %
// of the sweep's LDS cycles were conflict cycles, profiles/r02_sq_counters.json).  Their columns
// always differ in bit 4, so with the swap one of the two reads the other half of its cell: every
// T access of a step is conflict-free.  Every LDS accessor of a tile cell goes through these.
// Measured and OFF by default (profiles/r03h_swizzle_ab.log, r03h_sq_counters_swizzle_ab.json): the
// swapped halves cost a third ds_read per step (T and cost can no longer come in one b64 / b128
// read), LDS instructions +33 %; the conflict share fell 0.53 -> 0.30 (fp32) / 0.48 -> 0.42 (fp64),
// but C2 got 2-4 % slower -- the conflicted accesses are off the step's dependency chain (reads
// prefetched 4 steps ahead, ds_min not waited on), so their extra cycles were hidden anyway.
#ifndef EIK_SWZ
#define EIK_SWZ 0
#endif
__device__ __forceinline__ constexpr int cell_swz(int col) { return EIK_SWZ ? (col >> 4) & 1 : 0; }
template <typename R>
__device__ __forceinline__ R& cell_t(Cell<R>* Ts, int idx, int col) {
    return reinterpret_cast<R*>(Ts + idx)[cell_swz(col)];
}
template <typename R>
__device__ __forceinline__ R& cell_c(Cell<R>* Ts, int idx, int col) {
    return reinterpret_cast<R*>(Ts + idx)[1 - cell_swz(col)];
}
template <typename R>
__device__ __forceinline__ Cell<R> make_cell(R t, R c, int col) {
    return cell_swz(col) ? Cell<R>{c, t} : Cell<R>{t, c};
}

// One quadrant sweep of the staged tile.  DX/DY = +-1: direction of propagation.
// Lane l owns column x; at step s it updates row r = s - l (skewed Gauss-Seidel), so its
// upstream x neighbour is lane l-1's previous result (DPP) and its upstream y neighbour its own.
// Each quadrant sweep reads only its UPSTREAM neighbours: the four concurrent sweeps together
// evaluate the local solve on every combination of one x and one y neighbour, and since the
// Godunov update is monotone in both, the smallest of those four is the update on the two minima
// -- the same fixed point as reading both neighbours per axis in every sweep (tools/sched_sim.c:
// identical field, +1 % passes on the 4096^2 DEM), for 2 LDS reads per step instead of 5 (the
// sweep is LDS-bound at three workgroups per CU: 14 -> 8 LDS cycles per wave-step).
// Branch- and select-free: the LDS row is clamped once per group of kAhead steps (one add + one
// med3 per group, immediate offsets per step); the rows a lane outside the tile reaches are halo
// and guard rows, whose cost is +inf, so it computes +inf or NaN and its ds_min / min / `<` are
// no-ops.  TRACK: also report whether any cell decreased by
// more than the tolerance (only needed for multi-round visits; single-round visits read it off
// the write-back).
// Software pipeline depth of a sweep: the LDS reads of step s + kAhead are issued at step s,
// so the ~100-cycle LDS round trip overlaps kAhead steps of the Godunov chain instead of being
// exposed once per step.  Reading ahead is safe: a lane's own column is written only by itself
// within this sweep, and the upstream-x value of lanes 1..63 comes from the DPP register path (the
// LDS upstream-x read serves lane 0, whose upstream column is the halo, which no sweep writes).
// Another wave's concurrent ds_min may make a pre-read value stale (larger): that only delays
// convergence -- a visit whose sweeps changed nothing had no concurrent writes, so its reads
// were exact.
// (kAhead, fim_engine.hpp.)  Guard rows (kGuard, +inf T and cost) above and below the tile's halo
// ring in LDS: a sweep clamps its LDS row once per group of kAhead steps -- the group's lowest row
// into [-(kAhead - 1), kTile + 1] -- and addresses the group's steps with immediate offsets, so a
// group of a lane outside its window may reach kAhead - 1 rows past a halo row.

// EIK_SWEEP_UNROLL: groups of kAhead steps per loop iteration (one back-branch per iteration).
// The taken back-branch is paid on every step group of the sweep's dependent chain: 1 -> 2 -> 4
// groups per iteration took C2 fp64 2.35 -> 2.25 -> 2.23 ms, C2 fp32 1.63 -> 1.57 ms, C3 fp64 +4 %
// (profiles/r05n_sweep_unroll_ab.log, r05o_sweep_unroll_248_ab.log); 8 loses in fp64.
#ifndef EIK_SWEEP_UNROLL
#define EIK_SWEEP_UNROLL 4  // fp64
#endif
#ifndef EIK_SWEEP_UNROLL_F32
#define EIK_SWEEP_UNROLL_F32 8  // C4 fp32 +3 %, C2 / C3 within noise (profiles/r05v_sweep_unroll_f32_ab.log)
#endif
// REF (fp64, EIK_OPT_EXACT_BAND's fronts): the step in the reference's own getEikonal arithmetic
// (eik_ref) instead of the chain form, so the converged field is the reference's closed values bit
// for bit wherever its last update read the same upwind minima (bidir_exact.hip starts from it)
template <typename R, int DX, int DY, bool TRACK, bool REF = false, class Hook>
__device__ __forceinline__ bool sweep_quadrant(Cell<R>* __restrict__ Ts, int lane, R keep, Hook&& hook) {
    constexpr int S = (int)sizeof(Cell<R>);
    constexpr int kRow = kLds * S;
    constexpr int D = kAhead;
    static_assert((2 * kTile) % D == 0, "pipeline depth must divide the step count");
    char* const base = reinterpret_cast<char*>(Ts);
    const int col = (DX > 0 ? lane : kTile - 1 - lane) + 1;
    // step s: tile row r = s - lane -> LDS row (DY > 0 ? r + 1 : 64 - r).  A group of D steps
    // covers D consecutive rows; its LOWEST row (step s going south, s + D - 1 going north) is
    // clamped into [-(D - 1), 65] once per group and its steps are immediate offsets from it:
    // while the lane's window lies ahead the group reads guard rows and ends on the start-side
    // halo row (cur = its T, as the per-step clamp gave); past the window it reads the far halo
    // and guard rows (cost +inf: no update).  Within the window the rows are exact.
    // byte offsets within a row: this lane's T, its cost relative to it, and the upstream column's T
    constexpr int RB = (int)sizeof(R);
    const int colT = col * S + cell_swz(col) * RB;
    const int dC = (1 - 2 * cell_swz(col)) * RB;
    const int dU = (col - DX) * S + cell_swz(col - DX) * RB - colT;
    const int lo_b = -(D - 1) * kRow + colT, hi_b = (kLds - 1) * kRow + colT;
    int raw = DY > 0 ? (1 - lane) * kRow + colT : (kTile - (D - 1) + lane) * kRow + colT;
    auto off = [](int u) { return (DY > 0 ? u : D - 1 - u) * kRow; };
    auto clampb = [&](int x) {  // one v_med3_i32 (the compiler emits min + cmp + cndmask)
        int r;
        asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(lo_b), "v"(hi_b));
        return r;
    };
    bool changed = false;
    // the upstream halo row value is the lane's "previous row" result before it starts
    R cur = *reinterpret_cast<const R*>(base + (DY > 0 ? 0 : kLds - 1) * kRow + colT);
    R q_old[D], q_upx[D], q_c[D];
    int gb = clampb(raw);  // lowest row of the group being fetched (byte offset from Ts)
    raw += DY * D * kRow;
    auto fetch = [&](int u) {
        const int o = gb + off(u);
#if EIK_SWZ
        q_old[u] = *reinterpret_cast<const R*>(base + o);
        q_c[u] = *reinterpret_cast<const R*>(base + o + dC);
#else
        const Cell<R> v = *reinterpret_cast<const Cell<R>*>(base + o);  // one ds_read_b64 / b128
        q_old[u] = v.t;
        q_c[u] = v.c;
#endif
        q_upx[u] = *reinterpret_cast<const R*>(base + o + dU);
    };
#pragma unroll
    for (int u = 0; u < D; ++u) fetch(u);
    constexpr int kUnroll = sizeof(R) == 8 ? EIK_SWEEP_UNROLL : EIK_SWEEP_UNROLL_F32;
#pragma unroll kUnroll
    for (int s = 0; s < 2 * kTile; s += D) {
        hook(s);  // per group: the in-sweep duties of the persistent driver (process_tile)
        const int gcur = gb;  // this group's rows (its ds_min targets)
        gb = clampb(raw);     // the next group's (past the last step: guard / halo rows, unused)
        raw += DY * D * kRow;
#pragma unroll
        for (int u = 0; u < D; ++u) {
            // x side: lane 0 takes the halo column; lanes 1.. take lane l-1's fresh value (DPP)
            // -- the prefetched LDS value of that cell is a valid, possibly stale, upper bound, so
            // one v_min_u32_dpp serves both (lane 0, whose shift source is out of range, keeps
            // the LDS value); the chain to w is godunov2_chain's (see there)
            const R c2x2 = R(2) * (q_c[u] * q_c[u]);
            R w;
            if constexpr (sizeof(R) == 8) {
                // fp64: the DPP move cannot fold into a 64-bit min, so lanes 1.. take lane l-1's
                // fresh value alone (it is at most the prefetched LDS value of the same cell, read
                // one step earlier) and lane 0 keeps the halo column's LDS value (the DPP's old)
                if constexpr (REF) w = eik_ref(wave_shr1(cur, q_upx[u]), cur, q_c[u]);
                else w = godunov2_chain(wave_shr1(cur, q_upx[u]), cur, q_c[u], c2x2);
                lds_min(reinterpret_cast<R*>(base + gcur + off(u)), w);
                if constexpr (TRACK) changed |= w < q_old[u] * keep;
                cur = fmin_nn(w, q_old[u]);  // NaN (both-inf case): keeps old
            } else {
                w = godunov2_chain(umin(wave_shr1_umin_id(cur), q_upx[u]), cur, q_c[u], c2x2);
                lds_min(reinterpret_cast<R*>(base + gcur + off(u)), w);
                if constexpr (TRACK) changed |= w < q_old[u] * keep;
                cur = umin(w, q_old[u]);  // NaN (both-inf case) sorts above every value: keeps old
            }
            fetch(u);  // refill the slot: step s + u + D (past the last step: clamped halo rows)
            // keep each step's instructions in place: hoisting a later step's use of a slot
            // above this point would make the compiler wait for the newest reads (lgkmcnt(0))
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    return changed;
}
template <typename R, int DX, int DY, bool TRACK, bool REF = false>
__device__ __forceinline__ bool sweep_quadrant(Cell<R>* __restrict__ Ts, int lane, R keep) {
    return sweep_quadrant<R, DX, DY, TRACK, REF>(Ts, lane, keep, [](int) {});
}

// LDS of one tile visit
template <typename R>
struct TileLds {
    // tile + halo ring (66 x 66 at offset kGuard * kLds), plus kGuard guard rows above and below
    // (+inf T and cost: read by the groups of a sweep outside a lane's window, see sweep_quadrant);
    // halo ring cost = +inf
    Cell<R> Tc[(kLds + 2 * kGuard) * kLds];
    unsigned round, flags;
    unsigned flags_acc; // persistent mode: neighbour activations deferred to the visit's end
    unsigned pend;      // persistent mode: the tile's state word as the last pass consumed it
    unsigned key[5];    // min new value entering: self, N, S, W, E (f32 bits; ordered mode)
    int defer, tile, last;
    unsigned dirs;      // quadrant sweeps of this visit (bit w: wave w's direction)
    unsigned fresh;     // persistent mode: the tile's first visit (kFreshSkip)
};

// ---------------------------------------------------------------------------- tile body
// Stage, sweep and write back one tile; leaves the activation decisions in L.flags (bits 0..3:
// neighbour N/S/W/E can improve; 32/64: changed subdomain S/E edge inside a partial tile;
// 128: some cell decreased by more than the tolerance), L.last (multi-round visits: the last
// round changed something; -1 for single-round visits, which use flags bit 7) and L.key.
// The caller sets L.dirs (quadrant sweeps to run) before the barrier that precedes the call.
// Ends with a workgroup barrier; in COH mode every wave has drained its write-through stores
// before it.
// CAP: honour Fim2dArgs::tcap (the capped bidirectional fronts, eikonal_api.cpp solve_fronts) -- a
// separate instantiation: the compare in the edge test cost the uncapped fp64 solve 4-5 % (C2 2.36
// -> 2.47 ms, profiles/r04i_tcap_ab.log)
template <typename R, bool COH, bool CAP = false, bool REF = false>
__device__ __forceinline__ void process_tile(const Fim2dArgs& a, int tile, TileLds<R>& L, R keep) {
    constexpr R INF = Real<R>::inf();
    Cell<R>* const Ts = L.Tc + kGuard * kLds;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int map = tile / a.tiles_per_map;
    const int rem = tile - map * a.tiles_per_map;
    const int ty = rem / a.ntx, tx = rem - (rem / a.ntx) * a.ntx;
    const R* __restrict__ cost = static_cast<const R*>(a.cost) + (int64_t)map * a.H * a.W;
    const TMem<R, COH> T(static_cast<R*>(a.T) + (int64_t)map * a.H * a.W, a.H * a.W);
    // edge columns of every tile (kEcol): index (t * 2 + side) * kTile + row, side 0 west / 1 east
    const TMem<R, COH> E(static_cast<R*>(a.ecol), (int64_t)a.capacity * 2 * kTile);
    auto eidx = [&](int t, int side, int row) { return ((int64_t)t * 2 + side) * kTile + row; };
    const int64_t y0 = (int64_t)ty * kTile, x0 = (int64_t)tx * kTile;
    const bool full = (y0 + kTile <= a.H) && (x0 + kTile <= a.W) && ((a.W & 3) == 0);
    const R capv = CAP ? (R)a.tcap[map] : INF;  // edge values above it activate no neighbour

    EIK_PROBE(0);
    if (tid == 0) {
        L.round = 0;
        L.flags = 0;
        L.flags_acc = 0;
        L.pend = 0;
    }
    if (tid < 5) L.key[tid] = 0x7f800000u;
    // halo ring: wave 0 north row, 1 south row, 2 west column, 3 east column.  In a tile cut by
    // the raster's south / east end the south row / east column is the one just past the raster
    // (row H / column W) inside the tile: a subdomain's ghost strip lives there, and the in-place
    // passes' halo reload must refresh it like any halo (the cells beyond it are +inf cost, so
    // the ring's own row / column is never an upstream value of a finite-cost cell).
    const int64_t sy = y0 + kTile < a.H ? y0 + kTile : a.H;
    const int64_t sx = x0 + kTile < a.W ? x0 + kTile : a.W;
    // lane's cell of halo side k (0 north row, 1 south row, 2 west column, 3 east column): its LDS
    // cell and column, and its raster position (in range: one unconditional load, else a ghost
    // strip or +inf)
    struct Halo {
        int h, hcol;
        int64_t hy, hx, idx;
        bool in;
    };
    auto halo_of = [&](int k) {
        Halo q;
        if (k == 0)      { q.hcol = lane + 1;            q.h = 0 * kLds + q.hcol; }
        else if (k == 1) { q.hcol = lane + 1;            q.h = (int)(sy - y0 + 1) * kLds + q.hcol; }
        else if (k == 2) { q.hcol = 0;                   q.h = (lane + 1) * kLds + q.hcol; }
        else             { q.hcol = (int)(sx - x0 + 1);  q.h = (lane + 1) * kLds + q.hcol; }
        q.hy = k == 0 ? y0 - 1 : k == 1 ? sy : y0 + lane;
        q.hx = k == 0 || k == 1 ? x0 + lane : k == 2 ? x0 - 1 : sx;
        q.in = q.hy >= 0 && q.hy < a.H && q.hx >= 0 && q.hx < a.W;
        q.idx = q.in ? q.hy * a.W + q.hx : 0;
        // kEcol: the west halo is the west neighbour's east column, the east halo the east
        // neighbour's west column (both tiles of this map when in range)
        if (kEcol<R> && k >= 2 && q.in) q.idx = eidx(k == 2 ? tile - 1 : tile + 1, k == 2 ? 1 : 0, lane);
        return q;
    };
    auto load_halo_of = [&](const Halo& q, int k) {  // k: wave-uniform
        R v = kEcol<R> && k >= 2 ? E.ld(q.idx) : T.ld(q.idx);
        if (!q.in) v = load_T<R, COH>(a, T, q.hy, q.hx);
        return v;
    };
    // this wave's side (staging, and the synchronous in-place reload)
    const Halo hw = halo_of(wave);
    const int h = hw.h, hcol = hw.hcol;
    auto load_halo = [&]() { return load_halo_of(hw, wave); };
    // ---- stage the tile: 16 cells per thread (4 rows x 4 consecutive columns).  Every global
    // load of the visit (T, cost, halo) is issued before the first LDS store, and each path does
    // its own stores (no loaded value flows through a join, whose register copies would wait for
    // the loads): the compiler does not move the sc1 buffer loads across LDS stores, and the
    // interleaved form cost one memory round trip per row group (5 serial trips per staging).
    R told[16];
    const int cx = (tid & 15) * 4;
    auto store_tile = [&](const R (&cr)[16], R hv) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int ry = (tid >> 4) + 16 * k;
#pragma unroll
            for (int e = 0; e < 4; ++e)
                Ts[(ry + 1) * kLds + cx + e + 1] = make_cell<R>(told[4 * k + e], stage_cost(cr[4 * k + e]), cx + e + 1);
        }
        Ts[h] = make_cell<R>(hv, INF, hcol);
    };
    if (full && COH && kFreshSkip && __builtin_amdgcn_readfirstlane(L.fresh)) {
        // a tile's first visit: T is still the init kernel's +inf (the seed kernel marks the goal
        // tile visited), so only the cost is read
        R cr[16];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t gy = y0 + (tid >> 4) + 16 * k;
            if constexpr (sizeof(R) == 4) {
                const float4 c4 = *reinterpret_cast<const float4*>(&cost[gy * a.W + x0 + cx]);
                cr[4 * k] = c4.x; cr[4 * k + 1] = c4.y; cr[4 * k + 2] = c4.z; cr[4 * k + 3] = c4.w;
            } else {
                const double2 c0 = *reinterpret_cast<const double2*>(&cost[gy * a.W + x0 + cx]);
                const double2 c1 = *reinterpret_cast<const double2*>(&cost[gy * a.W + x0 + cx + 2]);
                cr[4 * k] = c0.x; cr[4 * k + 1] = c0.y; cr[4 * k + 2] = c1.x; cr[4 * k + 3] = c1.y;
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) told[4 * k + e] = INF;
        }
        store_tile(cr, load_halo());
        if (tid == 0) atomicAdd(a.visits + 2, 1ull);  // eik_stats::fresh_visits (the byte model)
    } else if (full) {
        R cr[16];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t gy = y0 + (tid >> 4) + 16 * k;
            R tv[4];
            T.ld4(gy * a.W + x0 + cx, tv);
            if constexpr (sizeof(R) == 4) {
                const float4 c4 = *reinterpret_cast<const float4*>(&cost[gy * a.W + x0 + cx]);
                cr[4 * k] = c4.x; cr[4 * k + 1] = c4.y; cr[4 * k + 2] = c4.z; cr[4 * k + 3] = c4.w;
            } else {
                const double2 c0 = *reinterpret_cast<const double2*>(&cost[gy * a.W + x0 + cx]);
                const double2 c1 = *reinterpret_cast<const double2*>(&cost[gy * a.W + x0 + cx + 2]);
                cr[4 * k] = c0.x; cr[4 * k + 1] = c0.y; cr[4 * k + 2] = c1.x; cr[4 * k + 3] = c1.y;
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) told[4 * k + e] = tv[e];
        }
        store_tile(cr, load_halo());
    } else {
        R cr[16];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t gy = y0 + (tid >> 4) + 16 * k;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int64_t gx = x0 + cx + e;
                const bool in = gy < a.H && gx < a.W;
                told[4 * k + e] = load_T<R, COH>(a, T, gy, gx);  // ghost cells land in padding
                cr[4 * k + e] = in ? cost[gy * a.W + gx] : INF;
            }
        }
        store_tile(cr, load_halo());
        // a cut tile's halo sits inside the tile: the ring's own row 65 / column 65, where DY < 0
        // sweeps start and lane 0 of DX < 0 sweeps reads its upstream x, would keep a previous
        // visit's values -- make them +inf (the moved halo row / column is <= 64, no overlap)
        if (tid < kLds) {
            if (sy - y0 < kTile) Ts[(kLds - 1) * kLds + tid] = Cell<R>{INF, INF};
            if (sx - x0 < kTile) Ts[tid * kLds + (kLds - 1)] = Cell<R>{INF, INF};
        }
    }
    if (lane < 4) cell_c(Ts, (lane >> 1) * (kLds - 1) * kLds + (lane & 1) * (kLds - 1), (lane & 1) * (kLds - 1)) = INF;  // corners
    __syncthreads();
    EIK_PROBE(1);

    // PERSISTENT mode revisits a tile that changed IN PLACE, up to a.max_passes times
    // (EIK_OPT_PASSES; by default 24 for one map, 2 for a batch): its interior is already in LDS
    // and nobody else writes it while it is busy, so a pass only refreshes the halo ring,
    // activates the neighbours its last write-back improved, and sweeps again -- no restaging,
    // no queue round trip.  (List mode: one pass; a changed tile re-lists itself.)
    // quadrant sweeps of this pass (bit w: wave w), in a register: the caller's L.dirs for the
    // first pass, then set by the in-place branch below
    unsigned dirs = L.dirs;
    // EIK_ACT_SPLIT: this lane's activation issued at the last pass boundary (-1: none)
    int act_tile = -1;
    unsigned act_old = 0u, act_kold = 0x7f800000u;
    float act_k = 0.f;  // priority mode: the activation's key and the neighbour's key before it
    auto act_complete = [&]() {
        if (act_tile >= 0) qpush_complete(a, act_tile, act_old, act_k, act_kold);
        act_tile = -1;
    };
    for (int pass = 0;; ++pass) {
        // in-sweep duties, by group step: wave 0's split activation (EIK_ACT_SPLIT)
        auto hook = [&](int st) {
            if (EIK_ACT_SPLIT && wave == 0 && st == kActStep) act_complete();
        };
        // ---- sweep rounds (quadrant directions concurrently, one per wave; `dirs` selects them)
        const bool sweep = (dirs >> wave) & 1u;
        bool last_changed = false;
        if (a.max_rounds == 1) {  // single round: "changed" is read off the write-back below
            if (sweep) {
                if (wave == 0)      sweep_quadrant<R, +1, +1, false, REF>(Ts, lane, keep, hook);
                else if (wave == 1) sweep_quadrant<R, -1, +1, false, REF>(Ts, lane, keep, hook);
                else if (wave == 2) sweep_quadrant<R, +1, -1, false, REF>(Ts, lane, keep, hook);
                else                sweep_quadrant<R, -1, -1, false, REF>(Ts, lane, keep, hook);
            } else {  // a wave without a sweep this pass still does its duties, in step order
                for (int st = 0; st < 2 * kTile; st += kAhead) hook(st);
            }
            __syncthreads();
        } else {
            for (int round = 0;; ++round) {
                bool ch = false;
                if (sweep) {
                    if (wave == 0)      ch = sweep_quadrant<R, +1, +1, true, REF>(Ts, lane, keep);
                    else if (wave == 1) ch = sweep_quadrant<R, -1, +1, true, REF>(Ts, lane, keep);
                    else if (wave == 2) ch = sweep_quadrant<R, +1, -1, true, REF>(Ts, lane, keep);
                    else                ch = sweep_quadrant<R, -1, -1, true, REF>(Ts, lane, keep);
                }
                if (__any(ch) && lane == 0) atomicOr(&L.round, 1u << (round & 31));
                __syncthreads();
                last_changed = (L.round >> (round & 31)) & 1u;
                if (!last_changed || round + 1 >= a.max_rounds) break;
            }
        }

        EIK_PROBE(2);
        // PERSISTENT mode, a.sched bit 0: consume the activations that reached this busy tile
        // during the pass (neighbours' edges drained before their atomicOr, and this clear comes
        // before the halo reload) -- an in-place pass then serves them instead of a re-queued
        // visit.  Issued now, awaited with the write-back's drain.
        unsigned pend_old = 0;
        if (COH && (a.sched & 1) && tid == 0) pend_old = atomicAnd(&a.qstate[tile], kBusy | kVisited);
        // ---- write back changed cells, collect side flags (and entering values, ordered mode).
        // EIK_EDGE_FIRST (persistent mode, full tiles): only the tile's edge cells -- the values a
        // neighbour's halo reads -- are stored and drained before the activations; the interior
        // row chunks (bit k of defer_rows: this thread's row chunk k) are stored after the pass's
        // halo has come in and drain during the next sweep, or before the visit's finish (the
        // persistent loop drains every wave before qfinish).  Nobody else reads a busy tile's
        // interior: its next visit starts after that finish.
        unsigned fl = 0;
        unsigned defer_rows = 0;
        R kmin_self = INF, kmin[4] = {INF, INF, INF, INF};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int ry = (tid >> 4) + 16 * k;
            const int64_t gy = y0 + ry;
            R nv[4];
            bool any = false;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                nv[e] = cell_t(Ts, (ry + 1) * kLds + cx + e + 1, cx + e + 1);
                any |= nv[e] < told[4 * k + e];
                // (a ghost cell inside a cut tile is lowered by the halo reload, never by a sweep)
                if (nv[e] < told[4 * k + e] * keep && (full || (gy < a.H && x0 + cx + e < a.W))) {
                    fl |= 128u;  // changed in this visit
                    kmin_self = umin(kmin_self, nv[e]);
                    // A neighbour can only improve if this edge value undercuts the neighbour's
                    // adjacent cell (the halo value, stale => larger => conservative).
                    // (a.tcap: an edge value above the map's cap activates nobody)
                    const int lx = cx + e + 1, ly = ry + 1;
                    const bool act = !CAP || nv[e] <= capv;
                    if (act && ry == 0 && nv[e] < cell_t(Ts, lx, lx)) { fl |= 1u; kmin[0] = umin(kmin[0], nv[e]); }
                    if (act && ry == kTile - 1 && nv[e] < cell_t(Ts, (kLds - 1) * kLds + lx, lx)) { fl |= 2u; kmin[1] = umin(kmin[1], nv[e]); }
                    if (act && cx + e == 0 && nv[e] < cell_t(Ts, ly * kLds, 0)) { fl |= 4u; kmin[2] = umin(kmin[2], nv[e]); }
                    if (act && cx + e == kTile - 1 && nv[e] < cell_t(Ts, ly * kLds + kLds - 1, kLds - 1)) { fl |= 8u; kmin[3] = umin(kmin[3], nv[e]); }
                    const int64_t gx = x0 + cx + e;  // subdomain edges inside a partial tile (DD)
                    if (gy == a.H - 1 && ry != kTile - 1) fl |= 32u;
                    if (gx == a.W - 1 && cx + e != kTile - 1) fl |= 64u;
                }
            }
#if EIK_WB_LINE
            // (A/B, round 6: store whole 128-B lines -- every chunk of a line whose any chunk changed)
            if (full) {
#pragma unroll
                for (int m = 1; m < 128 / (4 * (int)sizeof(R)); m <<= 1) any |= __shfl_xor((int)any, m) != 0;
            }
#endif
            if (any) {
                if (COH && EIK_EDGE_FIRST && full && ry != 0 && ry != kTile - 1) {
                    if (cx == 0 && nv[0] < told[4 * k]) T.st(gy * a.W + x0, nv[0]);
                    if (cx == kTile - 4 && nv[3] < told[4 * k + 3]) T.st(gy * a.W + x0 + kTile - 1, nv[3]);
                    defer_rows |= 1u << k;
                } else if (full) {
                    T.st4(gy * a.W + x0 + cx, nv);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int64_t gx = x0 + cx + e;
                        if (gy < a.H && gx < a.W && nv[e] < told[4 * k + e]) T.st(gy * a.W + gx, nv[e]);
                    }
                }
                // the edge columns' copies (kEcol), drained with T's stores; a cut tile's cells past
                // the raster are never read as a halo, so the copy may hold them too
                if (kEcol<R> && cx == 0 && nv[0] < told[4 * k]) E.st(eidx(tile, 0, ry), nv[0]);
                if (kEcol<R> && cx == kTile - 4 && nv[3] < told[4 * k + 3]) E.st(eidx(tile, 1, ry), nv[3]);
            }
            if (COH) {
#pragma unroll
                for (int e = 0; e < 4; ++e) told[4 * k + e] = nv[e];  // what memory holds now
            }
        }
        if (fl) atomicOr(&L.flags, fl);
        if (a.delta < INF || a.bctl) {  // ordered list mode / priority bands: the entering keys
            if (kmin_self < INF) atomicMin(&L.key[0], __float_as_uint((float)kmin_self));
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (kmin[q] < INF) atomicMin(&L.key[q + 1], __float_as_uint((float)kmin[q]));
        }
        if (tid == 0) L.last = a.max_rounds == 1 ? -1 : (int)last_changed;  // -1: see flags bit 7
        if (COH && (a.sched & 1) && tid == 0) L.pend = pend_old;
        if constexpr (COH) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
        __syncthreads();
        EIK_PROBE(7);
        // the deferred interior row chunks (told holds what they store)
        auto store_deferred = [&]() {
            asm volatile("" ::: "memory");  // not above the halo / activation round trips
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (defer_rows & (1u << k)) {
                    const R v[4] = {told[4 * k], told[4 * k + 1], told[4 * k + 2], told[4 * k + 3]};
                    T.st4((y0 + (tid >> 4) + 16 * k) * a.W + x0 + cx, v);
                }
            }
        };
        if (COH) {
            const unsigned f = L.flags;  // uniform
            const unsigned pend = L.pend & (kPending | kFromN | kFromS | kFromW | kFromE);
            const bool self = (f & 128u) != 0u;
            if ((!self && !pend) || pass + 1 >= a.max_passes || a.max_rounds != 1) {
                store_deferred();  // drained by the persistent loop before the finish
                break;
            }
            // the halo reload is issued first and the budget charge goes to wave 1, so wave 0's
            // activation atomics are the only round trips the next pass waits for
            const R hv = load_halo();
            if (tid == 64) charge_inplace_pass(a);  // in-place passes: stats and the visit budget
            // a.sched bit 1: after the first pass, neighbour activations wait for the visit's end
            // (one activation with the converged edges instead of one per pass)
            const bool defer = (a.sched & 2) && pass > 0;
            if constexpr (EIK_ACT_SPLIT)
                act_tile = activate_neighbours_issue(a, tile, defer ? 0u : f, act_old, L.key, act_k,
                                                     act_kold);  // completed in the next sweep
            else
                activate_neighbours(a, tile, defer ? 0u : f, L.key, 0, 0u);  // lanes 0..4 (T already drained)
            if (defer && tid == 0) L.flags_acc |= f & 0x6fu;
            dirs = self ? 0xFu : sweep_dirs(pend);  // a self revisit: every direction
            cell_t(Ts, h, hcol) = hv;
            store_deferred();  // after the halo value is in: they drain during the next sweep
            __syncthreads();  // every wave has read L.flags and its halo side is in
            if (tid == 0) {
                L.flags = 0;  // next OR-ed after the next sweep barrier
                L.pend = 0;   // consumed by this pass
            }
        } else {
            break;
        }
    }
    act_complete();  // (never pending here: every issue is followed by a pass)
    EIK_PROBE(3);
}

// Activations after a tile visit: the neighbours (with any deferred in-place ones), and the
// tile itself if it changed -- or if it consumed activations (L.pend) it then did not serve.
template <typename R>
__device__ __forceinline__ void activate_after(const Fim2dArgs& a, int tile, const TileLds<R>& L, int list,
                                               unsigned stamp) {
    const unsigned f = L.flags;
    activate_neighbours(a, tile, f | L.flags_acc, L.key, list, stamp);
    if (threadIdx.x == 0) {
        const bool self = L.last < 0 ? (f & 128u) != 0u : L.last != 0;
        if (a.mode == kModePersistent) {
            const unsigned p = L.pend & (kFromN | kFromS | kFromW | kFromE);
            if (self || (L.pend & kPending)) {
                if (self && a.bctl) atomicMin(&a.key[tile], 0u);  // priority mode: a self re-queue goes first
                atomicOr(&a.qstate[tile], kPending | (self ? kSelf : p));  // busy: re-queued by its own finish
            }
        } else if (self) {
            enqueue(a, tile, list, stamp, __uint_as_float(L.key[0]));
        }
    }
}

template <typename R>
__device__ __forceinline__ void init_guard_rows(TileLds<R>& L) {
    const int tid = threadIdx.x;
    for (int i = tid; i < kGuard * kLds; i += kThreads) {
        L.Tc[i] = Cell<R>{Real<R>::inf(), Real<R>::inf()};
        L.Tc[(kLds + kGuard) * kLds + i] = Cell<R>{Real<R>::inf(), Real<R>::inf()};
    }
}

// ------------------------------------------------------------------------ LIST-mode driver
template <typename R>
__global__ __launch_bounds__(kThreads) void fim2d_sweep_kernel(Fim2dArgs a) {
    constexpr R INF = Real<R>::inf();
    __shared__ TileLds<R> L;
    const int tid = threadIdx.x;
    init_guard_rows(L);
    const int cur = a.iter % 3, nxt = (a.iter + 1) % 3, rst = (a.iter + 2) % 3;
    const int cnt = a.counts[cur];
    if (blockIdx.x == 0 && tid == 0) {
        a.counts[rst] = 0;
        a.minkey[rst] = 0x7f800000u;
    }
    const unsigned stamp = a.iter + 2;  // "enqueued for iteration iter+1"
    const float thr = __uint_as_float(a.minkey[cur]) + a.delta;  // ordering window of this launch
    const R keep = (R)a.keep;
    if (tid == 0) L.dirs = 0xFu;  // list mode: every visit runs all four quadrant sweeps

    for (int it = blockIdx.x; it < cnt; it += gridDim.x) {
        const int tile = a.lists[(int64_t)cur * a.capacity + it];
        if (a.delta < INF) {  // ordered mode: defer tiles whose entering T is beyond the window
            if (tid == 0) {
                const float k = __uint_as_float(atomicOr(&a.key[tile], 0u));
                L.defer = k > thr;
                if (k > thr) enqueue(a, tile, nxt, stamp, k);
                else atomicExch(&a.key[tile], 0x7f800000u);  // entering values count afresh
            }
            __syncthreads();
            const bool defer = L.defer;
            __syncthreads();
            if (defer) continue;  // uniform across the workgroup
        }
        process_tile<R, false>(a, tile, L, keep);
        activate_after(a, tile, L, nxt, stamp);
        if (tid == 0 && a.visits) atomicAdd(a.visits, 1ull);
        __syncthreads();  // LDS reuse by the next tile of this workgroup
    }
}

// Min-merge of 64 received strip cells (one wave, all lanes: cell i, valid when i < len) into a
// ghost strip: every cell that drops is stored (made visible, agent scope) and the edge tile beside
// the wave's cells is activated ONCE, with the smallest dropped value as its key -- the wave's 64
// cells are one 64-aligned run, i.e. one tile's edge.  (Round 5 queued one activation per dropped
// cell; on the priority bands each could add a decrease-key entry.)  `count`: dropped cells are
// added there (nullable).
template <typename R>
__device__ __forceinline__ void merge_strip_cells(const Fim2dArgs& a, int side, const R* rv, R* g, int64_t i,
                                                  int64_t len, unsigned* count) {
    R v = Real<R>::inf();
    bool drop = false;
    if (i < len) {
        v = ld_system(rv + i);
        drop = v < ld_agent(g + i);
        if (drop) st_scoped(g + i, v, __HIP_MEMORY_SCOPE_AGENT);
    }
    const unsigned long long m = __ballot(drop);
    if (!m) return;  // wave-uniform
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // the wave's ghost stores before the activation
    // the key is f32 (the bands' entering-T words): reduce in f32, as unsigned bits (T >= 0)
    unsigned k = drop ? __float_as_uint((float)v) : 0x7f800000u;
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) k = min(k, (unsigned)__shfl_xor((int)k, d));
    if ((threadIdx.x & 63) == (unsigned)__builtin_ctzll(m)) {
        if (count) atomicAdd(count, (unsigned)__popcll(m));
        int ty, tx;
        if (side < 2) {
            tx = (int)(i / kTile);
            ty = side == 0 ? 0 : a.nty - 1;
        } else {
            ty = (int)(i / kTile);
            tx = side == 2 ? 0 : a.ntx - 1;
        }
        activate(a, ty * a.ntx + tx, a.iter % 3, a.iter + 1, __uint_as_float(k), kFromN << side);
    }
}

// Live DD halo agent of the 2D solver (fim_engine.hpp live_agent_loop: workgroup 0 of a live launch
// serves the host's mailbox).  PACK: the four edges of T into the neighbours' receive strips (peer
// memory over xGMI); MERGE: the received strips min-merged into the ghosts, one activation per edge
// tile and side (merge_strip_cells).
template <typename R>
__device__ __forceinline__ void live_agent(const Fim2dArgs& a, unsigned* sh) {
    const int tid = threadIdx.x;
    auto pack = [&](unsigned par, bool skip_busy) {
        const R* T = static_cast<const R*>(a.T);
        R* tg[4];
        for (int k = 0; k < 4; ++k) tg[k] = static_cast<R*>(a.live->send[par][k]);
        // EIK_OPT_LIVE_PACK 1 (skip_busy): a cell of a tile that is pending or busy is not packed -- the
        // receiver's strip of this parity keeps an older (larger) value, which the min-merge ignores; a
        // round whose snapshot saw no tile pending or busy packs every cell, so the convergence vote's
        // proof (dd.solve_live) is unchanged
        auto idle = [&](int64_t ty, int64_t tx) {
            return !skip_busy ||
                   (__hip_atomic_load(&a.qstate[ty * a.ntx + tx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) &
                    (kPending | kBusy)) == 0u;
        };
        for (int64_t i = tid; i < a.W; i += blockDim.x) {
            if (tg[0] && idle(0, i / kTile)) st_scoped(tg[0] + i, ld_agent(T + i), __HIP_MEMORY_SCOPE_SYSTEM);
            if (tg[1] && idle(a.nty - 1, i / kTile))
                st_scoped(tg[1] + i, ld_agent(T + (a.H - 1) * a.W + i), __HIP_MEMORY_SCOPE_SYSTEM);
        }
        for (int64_t i = tid; i < a.H; i += blockDim.x) {
            if (tg[2] && idle(i / kTile, 0)) st_scoped(tg[2] + i, ld_agent(T + i * a.W), __HIP_MEMORY_SCOPE_SYSTEM);
            if (tg[3] && idle(i / kTile, a.ntx - 1))
                st_scoped(tg[3] + i, ld_agent(T + i * a.W + a.W - 1), __HIP_MEMORY_SCOPE_SYSTEM);
        }
    };
    auto merge = [&](unsigned par, unsigned* count) {
        for (int side = 0; side < 4; ++side) {
            const R* rv = static_cast<const R*>(a.live->recv[par][side]);
            R* g = static_cast<R*>(const_cast<void*>(a.ghost[side]));
            if (!rv || !g) continue;
            const int64_t len = side < 2 ? a.W : a.H;
            for (int64_t i0 = 0; i0 < len; i0 += blockDim.x) merge_strip_cells<R>(a, side, rv, g, i0 + tid, len, count);
        }
    };
    live_agent_loop(a, sh, pack, merge);
}

// WPS: the launch-bounds occupancy target in waves per SIMD (1: the compiler's choice, 159
// VGPRs -> 3 workgroups per CU; 4: <= 128 VGPRs -> 4 per CU, a few spills).  Large rasters
// (maps of >= kWideTiles tiles: the throughput-bound regime) run the 4-wave form -- 16384^2 on one GPU
// +10-15 %, 4096^2 -3 % (profiles/r02r_wps_ab.log).
template <typename R, int WPS, bool CAP = false, bool REF = false>
__global__ __launch_bounds__(kThreads, WPS) void fim2d_persist_kernel(Fim2dArgs a) {
    __shared__ TileLds<R> L;
    if (a.live && blockIdx.x == 0) {
        __shared__ unsigned sh[4];
        live_agent<R>(a, sh);
        return;
    }
    init_guard_rows(L);
    EIK_KSTART();
    const R keep = (R)a.keep;
    int tile = -1;
    unsigned nvis = 0;  // wave 0 lane 0: visits not yet added to the global counter
    for (;;) {
        if (EIK_EDGE_FIRST && tile >= 0) {  // uniform: every wave's deferred interior stores
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // complete before the finish
            __syncthreads();
        }
        // wave 0 retires the previous tile (lanes 0..4 activate, then lane 0 finishes) while
        // wave 1 takes the next one; waves 2 and 3 go straight to the barrier
        if (threadIdx.x < 64) {
            if (tile >= 0) {
                EIK_PROBE(4);
                activate_after(a, tile, L, 0, 0u);
                // the activations' counter increments complete before the finish decrements
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (threadIdx.x == 0) {
                    qfinish(a, tile);
                    if (++nvis == 64u) {  // visit cap (negative costs never converge)
                        charge_visits(a, 64ull);
                        nvis = 0;
                    }
                }
            }
            EIK_PROBE(5);
        } else if (threadIdx.x < 128 && (a.bctl || threadIdx.x == 64)) {
            // wave 1 takes the next tile (priority bands: the whole wave; else lane 64)
            unsigned trig = 0;
            const int t = a.bctl ? qgrab_prio(a, trig) : qgrab(a, trig);
            if (threadIdx.x == 64) {
                L.tile = t;
                L.dirs = sweep_dirs(trig);
                L.fresh = !(trig & kVisited);
                if (t >= 0) EIK_VISIT(t, trig, L.dirs);
            }
        }
        __syncthreads();
        EIK_PROBE(6);
        tile = __builtin_amdgcn_readfirstlane(L.tile);
        if (tile < 0) break;  // uniform: solve finished (or failed)
        process_tile<R, true, CAP, REF>(a, tile, L, keep);  // sc1 loads; sc1 stores drained + barrier
    }
    if (threadIdx.x == 0 && nvis) atomicAdd(a.visits, (unsigned long long)nvis);
}
// ------------------------------------------------------------------------ init / seeding
// T = inf everywhere; marks / keys / queue state cleared.
template <typename R>
__global__ void fim2d_init_kernel(R* __restrict__ T, int64_t n, unsigned* __restrict__ mark, int64_t ntiles,
                                  unsigned* __restrict__ key, unsigned* __restrict__ minkey, unsigned* __restrict__ qstate,
                                  unsigned* __restrict__ qslot, int64_t nslots, unsigned* __restrict__ counts,
                                  unsigned* __restrict__ qctl, unsigned* __restrict__ visits, unsigned* __restrict__ edge,
                                  R* __restrict__ ecol) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    // the solve's control words (list counts, queue head / tail / active / error, visit counters,
    // DD edge flags) -- here rather than four memset nodes ahead of this kernel
    if (blockIdx.x == 0 && threadIdx.x < kQueueCtlBytes / 4) {
        const int t = threadIdx.x;
        if (qctl) qctl[t] = 0u;
        if (t < 4) {
            if (counts) counts[t] = 0u;
            if (edge) edge[t] = 0u;
        }
        if (t < 22 && visits) visits[t] = 0u;  // full visits, in-place passes, fresh visits, 8 queue counters (u64 each)
    }
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) T[i] = Real<R>::inf();
    if (ecol)
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ntiles * 2 * kTile; i += stride)
            ecol[i] = Real<R>::inf();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ntiles; i += stride) {
        mark[i] = 0;
        key[i] = 0x7f800000u;
        if (qstate) qstate[i] = 0;
    }
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += stride) qslot[i] = 0;
    if (blockIdx.x == 0 && threadIdx.x < 3) minkey[threadIdx.x] = threadIdx.x == 0 ? 0u : 0x7f800000u;
}

// T[goal] = 0 and the goal tile activated.  Goals: one per map (gx < 0: none).
template <typename R>
__global__ void fim2d_seed_kernel(Fim2dArgs a, const int64_t* __restrict__ goals, int nmaps) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m == 0) {
        a.counts[1] = 0;
        a.counts[2] = 0;
    }
    if (m >= nmaps) return;
    const int64_t gx = goals[2 * m], gy = goals[2 * m + 1];
    if (gx < 0 || gy < 0 || gx >= a.W || gy >= a.H) return;
    static_cast<R*>(a.T)[(int64_t)m * a.H * a.W + gy * a.W + gx] = R(0);
    const int tile = m * a.tiles_per_map + (int)(gy / kTile) * a.ntx + (int)(gx / kTile);
    if (kEcol<R> && a.ecol && (gx % kTile == 0 || gx % kTile == kTile - 1))  // the edge columns' copy
        static_cast<R*>(a.ecol)[((int64_t)tile * 2 + (gx % kTile == 0 ? 0 : 1)) * kTile + gy % kTile] = R(0);
    if (a.mode == kModePersistent) {
        qpush(a, tile, kSelf | kVisited);  // visited: its T is not all +inf (kFreshSkip)
        return;
    }
    a.mark[tile] = 1;  // enqueued for iteration 0
    a.key[tile] = 0u;  // T = 0 enters at the goal
    const int pos = atomicAdd(&a.counts[0], 1);
    a.lists[pos] = tile;
}

// Priority bands (EIK_OPT_PRIO): the band width, 64 x the geometric mean of the finite positive costs
// (one tile width of T at a typical cost; C2's cost mean is 40 but its median 3.6 -- obstacles
// dominate the mean) x the option's multiplier, from 4096 cells sampled across the raster (one block).
template <typename R>
__global__ __launch_bounds__(256) void prio_delta_kernel(const R* __restrict__ cost, int64_t n, float mult,
                                                          float* __restrict__ out) {
    __shared__ double ssum[4];
    __shared__ int scnt[4];
    double sum = 0.0;
    int cnt = 0;
    for (int i = threadIdx.x; i < 4096; i += 256) {
        // scattered over rows AND columns (an even stride over a 2^k raster would sample one column)
        const unsigned long long hsh = (unsigned long long)(i + 1) * 0x9E3779B97F4A7C15ull;
        const double c = (double)cost[(int64_t)((hsh >> 11) % (unsigned long long)n)];
        if (c > 0.0 && c < Real<double>::inf()) {
            sum += log(c);
            ++cnt;
        }
    }
    for (int d = 32; d > 0; d >>= 1) {
        sum += __shfl_down(sum, d);
        cnt += __shfl_down(cnt, d);
    }
    if ((threadIdx.x & 63) == 0) {
        ssum[threadIdx.x >> 6] = sum;
        scnt[threadIdx.x >> 6] = cnt;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const double s = ssum[0] + ssum[1] + ssum[2] + ssum[3];
        const int c = scnt[0] + scnt[1] + scnt[2] + scnt[3];
        const double g = c ? exp(s / c) : 1.0;
        *out = (float)(mult * 64.0 * g > 1e-30 ? mult * 64.0 * g : 1e-30);
    }
}

hipError_t fim2d_prio_delta(const void* cost, bool f64, int64_t n, float mult, float* out, hipStream_t st) {
    if (f64)
        hipLaunchKernelGGL(prio_delta_kernel<double>, dim3(1), dim3(256), 0, st, static_cast<const double*>(cost), n,
                           mult, out);
    else
        hipLaunchKernelGGL(prio_delta_kernel<float>, dim3(1), dim3(256), 0, st, static_cast<const float*>(cost), n,
                           mult, out);
    return hipGetLastError();
}

// After each persistent launch: the tickets of its idle waiters ran ahead of the tail --
// restart the ticket counter at the tail.  On the FIFO every slot is empty when a launch ends.
// With priority bands a dispatch may still move (stale) band entries into slots whose ticket
// holders have already left on qactive == 0: those entries are dropped here and their tiles'
// band-membership bits cleared (the relaunch schedule's next launch would otherwise read a
// leftover entry one ring lap later, and the bit would keep the tile out of its band).
__global__ void fim2d_qrewind_kernel(Fim2dArgs a) {
    if (a.bctl) {
        const int64_t stride = (int64_t)gridDim.x * blockDim.x;
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= (int64_t)a.qmask; i += stride) {
            const unsigned v = a.qslot[i];
            if (v == 0u) continue;
            const unsigned tag = v >> kBandTagShift;
            if (tag) atomicAnd(&a.bmem[(v & kSlotTileMask) - 1u], ~(1ull << (tag - 1u)));
            a.qslot[i] = 0u;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *a.qhead = *a.qtail;
}
static void launch_qrewind(const Fim2dArgs& a, hipStream_t st) {
    const int grid = a.bctl ? (int)std::min<int64_t>(256, ((int64_t)a.qmask + 256) / 256) : 1;
    hipLaunchKernelGGL(fim2d_qrewind_kernel, dim3(grid), dim3(a.bctl ? 256 : 1), 0, st, a);
}

// Domain decomposition: ghost = min(ghost, recv) and activate every edge tile next to a ghost
// cell that decreased (for list iteration `iter`, or into the FIFO).  side: 0 N 1 S 2 W 3 E.
// The strip may have been written by a peer GPU (system-scope loads); during a live launch the
// ghost store is made visible (agent scope, released) before the tile is queued.
// (Blocks of 256: each wave's cells are one 64-aligned run, merge_strip_cells.)
template <typename R>
__global__ __launch_bounds__(256) void fim2d_merge_ghost_kernel(Fim2dArgs a, int side, const R* __restrict__ recv,
                                                                int64_t len) {
    R* g = static_cast<R*>(const_cast<void*>(a.ghost[side]));
    merge_strip_cells<R>(a, side, recv, g, (int64_t)blockIdx.x * blockDim.x + threadIdx.x, len, nullptr);
}

// Copy this subdomain's edge rows/columns of T into contiguous send strips -- local buffers or a
// peer GPU's receive strips (system-scope stores).  T may be in flight (live launch): agent loads.
template <typename R>
__global__ void fim2d_pack_edges_kernel(Fim2dArgs a, R* __restrict__ n, R* __restrict__ s, R* __restrict__ w,
                                        R* __restrict__ e) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const R* T = static_cast<const R*>(a.T);
    if (i < a.W) {
        if (n) st_scoped(n + i, ld_agent(T + i), __HIP_MEMORY_SCOPE_SYSTEM);
        if (s) st_scoped(s + i, ld_agent(T + (a.H - 1) * a.W + i), __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (i < a.H) {
        if (w) st_scoped(w + i, ld_agent(T + i * a.W), __HIP_MEMORY_SCOPE_SYSTEM);
        if (e) st_scoped(e + i, ld_agent(T + i * a.W + a.W - 1), __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ------------------------------------------------------------------------- host launchers
hipError_t fim2d_sweep(const Fim2dArgs& a, bool f64, int grid, hipStream_t st) {
    if (f64)
        hipLaunchKernelGGL(fim2d_sweep_kernel<double>, dim3(grid), dim3(kThreads), 0, st, a);
    else
        hipLaunchKernelGGL(fim2d_sweep_kernel<float>, dim3(grid), dim3(kThreads), 0, st, a);
    return hipGetLastError();
}

// Workgroups of the persistent kernel that can be co-resident (a larger grid only adds
// workgroups that start after the solve ended and leave at once).
int fim2d_persist_resident(bool f64, int cus, bool wide) {
    int per_cu = 0;
    const hipError_t e =
        f64    ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fim2d_persist_kernel<double, 1>, kThreads, 0)
        : wide ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fim2d_persist_kernel<float, 4>, kThreads, 0)
               : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fim2d_persist_kernel<float, 1>, kThreads, 0);
    if (e != hipSuccess || per_cu < 1) per_cu = 1;
    return per_cu * cus;
}

hipError_t fim2d_persist(const Fim2dArgs& a, bool f64, int grid, hipStream_t st, bool wide, bool rewind) {
    // (a.tcap: fp64 only -- the fp32 kernels and list mode solve in full, which the capped fronts'
    // clean pass and check accept as well)
    if (f64 && a.ref_arith && a.tcap)
        hipLaunchKernelGGL((fim2d_persist_kernel<double, 1, true, true>), dim3(grid), dim3(kThreads), 0, st, a);
    else if (f64 && a.ref_arith)
        hipLaunchKernelGGL((fim2d_persist_kernel<double, 1, false, true>), dim3(grid), dim3(kThreads), 0, st, a);
    else if (f64 && a.tcap)
        hipLaunchKernelGGL((fim2d_persist_kernel<double, 1, true>), dim3(grid), dim3(kThreads), 0, st, a);
    else if (f64)
        hipLaunchKernelGGL((fim2d_persist_kernel<double, 1>), dim3(grid), dim3(kThreads), 0, st, a);
    else if (wide)
        hipLaunchKernelGGL((fim2d_persist_kernel<float, 4>), dim3(grid), dim3(kThreads), 0, st, a);
    else
        hipLaunchKernelGGL((fim2d_persist_kernel<float, 1>), dim3(grid), dim3(kThreads), 0, st, a);
    // before anything (merge kernel, next launch) appends again
    if (rewind) launch_qrewind(a, st);
    return hipGetLastError();
}

hipError_t fim2d_qrewind(const Fim2dArgs& a, hipStream_t st) {
    launch_qrewind(a, st);
    return hipGetLastError();
}

hipError_t fim2d_init(const Fim2dArgs& a, bool f64, int nmaps, const int64_t* d_goals, unsigned* edge, hipStream_t st) {
    static_assert(kQueueCtlBytes / 4 <= 256, "the init kernel's block 0 clears the queue words");
    const int64_t n = (int64_t)nmaps * a.H * a.W;
    const int64_t ntiles = (int64_t)nmaps * a.tiles_per_map;
    const int grid = (int)std::min<int64_t>(4096, (n + 255) / 256);
    const int64_t nslots = a.qslot ? (int64_t)a.qmask + 1 : 0;
    unsigned* const counts = reinterpret_cast<unsigned*>(a.counts);
    unsigned* const qctl = reinterpret_cast<unsigned*>(a.qhead);  // head tail active error
    unsigned* const visits = reinterpret_cast<unsigned*>(a.visits);
    if (f64) {
        hipLaunchKernelGGL(fim2d_init_kernel<double>, dim3(grid), dim3(256), 0, st, static_cast<double*>(a.T), n,
                           a.mark, ntiles, a.key, a.minkey, a.qstate, a.qslot, nslots, counts, qctl, visits, edge,
                           kEcol<double> ? static_cast<double*>(a.ecol) : nullptr);
        hipLaunchKernelGGL(fim2d_seed_kernel<double>, dim3((nmaps + 255) / 256), dim3(256), 0, st, a, d_goals, nmaps);
    } else {
        hipLaunchKernelGGL(fim2d_init_kernel<float>, dim3(grid), dim3(256), 0, st, static_cast<float*>(a.T), n,
                           a.mark, ntiles, a.key, a.minkey, a.qstate, a.qslot, nslots, counts, qctl, visits, edge,
                           kEcol<float> ? static_cast<float*>(a.ecol) : nullptr);
        hipLaunchKernelGGL(fim2d_seed_kernel<float>, dim3((nmaps + 255) / 256), dim3(256), 0, st, a, d_goals, nmaps);
    }
    return hipGetLastError();
}

hipError_t fim2d_merge_ghost(const Fim2dArgs& a, bool f64, int side, const void* recv, int64_t len, hipStream_t st) {
    const int grid = (int)((len + 255) / 256);
    if (f64)
        hipLaunchKernelGGL(fim2d_merge_ghost_kernel<double>, dim3(grid), dim3(256), 0, st, a, side,
                           static_cast<const double*>(recv), len);
    else
        hipLaunchKernelGGL(fim2d_merge_ghost_kernel<float>, dim3(grid), dim3(256), 0, st, a, side,
                           static_cast<const float*>(recv), len);
    return hipGetLastError();
}

hipError_t fim2d_pack_edges(const Fim2dArgs& a, bool f64, void* n, void* s, void* w, void* e, hipStream_t st) {
    const int64_t len = a.H > a.W ? a.H : a.W;
    const int grid = (int)((len + 255) / 256);
    if (f64)
        hipLaunchKernelGGL(fim2d_pack_edges_kernel<double>, dim3(grid), dim3(256), 0, st, a, (double*)n, (double*)s,
                           (double*)w, (double*)e);
    else
        hipLaunchKernelGGL(fim2d_pack_edges_kernel<float>, dim3(grid), dim3(256), 0, st, a, (float*)n, (float*)s,
                           (float*)w, (float*)e);
    return hipGetLastError();
}

}  // namespace eik
