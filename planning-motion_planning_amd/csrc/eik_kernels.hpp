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
    unsigned long long* visits;  // tile-visit counter (stats / roofline bytes)
    unsigned* edge_dirty;  // DD: bit per subdomain side whose edge row/column changed
};

hipError_t fim2d_init(const Fim2dArgs& a, bool f64, int nmaps, const int64_t* d_goals, hipStream_t st);
hipError_t fim2d_sweep(const Fim2dArgs& a, bool f64, int grid, hipStream_t st);
hipError_t fim2d_merge_ghost(const Fim2dArgs& a, bool f64, int side, const void* recv, int64_t len, hipStream_t st);
hipError_t fim2d_pack_edges(const Fim2dArgs& a, bool f64, void* n, void* s, void* w, void* e, hipStream_t st);

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
};
hipError_t gdm2d(const Gdm2dArgs& a, bool f64, hipStream_t st);

// Full-field inf-aware normalised gradient (computeGradient(T, point=[]), FastMarching.py:242-300)
hipError_t gradient2d(const double* T, int64_t H, int64_t W, double* gnx, double* gny, hipStream_t st);

}  // namespace eik
