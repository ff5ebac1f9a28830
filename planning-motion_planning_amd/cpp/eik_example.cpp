// eik_example.cpp -- C++ host calling the HIP solver through the C ABI only (include/eikonal.h):
// cost raster -> arrival field (computeTmap) -> gradient-descent path (getPathGDM).
//   eik_example [N]      (N x N random cost with an inf border; goal at the centre)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../include/eikonal.h"

static int check(eik_ctx* ctx, int rc, const char* what)
{
    if (rc != EIK_OK) std::fprintf(stderr, "%s failed (%d): %s\n", what, rc, eik_last_error(ctx));
    return rc;
}

int main(int argc, char** argv)
{
    const int64_t N = argc > 1 ? std::atoll(argv[1]) : 512;
    eik_ctx* ctx = nullptr;
    if (check(nullptr, eik_create(0, &ctx), "eik_create")) return 1;
    std::vector<float> cost((size_t)(N * N));
    std::mt19937 rng(1);
    std::uniform_real_distribution<float> u(1.f, 10.f);
    for (int64_t y = 0; y < N; ++y)
        for (int64_t x = 0; x < N; ++x)
            cost[y * N + x] = (x == 0 || y == 0 || x == N - 1 || y == N - 1) ? INFINITY : u(rng);
    std::vector<float> T((size_t)(N * N));
    const int64_t gx = N / 2, gy = N / 2;
    if (check(ctx, eik_tmap2d_f32(ctx, cost.data(), N, N, gx, gy, T.data()), "eik_tmap2d_f32")) return 1;
    eik_stats st;
    eik_get_stats(ctx, &st);
    std::vector<double> T64(T.begin(), T.end());
    const double init[2] = {8.0, 8.0}, end[2] = {(double)gx, (double)gy};
    std::vector<double> path(2 * 30004);
    int64_t n = 0;
    int status = 0;
    if (check(ctx, eik_path2d_f64(ctx, T64.data(), N, N, init, end, 0.5, path.data(), 30004, &n, &status),
              "eik_path2d_f64"))
        return 1;
    std::printf("%s\nT[8,8] = %.4f  solve %.3f ms  %lld tile visits  path %lld points (status %d), ends at (%.1f, %.1f)\n",
                eik_version(), T[8 * N + 8], st.solve_ms, (long long)st.tile_visits, (long long)n, status,
                path[2 * (n - 1)], path[2 * (n - 1) + 1]);
    eik_destroy(ctx);
    return 0;
}
