// rover.cpp -- host tail of the planner's step 1 (Coupled_motion_planner.py:1222-1258): the two
// GDM paths -> one rover path in metres with z and heading.  No GPU: callable without a device
// (the CPU tests pin it against the oracle's restatement bit for bit).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <vector>

#include "../../include/eikonal.h"

// zmin_known: min(Z) when the caller has it (eik_rover_path_f64: the cost builder's device minimum,
// exact), else NaN -- a host pass over the whole DEM (7 ms of planner step 1 at 4096^2, one core)
int rover_assemble(const double* pathS, int64_t nS, const double* pathG, int64_t nG, const double* Z, int64_t H,
                   int64_t W, const eik_rover_query* q, double* path_xyz, double* heading, int64_t cap, int64_t* n_out,
                   double zmin_known) {
#pragma clang fp contract(off)  // numpy's elementwise arithmetic: no fused multiply-adds
    if (!pathS || !pathG || !Z || !q || !path_xyz || !heading || !n_out || nS < 1 || nG < 1 || H < 1 || W < 1 ||
        !(q->resolution > 0))
        return EIK_ERR_ARG;
    const double res = q->resolution;
    // roverPath = vstack(flipud(pathS), pathG[1:]); roverPath = res * (roverPath + 1)   :1228-1230
    std::vector<double> px, py;
    px.reserve((size_t)(nS + nG));
    py.reserve((size_t)(nS + nG));
    for (int64_t i = nS - 1; i >= 0; --i) {
        px.push_back(res * (pathS[2 * i] + 1.0));
        py.push_back(res * (pathS[2 * i + 1] + 1.0));
    }
    for (int64_t i = 1; i < nG; ++i) {
        px.push_back(res * (pathG[2 * i] + 1.0));
        py.push_back(res * (pathG[2 * i + 1] + 1.0));
    }
    // drop waypoints within 0.1 m of the rover, then of the sample (np.linalg.norm)   :1232-1243
    auto norm2 = [](double dx, double dy) {
        const double a = dx * dx;
        const double b = dy * dy;
        return std::sqrt(a + b);
    };
    std::vector<size_t> keep;
    keep.reserve(px.size());
    for (size_t i = 0; i < px.size(); ++i) {
        if (norm2(px[i] - q->xr, py[i] - q->yr) < 0.1) continue;
        if (norm2(px[i] - q->xm, py[i] - q->ym) < 0.1) continue;
        keep.push_back(i);
    }
    const int64_t n = (int64_t)keep.size();
    *n_out = n;
    if (n > cap) return EIK_ERR_ARG;
    // z = zp + Zs[uint32(round(y / res)), uint32(round(x / res))], Zs = Z - min(Z)   :1101, :1246
    double zmin = zmin_known;
    if (std::isnan(zmin)) {
        zmin = std::numeric_limits<double>::infinity();
        for (int64_t i = 0; i < H * W; ++i) zmin = std::min(zmin, Z[i]);  // np.min (no NaN in a DEM)
    }
    for (int64_t k = 0; k < n; ++k) {
        const size_t i = keep[k];
        const double fy = std::nearbyint(py[i] / res), fx = std::nearbyint(px[i] / res);  // half to even
        if (!(fy >= 0 && fx >= 0 && fy < (double)H && fx < (double)W)) return EIK_ERR_ARG;  // IndexError
        const int64_t iy = (int64_t)fy, ix = (int64_t)fx;
        path_xyz[3 * k] = px[i];
        path_xyz[3 * k + 1] = py[i];
        path_xyz[3 * k + 2] = q->zp + (Z[iy * W + ix] - zmin);
    }
    // heading = [initialHeading, arctan2(diff(y), diff(x))]   :1249-1252
    if (n > 0) heading[0] = q->initial_heading;
    for (int64_t k = 1; k < n; ++k)
        heading[k] = std::atan2(path_xyz[3 * k + 1] - path_xyz[3 * (k - 1) + 1], path_xyz[3 * k] - path_xyz[3 * (k - 1)]);
    return EIK_OK;
}

extern "C" int eik_rover_assemble(const double* pathS, int64_t nS, const double* pathG, int64_t nG, const double* Z,
                                  int64_t H, int64_t W, const eik_rover_query* q, double* path_xyz, double* heading,
                                  int64_t cap, int64_t* n_out) {
    return rover_assemble(pathS, nS, pathG, nG, Z, H, W, q, path_xyz, heading, cap, n_out,
                          std::numeric_limits<double>::quiet_NaN());
}
