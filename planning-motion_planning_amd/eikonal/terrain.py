"""Synthetic DEM-derived cost rasters for benchmarks and large-map tests.

There is no DEM in the reference repo (Coupled_motion_planner.py:1098 reads PRL_DEM.txt, which
is not shipped), so benchmarks build one.  The heights are a fractal (1/f^beta) surface from
sparse spectral synthesis: a sum of random plane waves with power-law amplitudes.  It can be
evaluated on ANY sub-block from global coordinates, so every rank of a decomposed raster builds
exactly its own part of one seamless global map.

The cost follows the planner's recipe (Coupled_motion_planner.py:1144-1216):
  slope = arccos(Nz) > 0.20 rad -> obstacle (:1147-1154)
  opening with disk(10) (:1168-1171), closing with disk(round(0.45/res)) (:1173-1180)
  map border is an obstacle (:1182-1186)
  cost = 1 + 300*obstacle + 10*ramp, ramp = distance ramp within 1 m of obstacles (:1188-1205)
  50 x 50 box blur with fill value 300 outside the map (:1208-1210)
  border cells = +inf (:1213-1216)
Deviations (documented, synthetic input only): the hole filling (cv2.floodFill, :66-78) is a
global connectivity operation and is skipped; the distance ramp uses a bounded-radius
distance (<= 1 m) instead of the global EDT normalisation (its contribution is < 10 cost units
either way).  Everything is float32 torch on the device the caller chooses.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

RES = 0.05          # m per cell
SLOPE_MAX = 0.20    # rad, Coupled_motion_planner.py:1154
RMS_SLOPE = 0.17    # m/m: ~22 % of raw cells above SLOPE_MAX, ~6 % obstacle cost after morphology
MARGIN = 96         # halo (cells) computed around a block so blocks agree with the global map
                    # (influence radius of the recipe: 10+10+9+9+20+25 = 83 cells)


def _waves(seed, n_waves=160, beta=2.2, fmin=1.0 / 4096, fmax=1.0 / 32):
    rng = np.random.default_rng(seed)
    f = np.exp(rng.uniform(np.log(fmin), np.log(fmax), n_waves))  # cycles per cell
    th = rng.uniform(0, 2 * np.pi, n_waves)
    ph = rng.uniform(0, 2 * np.pi, n_waves)
    amp = f ** (-beta / 2.0) * np.sqrt(f)  # power ~ f^-beta with log-uniform frequency density
    kx, ky = 2 * np.pi * f * np.cos(th), 2 * np.pi * f * np.sin(th)
    return kx, ky, ph, amp


def dem_block(y0, x0, h, w, seed=42, device="cpu"):
    """Heights (m) on global rows [y0, y0+h), cols [x0, x0+w).  Slopes are scaled so that about
    a fifth of the raw cells exceed SLOPE_MAX (obstacle fields of ~1 m scale)."""
    kx, ky, ph, amp = _waves(seed)
    # normalise the RMS slope: sum over waves of (amp*k)^2/2 = target^2
    rms_slope_cells = math.sqrt(0.5 * float(np.sum((amp * np.hypot(kx, ky)) ** 2)))
    scale = RMS_SLOPE * RES / rms_slope_cells  # metres per unit amplitude
    ys = torch.arange(y0, y0 + h, device=device, dtype=torch.float64)[:, None]
    xs = torch.arange(x0, x0 + w, device=device, dtype=torch.float64)[None, :]
    z = torch.zeros((h, w), device=device, dtype=torch.float64)
    for i in range(len(amp)):
        z += float(amp[i] * scale) * torch.sin(float(kx[i]) * xs + float(ky[i]) * ys + float(ph[i]))
    return z.float()


def _grow(m, r):
    """Dilation by an octagon of radius r (alternating 3x3 square / cross steps): a GPU-cheap
    stand-in for cv2.dilate with structural_disk(r) (Coupled_motion_planner.py:92-103)."""
    x = m[None, None]
    for i in range(r):
        if i % 2 == 0:
            x = F.max_pool2d(x, 3, stride=1, padding=1)
        else:
            p = F.pad(x, (1, 1, 1, 1))
            x = torch.maximum(torch.maximum(p[..., 1:-1, 1:-1], p[..., :-2, 1:-1]),
                              torch.maximum(torch.maximum(p[..., 2:, 1:-1], p[..., 1:-1, :-2]), p[..., 1:-1, 2:]))
    return x[0, 0]


def _grow_cross(m):
    p = F.pad(m[None, None], (1, 1, 1, 1))
    x = torch.maximum(torch.maximum(p[..., 1:-1, 1:-1], p[..., :-2, 1:-1]),
                      torch.maximum(torch.maximum(p[..., 2:, 1:-1], p[..., 1:-1, :-2]), p[..., 1:-1, 2:]))
    return x[0, 0]


def _dilate(m, r):
    return _grow(m, r)


def _erode(m, r):
    return 1.0 - _grow(1.0 - m, r)


def cost_block(y0, x0, h, w, H, W, seed=42, device="cpu"):
    """Cost raster (float32, [h][w]) of the global H x W map restricted to the block."""
    m = MARGIN
    Y0, X0, hh, ww = y0 - m, x0 - m, h + 2 * m, w + 2 * m
    z = dem_block(Y0, X0, hh, ww, seed, device)
    gy = torch.zeros_like(z)
    gx = torch.zeros_like(z)
    gy[1:-1] = (z[2:] - z[:-2]) / (2 * RES)
    gx[:, 1:-1] = (z[:, 2:] - z[:, :-2]) / (2 * RES)
    slope = torch.atan(torch.sqrt(gx * gx + gy * gy))  # == arccos(Nz) of the surface normal
    ys = torch.arange(Y0, Y0 + hh, device=device)[:, None]
    xs = torch.arange(X0, X0 + ww, device=device)[None, :]
    inside = (ys >= 0) & (ys < H) & (xs >= 0) & (xs < W)
    border = inside & ((ys == 0) | (ys == H - 1) | (xs == 0) | (xs == W - 1))
    obst = ((slope > SLOPE_MAX) & inside & ~border).float()
    obst = _dilate(_erode(obst, 10), 10)                                     # :1168-1171
    rc = int(round(0.45 / RES))
    obst = _erode(_dilate(obst, rc), rc)                                     # :1173-1180
    obst = torch.where(border | ~inside, torch.ones_like(obst), obst)       # :1182-1186
    r1 = int(round(1.0 / RES))                                               # :1191-1193
    dist = torch.full_like(obst, float(r1 + 1))
    ring = obst
    for r in range(1, r1 + 1):                                               # bounded distance
        nxt = _grow(ring, 1) if r % 2 == 1 else _grow_cross(ring)
        dist = torch.where((nxt > 0) & (ring == 0), torch.full_like(dist, float(r)), dist)
        ring = nxt
    dist = torch.where(obst > 0, torch.zeros_like(dist), dist)
    ramp = torch.clamp(1.0 - dist / (r1 + 1), min=0.0) * (dist > 0)          # :1195-1200
    cost = 1.0 + 300.0 * obst + 10.0 * ramp                                  # :1203-1205
    cost = torch.where(inside, cost, torch.full_like(cost, 300.0))          # fill value 300
    k = 50
    cpad = F.pad(cost[None, None], (k // 2, k - 1 - k // 2, k // 2, k - 1 - k // 2), value=300.0)
    cost = F.avg_pool2d(cpad, k, stride=1)[0, 0]                             # :1208-1210
    cost = cost[m:m + h, m:m + w].contiguous()
    yy = torch.arange(y0, y0 + h, device=device)[:, None]
    xx = torch.arange(x0, x0 + w, device=device)[None, :]
    edge = (yy == 0) | (yy == H - 1) | (xx == 0) | (xx == W - 1)
    return torch.where(edge, torch.full_like(cost, float("inf")), cost)     # :1213-1216
