"""GPU cost-raster builder: the producer of the Eikonal solver's input.

Mirrors the cost-map helpers of the reference planner (src/Coupled_motion_planner.py), which
cannot be imported here (it needs OpenCV):
  surface_normal(resolution, size, z)   :37-80   -> (Nx, Ny, Nz), GPU
  image_filling(im)                     :82-94   -> filled uint8 image, GPU (flood fill = FIM
                                                    reachability from (0, 0))
  structural_disk(r)                    :96-105  -> uint8 disk (host, as the reference)
  cost_map(Zs, resolution, size)        :1101-1216 -> (cMap, obstMap) exactly as main() holds
                                                    them before FM.biComputeTmap(cMap.T, ...)
  load_dem(mapDirectory)                :1098-1099 -> Zs, the DEM text parsed by host threads
All GPU work goes through libeikonal.so (include/eikonal.h: eik_costmap_*); no CPU fallback.
"""
import math

import numpy as np

from eikonal import _lib as L


def load_dem(mapDirectory):
    """Coupled_motion_planner.py:1098-1099: Zs from <mapDirectory>PRL_DEM.txt (comma-separated
    rows), parsed by libeikonal's host threads; values identical to float() per entry."""
    return L.load_dem_txt(str(mapDirectory) + "PRL_DEM.txt")


def _ctx():
    return L.default_context()


def surface_normal(resolution, size, z):
    """Coupled_motion_planner.py:37-80.  The reference builds its grid with
    linspace(0, size, round(size / resolution)) and requires z of that shape."""
    z = np.asarray(z, dtype=np.float64)
    n0 = int(round(size / resolution))
    if z.shape != (n0, n0):
        raise ValueError(f"z has shape {z.shape}, the grid of size/resolution is {(n0, n0)}")
    return _ctx().surface_normal(z, size)


def image_filling(im):
    """Coupled_motion_planner.py:82-94: holes of a 0/1 uint8 image filled (cv2.floodFill from
    (0, 0), 4-connected; an image whose (0, 0) pixel is 1 comes back all ones, as the reference's)."""
    im = np.asarray(im)
    if im.dtype != np.uint8:
        raise TypeError("image_filling expects a uint8 image (the reference calls it on np.uint8)")
    return _ctx().image_fill(im)


def structural_disk(r):
    """Coupled_motion_planner.py:96-105: (2r+1) x (2r+1) uint8 disk of radius r."""
    se = np.zeros((2 * r + 1, 2 * r + 1), np.uint8)
    for i in range(2 * r + 1):
        for j in range(2 * r + 1):
            if math.sqrt((r - i) ** 2 + (r - j) ** 2) <= r:
                se[i][j] = 1
    return se


def cost_map(Zs, resolution, size, slope_max=0.20, diagonal=0.9, expansion=1.0, gradient=10.0):
    """main()'s cost raster (Coupled_motion_planner.py:1101-1216) from the DEM Zs (:1098-1099).
    Returns (cMap, obstMap) as the reference holds them: cMap indexed [x, y] (the planner passes
    cMap.T to FM.biComputeTmap, :1222), obstMap [y, x] float64."""
    Zs = np.asarray(Zs, dtype=np.float64)
    p = L.CostmapParams(slope_max, diagonal, expansion, gradient, 300.0)
    cost, obst = _ctx().costmap(Zs, resolution, size, p)
    return cost.T, obst.astype(np.float64)
