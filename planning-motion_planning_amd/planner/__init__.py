"""Step 1 of the coupled rover planner on the GPU.

Coupled_motion_planner.py main() (:1092-1258) plans the rover's path to the sample as: DEM ->
cost raster (:1101-1216) -> FM.biComputeTmap(cMap.T, sampleNode, roverNode) (:1222) -> two
FM.getPathGDM descents from nodeJoin (:1225-1226) -> one path in metres with z and heading
(:1228-1252).  `rover_path` runs that chain as one device-resident pipeline through the C ABI
(eik_rover_path_f64: cost builder, both fronts as one fp64 batch, device join, path kernels),
with the host tail (eik_rover_assemble) bit-identical to the reference's numpy statements.
The join is evaluated from the two full fields' pop ranks (ties ranked by node index), see
FastMarching.biComputeTmap.
"""
import numpy as np

from eikonal import _lib as L

ZP = 0.07   # height of the rover reference system above the floor, :1132
TAU = 0.5   # GDM step, :1225-1226

_ctx_obj = None


def _ctx():
    global _ctx_obj
    if _ctx_obj is None:
        import eikonal

        _ctx_obj = eikonal.Context(0)
    return _ctx_obj


def query(xm, ym, xr, yr, initialHeading, resolution, size, zp=ZP, tau=TAU):
    return L.RoverQuery(float(xm), float(ym), float(xr), float(yr), float(initialHeading), float(resolution),
                        float(size), float(zp), float(tau))


def rover_path(Zs, xm, ym, xr, yr, initialHeading, resolution, size, zp=ZP, tau=TAU):
    """main()'s step 1 from the raw DEM Zs (as loaded at :1098-1099) with main()'s arguments.
    Returns (roverPath (N, 3) float64 metres, heading (N,) float64, nodeJoin uint32 (2,))."""
    q = query(xm, ym, xr, yr, initialHeading, resolution, size, zp, tau)
    return _ctx().rover_path(np.asarray(Zs, dtype=np.float64), q)


def assemble(pathS, pathG, Zs, xm, ym, xr, yr, initialHeading, resolution, size=1.0, zp=ZP, tau=TAU):
    """The host tail alone (:1228-1252): the two GDM paths -> (roverPath, heading).  No GPU."""
    q = query(xm, ym, xr, yr, initialHeading, resolution, size, zp, tau)
    return L.rover_assemble(pathS, pathG, Zs, q)
