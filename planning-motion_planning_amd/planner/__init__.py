"""Step 1 of the coupled rover planner on the GPU.

Coupled_motion_planner.py main() (:1092-1258) plans the rover's path to the sample as: DEM ->
cost raster (:1101-1216) -> FM.biComputeTmap(cMap.T, sampleNode, roverNode) (:1222) -> two
FM.getPathGDM descents from nodeJoin (:1225-1226) -> one path in metres with z and heading
(:1228-1252).  `rover_path` runs that chain as one device-resident pipeline through the C ABI
(eik_rover_path_f64: cost builder, both fronts as one fp64 batch, device join, path kernels),
with the host tail (eik_rover_assemble) bit-identical to the reference's numpy statements.
The join is evaluated from the two full fields' pop ranks (ties ranked by node index), see
FastMarching.biComputeTmap; EIKONAL_EXACT_BAND=1 (read per call, as the FastMarching drop-ins do)
replays the reference's own band instead -- its nodeJoin and partial fields bit for bit, and the
end-effector early exit's band (EIK_OPT_EXACT_BAND).
"""
import os

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
    _ctx_obj.set_option(L.OPT_EXACT_BAND, 1 if os.environ.get("EIKONAL_EXACT_BAND", "0") not in ("", "0") else 0)
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


# ------------------------------------------------------------------ step 3: the end-effector volume
def volume(sX, sY, sZ, resX, resY, resZ, xm=0.0, ym=0.0, rlim=0.527, rO=(0.4241 + 0.1105) / 2, rm=0.1105,
           finalWayPointArm=(0, 0, 0), initialWayPointArm=(0, 0, 0)):
    """eik_arm_volume from main()'s variables (:1121-1124, :1528-1534, :1573-1574)."""
    v = L.ArmVolume()
    v.sX, v.sY, v.sZ = int(sX), int(sY), int(sZ)
    v.resX, v.resY, v.resZ = float(resX), float(resY), float(resZ)
    v.xm, v.ym = float(xm), float(ym)
    v.rlim, v.rO, v.rm = float(rlim), float(rO), float(rm)
    for k in range(3):
        v.final_wp[k] = int(finalWayPointArm[k])
        v.initial_wp[k] = int(initialWayPointArm[k])
    return v


def GetObstMap(ZsMap, resX, resY, resZ, sX, sY, sZ, newObstMap, xm, ym):
    """Drop-in of Coupled_motion_planner.py:319-358 -> (finalMap, obstMap, groundMap) on the GPU."""
    v = volume(sX, sY, sZ, resX, resY, resZ, xm, ym)
    return _ctx().arm_obst_map(np.asarray(ZsMap, np.float64), np.asarray(newObstMap, np.float64), v)


def TunnelCost(rlim, rO, rm, gamma2D, sX, sY, sZ, resX, resY, resZ, finalBaseHeading, finalWayPointArm,
               initialWayPointArm):
    """Drop-in of Coupled_motion_planner.py:505-725 -> Cmap (sY, sX, sZ) on the GPU, bit-identical."""
    v = volume(sX, sY, sZ, resX, resY, resZ, rlim=rlim, rO=rO, rm=rm, finalWayPointArm=finalWayPointArm,
               initialWayPointArm=initialWayPointArm)
    return _ctx().arm_tunnel_cost(np.asarray(gamma2D, np.float64), np.asarray(finalBaseHeading, np.float64), v)


def arm_path(ZsMap, newObstMap, effectorBasePath, effectorBaseHeading, sX, sY, sZ, resX, resY, resZ, xm, ym,
             finalWayPointArm, initialWayPointArm, Rlim=0.527, rO=(0.4241 + 0.1105) / 2, rm=0.1105, tau=TAU):
    """main() :1562-1588 as one device pipeline: Cmap = GetObstMap * TunnelCost, FM3D.computeTmap from
    the sample node, FM3D.getPathGDM from the start node -> (gamma3D node coordinates (K, 3), status)."""
    v = volume(sX, sY, sZ, resX, resY, resZ, xm, ym, Rlim, rO, rm, finalWayPointArm, initialWayPointArm)
    return _ctx().arm_path(ZsMap, newObstMap, effectorBasePath, effectorBaseHeading, v, tau)
