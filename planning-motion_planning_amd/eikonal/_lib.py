"""ctypes binding of libeikonal.so (include/eikonal.h), mirroring the C ABI one-to-one."""
import ctypes as C
import os
import threading

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("EIKONAL_LIB", os.path.join(PKG_DIR, "lib", "libeikonal.so"))

EIK_OK, EIK_ERR_ARG, EIK_ERR_HIP, EIK_ERR_NOMEM, EIK_ERR_NOCONVERGE, EIK_ERR_UNREACHABLE, EIK_ERR_NODEVICE = \
    0, -1, -2, -3, -4, -5, -6
EIK_F32, EIK_F64 = 0, 1
PATH_DONE, PATH_FALLBACK, PATH_ERROR = 0, 1, 2
OPT_MAX_ROUNDS, OPT_SYNC_EVERY, OPT_TIMING, OPT_GRID, OPT_TOL, OPT_DELTA = 0, 1, 2, 3, 4, 5
OPT_MODE, OPT_QTIMEOUT, OPT_MAX_VISITS, OPT_PASSES, OPT_FRESH_FIRST, OPT_SCHED, OPT_PATH_LOOP = 6, 7, 8, 9, 10, 11, 12
OPT_FRONTS_CAP, OPT_LIVE_PACK, OPT_PRIO, OPT_LAYER_PLANAR, OPT_PRIO_RING, OPT_PRIO_DISPATCH = 13, 14, 15, 16, 17, 18
OPT_EXACT_BAND = 19
MODE_LIST, MODE_PERSISTENT = 0, 1

i64 = C.c_int64
vp = C.c_void_p
_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")


class CostmapParams(C.Structure):
    """eik_costmap_params (include/eikonal.h): the cost builder's constants."""
    _fields_ = [("slope_max", C.c_double), ("diagonal", C.c_double), ("expansion", C.c_double),
                ("gradient", C.c_double), ("high", C.c_double)]


class RoverQuery(C.Structure):
    """eik_rover_query (include/eikonal.h): main()'s step-1 arguments (Coupled_motion_planner.py:1092)."""
    _fields_ = [("xm", C.c_double), ("ym", C.c_double), ("xr", C.c_double), ("yr", C.c_double),
                ("initial_heading", C.c_double), ("resolution", C.c_double), ("size", C.c_double),
                ("zp", C.c_double), ("tau", C.c_double)]


class ArmVolume(C.Structure):
    """eik_arm_volume (include/eikonal.h): the end-effector volume of main() step 3."""
    _fields_ = [("sX", i64), ("sY", i64), ("sZ", i64), ("resX", C.c_double), ("resY", C.c_double),
                ("resZ", C.c_double), ("xm", C.c_double), ("ym", C.c_double), ("rlim", C.c_double),
                ("rO", C.c_double), ("rm", C.c_double), ("final_wp", C.c_uint32 * 3), ("initial_wp", C.c_uint32 * 3)]


class EikStats(C.Structure):
    _fields_ = [("iterations", i64), ("tile_visits", i64), ("host_syncs", i64), ("solve_ms", C.c_double),
                ("sweep_ms", C.c_double), ("bytes_alg", C.c_double), ("inplace_passes", i64),
                ("fresh_visits", i64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class EikError(RuntimeError):
    def __init__(self, code, msg):
        self.code = code
        super().__init__(f"eikonal error {code}: {msg}")


_lib = None
_lock = threading.Lock()


def _share_hip_runtime():
    """Use ONE HIP runtime per process.  PyTorch-ROCm ships its own libamdhip64 (requested by
    its libraries as "libamdhip64.so", soname libamdhip64.so.7); libeikonal asks for
    "libamdhip64.so.7".  Whichever loads first, the other would otherwise map a second copy of
    the runtime (and of HSA) into the process.  When torch is installed, pre-load the very file
    torch uses so both resolve to it (the loader de-duplicates by soname and by file)."""
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    libdir = os.path.join(list(spec.submodule_search_locations)[0], "lib")
    for name in ("libhsa-runtime64.so", "libamdhip64.so"):
        p = os.path.join(libdir, name)
        if os.path.exists(p):
            C.CDLL(p, mode=C.RTLD_GLOBAL)


# Sanitizer runs only (tools/san.sh): EIKONAL_HOST_LIB names an ASan/UBSan build of the
# host-only sources (dem_io.cpp, rover.cpp, node_sync.cpp: `make -C csrc san`), and lib() then binds
# just their entry points from it -- no HIP runtime in the process, nothing of the GPU path.
HOST_LIB = os.environ.get("EIKONAL_HOST_LIB")


def _bind_host(L):
    P = C.POINTER
    L.eik_load_dem_txt.argtypes = [C.c_char_p, vp, i64, P(i64), P(i64), C.c_int]
    L.eik_io_last_error.restype = C.c_char_p
    L.eik_node_allreduce.argtypes = [vp, C.c_int, C.c_int, C.c_uint64, i64, P(i64), C.c_double]
    L.eik_node_shm_open.argtypes = [C.c_char_p, i64, C.c_int, P(vp)]
    L.eik_node_shm_close.argtypes = [vp, i64]
    L.eik_node_shm_unlink.argtypes = [C.c_char_p]
    L.eik_rover_assemble.argtypes = [_f64p, i64, _f64p, i64, _f64p, i64, i64, P(RoverQuery), _f64p, _f64p, i64,
                                     P(i64)]


def lib():
    """Load libeikonal.so; raise (never fall back) when it is absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if HOST_LIB:
            _lib = C.CDLL(HOST_LIB)
            _bind_host(_lib)
            return _lib
        if not os.path.exists(LIB_PATH):
            raise EikError(EIK_ERR_NODEVICE, f"{LIB_PATH} not built (run __graft_entry__.build())")
        _share_hip_runtime()
        L = C.CDLL(LIB_PATH)
        P = C.POINTER
        L.eik_version.restype = C.c_char_p
        L.eik_create.argtypes = [C.c_int, P(vp)]
        L.eik_destroy.argtypes = [vp]
        L.eik_destroy.restype = None
        L.eik_last_error.argtypes = [vp]
        L.eik_last_error.restype = C.c_char_p
        L.eik_set_option.argtypes = [vp, C.c_int, C.c_double]
        L.eik_get_stats.argtypes = [vp, P(EikStats)]
        L.eik_tmap2d_f32.argtypes = [vp, _f32p, i64, i64, i64, i64, _f32p]
        L.eik_tmap2d_f64.argtypes = [vp, _f64p, i64, i64, i64, i64, _f64p]
        L.eik_tmap2d_bidir_f64.argtypes = [vp, _f64p, i64, i64, i64, i64, i64, i64, _f64p, _f64p, _u32p]
        L.eik_bidir_join_f64.argtypes = [vp, _f64p, _f64p, i64, i64, _f64p, _f64p, _u32p, _i64p]
        L.eik_fronts_info.argtypes = [vp, _i64p]
        L.eik_exact_info.argtypes = [vp, _i64p]
        L.eik_tmap2d_batch_f32.argtypes = [vp, _f32p, i64, i64, i64, _i64p, _f32p]
        L.eik_path2d_f64.argtypes = [vp, _f64p, i64, i64, _f64p, _f64p, C.c_double, _f64p, i64, P(i64), P(C.c_int)]
        L.eik_gradient2d_f64.argtypes = [vp, _f64p, i64, i64, _f64p, _f64p]
        L.eik_selftest_walker_math.argtypes = [vp, i64, C.c_uint64, _i64p]
        L.eik_fim2d_create.argtypes = [vp, i64, i64, i64, C.c_int, P(vp)]
        L.eik_fim2d_destroy.argtypes = [vp]
        L.eik_fim2d_destroy.restype = None
        L.eik_fim2d_set_ghosts.argtypes = [vp, vp, vp, vp, vp]
        L.eik_fim2d_start.argtypes = [vp, vp, vp, _i64p, vp]
        L.eik_fim2d_iterate.argtypes = [vp, i64, P(i64)]
        L.eik_fim2d_solve.argtypes = [vp, vp, vp, _i64p, vp]
        L.eik_fim2d_pack_edges.argtypes = [vp, vp, vp, vp, vp]
        L.eik_fim2d_merge_ghost.argtypes = [vp, C.c_int, vp]
        L.eik_fim2d_active.argtypes = [vp, P(i64)]
        L.eik_fim2d_stats.argtypes = [vp, P(EikStats)]
        L.eik_path2d_dev.argtypes = [vp, vp, C.c_int, i64, i64, _f64p, _f64p, C.c_double, vp, i64, vp, vp, vp]
        L.eik_tmap3d_f32.argtypes = [vp, _f32p, i64, i64, i64, _i64p, _f32p]
        L.eik_tmap3d_f64.argtypes = [vp, _f64p, i64, i64, i64, _i64p, _f64p]
        L.eik_tmap3d_early_f32.argtypes = [vp, _f32p, i64, i64, i64, _i64p, _i64p, _f32p]
        L.eik_tmap3d_early_f64.argtypes = [vp, _f64p, i64, i64, i64, _i64p, _i64p, _f64p]
        L.eik_fim3d_early_exit.argtypes = [vp, vp, vp, vp, i64, i64, i64, C.c_int, _i64p, _i64p, vp]
        L.eik_path3d_f64.argtypes = [vp, _f64p, i64, i64, i64, _f64p, _f64p, C.c_double, _f64p, i64, P(i64),
                                     P(C.c_int)]
        L.eik_fim3d_solve.argtypes = [vp, vp, vp, i64, i64, i64, C.c_int, _i64p, vp]
        L.eik_path3d_dev.argtypes = [vp, vp, C.c_int, i64, i64, i64, _f64p, _f64p, C.c_double, vp, i64, vp, vp, vp]
        L.eik_costmap_f64.argtypes = [vp, _f64p, i64, i64, C.c_double, C.c_double, P(CostmapParams), _f64p, vp]
        L.eik_costmap_dev.argtypes = [vp, vp, i64, i64, C.c_double, C.c_double, P(CostmapParams), vp, vp, vp]
        L.eik_surface_normal_f64.argtypes = [vp, _f64p, i64, i64, C.c_double, _f64p, _f64p, _f64p]
        L.eik_image_fill_u8.argtypes = [vp, _u8p, i64, i64, _u8p]
        L.eik_disk_morph_u8.argtypes = [vp, _u8p, i64, i64, C.c_int, C.c_int, _u8p]
        L.eik_load_dem_txt.argtypes = [C.c_char_p, vp, i64, P(i64), P(i64), C.c_int]
        L.eik_io_last_error.restype = C.c_char_p
        L.eik_fim2d_live_bind.argtypes = [vp, vp * 8, vp * 8]
        L.eik_fim2d_launch.argtypes = [vp, C.c_int]
        L.eik_fim2d_live_pack.argtypes = [vp, C.c_int]
        L.eik_fim2d_live_merge.argtypes = [vp, C.c_int, P(i64), P(i64)]
        L.eik_fim2d_release.argtypes = [vp, P(i64)]
        L.eik_node_allreduce.argtypes = [vp, C.c_int, C.c_int, C.c_uint64, i64, P(i64), C.c_double]
        L.eik_node_shm_open.argtypes = [C.c_char_p, i64, C.c_int, P(vp)]
        L.eik_node_shm_close.argtypes = [vp, i64]
        L.eik_node_shm_unlink.argtypes = [C.c_char_p]
        L.eik_host_alloc.argtypes = [i64, P(vp)]
        L.eik_host_free.argtypes = [vp]
        L.eik_ipc_alloc.argtypes = [vp, i64, P(vp), C.c_char_p]
        L.eik_ipc_free.argtypes = [vp, vp]
        L.eik_ipc_open.argtypes = [vp, C.c_char_p, P(vp)]
        L.eik_ipc_close.argtypes = [vp, vp]
        L.eik_rover_assemble.argtypes = [_f64p, i64, _f64p, i64, _f64p, i64, i64, P(RoverQuery), _f64p, _f64p, i64,
                                         P(i64)]
        L.eik_rover_path_f64.argtypes = [vp, _f64p, i64, i64, P(RoverQuery), P(CostmapParams), _f64p, _f64p, i64,
                                         P(i64), _u32p, vp]
        L.eik_arm_obst_map_f64.argtypes = [vp, _f64p, _f64p, i64, i64, P(ArmVolume), _f64p, vp, vp]
        L.eik_arm_tunnel_cost_f64.argtypes = [vp, _f64p, _f64p, i64, P(ArmVolume), _f64p]
        L.eik_arm_path_f64.argtypes = [vp, _f64p, _f64p, i64, i64, _f64p, _f64p, i64, P(ArmVolume), C.c_double, _f64p,
                                       i64, P(i64), P(C.c_int), vp, vp]
        L.eik_tmap3d_batch_f64.argtypes = [vp, _f64p, i64, i64, i64, i64, _i64p, _f64p]
        L.eik_fim3dl_create.argtypes = [vp, i64, i64, i64, C.c_int, C.c_int, C.c_int, P(vp)]
        L.eik_fim3dl_start.argtypes = [vp, vp, vp, _i64p, vp]
        L.eik_fim2d_qcount.argtypes = [vp, P(C.c_uint64)]
        _lib = L
        return L


EXPORTED = [
    "eik_version", "eik_create", "eik_destroy", "eik_last_error", "eik_set_option", "eik_get_stats",
    "eik_tmap2d_f32", "eik_tmap2d_f64", "eik_tmap2d_bidir_f64", "eik_bidir_join_f64", "eik_fronts_info", "eik_exact_info", "eik_tmap2d_batch_f32", "eik_path2d_f64",
    "eik_gradient2d_f64", "eik_fim2d_create", "eik_fim2d_destroy", "eik_fim2d_set_ghosts", "eik_fim2d_start",
    "eik_fim2d_iterate", "eik_fim2d_solve", "eik_fim2d_pack_edges", "eik_fim2d_merge_ghost", "eik_fim2d_active",
    "eik_fim2d_stats", "eik_path2d_dev", "eik_selftest_walker_math", "eik_tmap3d_f32", "eik_tmap3d_f64",
    "eik_tmap3d_early_f32", "eik_tmap3d_early_f64", "eik_fim3d_early_exit", "eik_path3d_f64", "eik_fim3d_solve",
    "eik_path3d_dev", "eik_costmap_f64", "eik_costmap_dev", "eik_surface_normal_f64", "eik_image_fill_u8", "eik_disk_morph_u8",
    "eik_load_dem_txt", "eik_io_last_error", "eik_fim2d_live_bind", "eik_fim2d_launch", "eik_fim2d_live_pack",
    "eik_fim2d_live_merge", "eik_fim2d_release", "eik_node_allreduce", "eik_node_shm_open",
    "eik_node_shm_close", "eik_node_shm_unlink", "eik_ipc_alloc", "eik_ipc_free", "eik_ipc_open", "eik_ipc_close",
    "eik_rover_assemble", "eik_rover_path_f64", "eik_arm_obst_map_f64", "eik_arm_tunnel_cost_f64",
    "eik_arm_path_f64", "eik_tmap3d_batch_f64", "eik_host_alloc", "eik_host_free", "eik_fim2d_qcount",
    "eik_fim3dl_create", "eik_fim3dl_start",
]


def rover_assemble(pathS, pathG, Z, query, cap=None):
    """Host tail of the planner's step 1 (Coupled_motion_planner.py:1228-1252), no GPU:
    (roverPath (N, 3) metres, heading (N,))."""
    pathS = np.ascontiguousarray(pathS, np.float64)
    pathG = np.ascontiguousarray(pathG, np.float64)
    Z = np.ascontiguousarray(Z, np.float64)
    cap = cap or len(pathS) + len(pathG)
    out = np.empty((cap, 3))
    hd = np.empty(cap)
    n = i64(0)
    rc = lib().eik_rover_assemble(pathS, len(pathS), pathG, len(pathG), Z, Z.shape[0], Z.shape[1], C.byref(query),
                                  out, hd, cap, C.byref(n))
    if rc != EIK_OK:
        raise IndexError(f"rover path: waypoint outside the DEM or buffer too small (rc {rc}, {n.value} rows)")
    return out[: n.value].copy(), hd[: n.value].copy()


def load_dem_txt(path, nthreads=0):
    """Coupled_motion_planner.py:1098-1099 (comma-separated DEM text) -> float64 (H, W), parsed
    by host threads in libeikonal (no GPU)."""
    L = lib()
    H, W = i64(0), i64(0)
    p = os.fsencode(path)
    if L.eik_load_dem_txt(p, None, 0, C.byref(H), C.byref(W), int(nthreads)) != EIK_OK:
        raise ValueError(L.eik_io_last_error().decode())
    out = np.empty((H.value, W.value), np.float64)
    if L.eik_load_dem_txt(p, out.ctypes.data, out.size, C.byref(H), C.byref(W), int(nthreads)) != EIK_OK:
        raise ValueError(L.eik_io_last_error().decode())
    return out


def parse_options(options):
    """{name: value} from a dict or an "A=1,B=2" string; unknown names raise ValueError."""
    if not options:
        return {}
    if isinstance(options, str):
        items = {}
        for item in filter(None, (x.strip() for x in options.split(","))):
            name, eq, val = item.partition("=")
            if not eq:
                raise ValueError(f"solver option {item!r}: expected NAME=VALUE")
            items[name.strip()] = float(val)
        options = items
    out = {}
    for name, val in options.items():
        if "OPT_" + name not in globals():
            known = sorted(k[4:] for k in globals() if k.startswith("OPT_"))
            raise ValueError(f"unknown solver option {name!r} (known: {', '.join(known)})")
        out[name] = float(val)
    return out


def options_from_env(var="EIK_OPTIONS"):
    """The A/B hook of bench.py and tools/: EIK_OPTIONS="PASSES=16,SCHED=1" (opt-in, explicit)."""
    return os.environ.get(var, "")


class Context:
    """One eik_ctx (device state + HIP stream); use one per host thread."""

    def __init__(self, device=0, options=None):
        """options: solver options applied at creation, a dict {name: value} or a string
        "PASSES=16,SCHED=1" (names of the OPT_* constants without the prefix).  Nothing is read
        from the environment here: benches and tools pass options_from_env() explicitly."""
        L = lib()
        h = vp()
        rc = L.eik_create(int(device), C.byref(h))
        if rc != EIK_OK:
            raise EikError(rc, L.eik_last_error(None).decode())
        self._h = h
        self.device = device
        for name, val in parse_options(options).items():
            self.set_option(globals()["OPT_" + name], float(val))

    def _chk(self, rc):
        if rc != EIK_OK:
            raise EikError(rc, lib().eik_last_error(self._h).decode())

    def close(self):
        if getattr(self, "_h", None):
            lib().eik_destroy(self._h)
            self._h = None
            release_pinned()  # the recycled result blocks (bounded, and freed here)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_option(self, opt, value):
        self._chk(lib().eik_set_option(self._h, int(opt), float(value)))

    def stats(self):
        s = EikStats()
        self._chk(lib().eik_get_stats(self._h, C.byref(s)))
        return s.as_dict()

    # -- host-buffer drop-ins -------------------------------------------------------------
    def tmap2d(self, cost, goal, dtype=np.float64):
        cost = np.ascontiguousarray(cost, dtype=dtype)
        H, W = cost.shape
        T = result_empty(cost.shape, cost.dtype)
        fn = lib().eik_tmap2d_f64 if cost.dtype == np.float64 else lib().eik_tmap2d_f32
        self._chk(fn(self._h, cost, H, W, int(goal[0]), int(goal[1]), T))
        return T

    def tmap2d_batch(self, costs, goals):
        costs = np.ascontiguousarray(costs, dtype=np.float32)
        B, H, W = costs.shape
        T = np.empty_like(costs)
        self._chk(lib().eik_tmap2d_batch_f32(self._h, costs, B, H, W, np.ascontiguousarray(goals, np.int64), T))
        return T

    def tmap2d_bidir(self, cost, goal, start):
        cost = np.ascontiguousarray(cost, dtype=np.float64)
        H, W = cost.shape
        TG, TS = result_empty(cost.shape, cost.dtype), result_empty(cost.shape, cost.dtype)
        join = np.zeros(2, np.uint32)
        self._chk(lib().eik_tmap2d_bidir_f64(self._h, cost, H, W, int(goal[0]), int(goal[1]), int(start[0]),
                                             int(start[1]), TG, TS, join))
        return TG, TS, join

    def bidir_join(self, TG, TS):
        """The join step of biComputeTmap (FastMarching.py:141-162) on two given full fields ->
        (TGp, TSp, nodeJoin uint32 (x, y), members: the cells ranked per front)."""
        TG = np.ascontiguousarray(TG, dtype=np.float64)
        TS = np.ascontiguousarray(TS, dtype=np.float64)
        if TG.shape != TS.shape or TG.ndim != 2:
            raise ValueError("TG and TS must be two H x W fields")
        H, W = TG.shape
        TGp, TSp = np.empty_like(TG), np.empty_like(TS)
        join = np.zeros(2, np.uint32)
        members = np.zeros(2, np.int64)
        self._chk(lib().eik_bidir_join_f64(self._h, TG, TS, H, W, TGp, TSp, join, members))
        return TGp, TSp, join, members

    def fronts_info(self):
        """How the last tmap2d_bidir / rover_path formed its fronts (eik_fronts_info)."""
        out = np.zeros(10, np.int64)
        self._chk(lib().eik_fronts_info(self._h, out))
        return {"capped": bool(out[0]), "fallback": bool(out[1]), "kept": out[2:4].tolist(),
                "members": out[4:6].tolist(), "band": out[6:8].tolist(), "band_sweeps": out[8:10].tolist()}

    def exact_info(self):
        """The last tmap2d_bidir / rover_path's exact band replay (EIK_OPT_EXACT_BAND, eik_exact_info):
        re-ranking passes, relaxation sweeps per front, tie-run launches, device time in ms (all 0: it
        did not run)."""
        out = np.zeros(5, np.int64)
        self._chk(lib().eik_exact_info(self._h, out))
        return {"passes": int(out[0]), "sweeps": out[1:3].tolist(), "tie_launches": int(out[3]),
                "ms": out[4] / 1000.0}

    def path2d(self, T, init, end, tau=0.5):
        T = np.ascontiguousarray(T, dtype=np.float64)
        H, W = T.shape
        cap = int(round(15000 / tau)) + 4
        out = np.empty((cap, 2))
        n, st = i64(0), C.c_int(0)
        self._chk(lib().eik_path2d_f64(self._h, T, H, W, np.asarray(init, np.float64)[:2].copy(),
                                       np.asarray(end, np.float64)[:2].copy(), float(tau), out, cap, C.byref(n),
                                       C.byref(st)))
        return out[: n.value].copy(), st.value

    def tmap3d(self, cost, goal, dtype=np.float64, start=None):
        """FastMarching3D.computeTmap: the full field, or with `start` (x, y, z) the reference's
        early-exit field (break once `start` is popped, FastMarching3D.py:141)."""
        cost = np.ascontiguousarray(cost, dtype=dtype)
        H, W, Lz = cost.shape
        T = result_empty(cost.shape, cost.dtype)
        g = np.ascontiguousarray(np.asarray(goal).reshape(-1)[:3], np.int64)
        f64 = cost.dtype == np.float64
        if start is None:
            fn = lib().eik_tmap3d_f64 if f64 else lib().eik_tmap3d_f32
            self._chk(fn(self._h, cost, H, W, Lz, g, T))
        else:
            s = np.ascontiguousarray(np.asarray(start).reshape(-1)[:3], np.int64)
            fn = lib().eik_tmap3d_early_f64 if f64 else lib().eik_tmap3d_early_f32
            self._chk(fn(self._h, cost, H, W, Lz, g, s, T))
        return T

    def path3d(self, T, init, end, tau=0.5):
        T = np.ascontiguousarray(T, dtype=np.float64)
        H, W, Lz = T.shape
        cap = int(round(15000 / tau)) + 4
        out = np.empty((cap, 3))
        n, st = i64(0), C.c_int(0)
        self._chk(lib().eik_path3d_f64(self._h, T, H, W, Lz, np.asarray(init, np.float64)[:3].copy(),
                                       np.asarray(end, np.float64)[:3].copy(), float(tau), out, cap, C.byref(n),
                                       C.byref(st)))
        return out[: n.value].copy(), st.value

    def costmap(self, Z, resolution, size, params=None):
        """Coupled_motion_planner.py:1101-1216 on the GPU: (cost [y][x] = the reference's cMap.T,
        obstacle map [y][x] uint8)."""
        Z = np.ascontiguousarray(Z, dtype=np.float64)
        H, W = Z.shape
        cost = np.empty_like(Z)
        obst = np.empty((H, W), np.uint8)
        p = C.byref(params) if params is not None else None
        self._chk(lib().eik_costmap_f64(self._h, Z, H, W, float(resolution), float(size), p, cost, obst.ctypes.data))
        return cost, obst

    def rover_path(self, Z, query, params=None, want_cost=False):
        """Planner step 1 on the GPU (Coupled_motion_planner.py:1097-1258): DEM -> (roverPath (N, 3),
        heading (N,), nodeJoin uint32 (2,)[, cost raster [y][x]])."""
        Z = np.ascontiguousarray(Z, dtype=np.float64)
        H, W = Z.shape
        cap = 2 * int(round(15000 / query.tau)) + 8
        out = np.empty((cap, 3))
        hd = np.empty(cap)
        n = i64(0)
        join = np.zeros(2, np.uint32)
        cost = np.empty_like(Z) if want_cost else None
        p = C.byref(params) if params is not None else None
        self._chk(lib().eik_rover_path_f64(self._h, Z, H, W, C.byref(query), p, out, hd, cap, C.byref(n), join,
                                           cost.ctypes.data if want_cost else None))
        res = (out[: n.value].copy(), hd[: n.value].copy(), join)
        return res + (cost,) if want_cost else res

    def arm_obst_map(self, ZsMap, newObstMap, vol, all_maps=True):
        """GetObstMap (Coupled_motion_planner.py:319-358) -> (finalMap, obstMap, groundMap)."""
        Z = np.ascontiguousarray(ZsMap, dtype=np.float64)
        O = np.ascontiguousarray(newObstMap, dtype=np.float64)
        shape = (vol.sX, vol.sY, vol.sZ)
        f = np.empty(shape)
        o = np.empty(shape) if all_maps else None
        g = np.empty(shape) if all_maps else None
        self._chk(lib().eik_arm_obst_map_f64(self._h, Z, O, Z.shape[0], Z.shape[1], C.byref(vol), f,
                                             o.ctypes.data if all_maps else None, g.ctypes.data if all_maps else None))
        return f, o, g

    def arm_tunnel_cost(self, gamma2D, heading, vol):
        """TunnelCost (Coupled_motion_planner.py:505-725) -> Cmap (sY, sX, sZ)."""
        g = np.ascontiguousarray(gamma2D, dtype=np.float64)
        h = np.ascontiguousarray(heading, dtype=np.float64)
        out = np.empty((vol.sY, vol.sX, vol.sZ))
        self._chk(lib().eik_arm_tunnel_cost_f64(self._h, g, h, g.shape[0], C.byref(vol), out))
        return out

    def arm_path(self, ZsMap, newObstMap, gamma2D, heading, vol, tau=0.5, want_fields=False):
        """:1562-1593: cost volume -> FM3D field -> end-effector path (K, 3) node coordinates."""
        Z = np.ascontiguousarray(ZsMap, dtype=np.float64)
        O = np.ascontiguousarray(newObstMap, dtype=np.float64)
        g = np.ascontiguousarray(gamma2D, dtype=np.float64)
        h = np.ascontiguousarray(heading, dtype=np.float64)
        cap = int(round(15000 / tau)) + 4
        out = np.empty((cap, 3))
        n, st = i64(0), C.c_int(0)
        shape = (vol.sY, vol.sX, vol.sZ)
        cost = np.empty(shape) if want_fields else None
        T = np.empty(shape) if want_fields else None
        self._chk(lib().eik_arm_path_f64(self._h, Z, O, Z.shape[0], Z.shape[1], g, h, g.shape[0], C.byref(vol),
                                         float(tau), out, cap, C.byref(n), C.byref(st),
                                         cost.ctypes.data if want_fields else None,
                                         T.ctypes.data if want_fields else None))
        res = (out[: n.value].copy(), st.value)
        return res + (cost, T) if want_fields else res

    def tmap3d_batch(self, cost, goals):
        """FastMarching3D.computeTmap on B volumes (B, H, W, L) in one solve; goals (B, 3) (x, y, z)."""
        cost = np.ascontiguousarray(cost, dtype=np.float64)
        B, H, W, Lz = cost.shape
        g = np.ascontiguousarray(goals, np.int64).reshape(-1)
        T = result_empty(cost.shape, cost.dtype)
        self._chk(lib().eik_tmap3d_batch_f64(self._h, cost, B, H, W, Lz, g, T))
        return T

    def surface_normal(self, Z, size):
        Z = np.ascontiguousarray(Z, dtype=np.float64)
        H, W = Z.shape
        nx, ny, nz = np.empty_like(Z), np.empty_like(Z), np.empty_like(Z)
        self._chk(lib().eik_surface_normal_f64(self._h, Z, H, W, float(size), nx, ny, nz))
        return nx, ny, nz

    def image_fill(self, im):
        im = np.ascontiguousarray(im, dtype=np.uint8)
        H, W = im.shape
        out = np.empty_like(im)
        self._chk(lib().eik_image_fill_u8(self._h, im, H, W, out))
        return out

    def disk_morph(self, im, radius, erode):
        """cv2.erode / cv2.dilate of a 0/1 mask with structural_disk(radius) (eik_disk_morph_u8)."""
        im = np.ascontiguousarray(im, dtype=np.uint8)
        H, W = im.shape
        out = np.empty_like(im)
        self._chk(lib().eik_disk_morph_u8(self._h, im, H, W, int(radius), int(bool(erode)), out))
        return out

    def gradient2d(self, T):
        T = np.ascontiguousarray(T, dtype=np.float64)
        H, W = T.shape
        gx, gy = np.empty_like(T), np.empty_like(T)
        self._chk(lib().eik_gradient2d_f64(self._h, T, H, W, gx, gy))
        return gx, gy


class Fim2d:
    """Device-resident solver (eik_fim2d): device pointers in, async on a caller stream."""

    def __init__(self, ctx, B, H, W, dtype=EIK_F32):
        self.ctx = ctx
        h = vp()
        ctx._chk(lib().eik_fim2d_create(ctx._h, int(B), int(H), int(W), int(dtype), C.byref(h)))
        self._h = h
        self.B, self.H, self.W, self.dtype = B, H, W, dtype

    def close(self):
        if getattr(self, "_h", None):
            lib().eik_fim2d_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_ghosts(self, n, s, w, e):
        self.ctx._chk(lib().eik_fim2d_set_ghosts(self._h, n, s, w, e))

    def start(self, d_cost, d_T, goals, stream=None):
        self.ctx._chk(lib().eik_fim2d_start(self._h, d_cost, d_T, np.ascontiguousarray(goals, np.int64).reshape(-1),
                                            stream))

    def iterate(self, max_iters):
        a = i64(0)
        self.ctx._chk(lib().eik_fim2d_iterate(self._h, int(max_iters), C.byref(a)))
        return a.value

    def solve(self, d_cost, d_T, goals, stream=None):
        self.ctx._chk(lib().eik_fim2d_solve(self._h, d_cost, d_T, np.ascontiguousarray(goals, np.int64).reshape(-1),
                                            stream))

    def pack_edges(self, n, s, w, e):
        self.ctx._chk(lib().eik_fim2d_pack_edges(self._h, n, s, w, e))

    def merge_ghost(self, side, recv):
        self.ctx._chk(lib().eik_fim2d_merge_ghost(self._h, int(side), recv))

    def active(self):
        a = i64(0)
        self.ctx._chk(lib().eik_fim2d_active(self._h, C.byref(a)))
        return a.value

    def stats(self):
        s = EikStats()
        self.ctx._chk(lib().eik_fim2d_stats(self._h, C.byref(s)))
        return s.as_dict()

    # live domain decomposition (eik_fim2d_live_bind / launch / live_pack / live_merge / release)
    def live_bind(self, send, recv):
        """send, recv: [parity][side] device addresses (int) or None"""
        S = (vp * 8)(*[send[p][s] for p in range(2) for s in range(4)])
        R = (vp * 8)(*[recv[p][s] for p in range(2) for s in range(4)])
        self.ctx._chk(lib().eik_fim2d_live_bind(self._h, S, R))

    def launch(self, live=True):
        self.ctx._chk(lib().eik_fim2d_launch(self._h, 1 if live else 0))

    def live_pack(self, parity):
        self.ctx._chk(lib().eik_fim2d_live_pack(self._h, int(parity)))

    def live_merge(self, parity):
        a, c = i64(0), i64(0)
        self.ctx._chk(lib().eik_fim2d_live_merge(self._h, int(parity), C.byref(a), C.byref(c)))
        return a.value, c.value

    def release(self):
        a = i64(0)
        self.ctx._chk(lib().eik_fim2d_release(self._h, C.byref(a)))
        return a.value


class Fim3dLayered(Fim2d):
    """A block of a domain-decomposed few-layer 3D volume (eik_fim3dl_create: the layered solver on a
    [H][W][L] block, layers z0 .. z0+nl-1; ghost strips of nl values per edge cell).  The eik_fim2d
    methods apply; start takes the goal as (x, y, z) with z absolute (x < 0: not in this block)."""

    def __init__(self, ctx, H, W, L, z0, nl, dtype=EIK_F32):
        self.ctx = ctx
        h = vp()
        ctx._chk(lib().eik_fim3dl_create(ctx._h, int(H), int(W), int(L), int(z0), int(nl), int(dtype), C.byref(h)))
        self._h = h
        self.B, self.H, self.W, self.dtype = 1, H, W, dtype
        self.L, self.z0, self.nl = L, z0, nl

    def start(self, d_cost, d_T, goal, stream=None):
        g = np.asarray(goal, np.int64).reshape(3)
        self.ctx._chk(lib().eik_fim3dl_start(self._h, d_cost, d_T, g, stream))


# ----------------------------------------------------------------- pinned result arrays
# The drop-in returns fields of up to hundreds of MiB (a 4096^2 float64 raster is 128 MiB) that the
# caller hands straight back (computeTmap -> getPathGDM).  Allocated in page-locked memory
# (eik_host_alloc), they cross PCIe as one DMA each way instead of through the C ABI's staging
# ring.  Blocks are recycled by size: a returned array owns its block until the last view of it
# is gone, then the block goes back to the pool (hipHostMalloc of 128 MiB costs milliseconds).
PINNED_MIN_BYTES = 16 << 20  # below this the ABI copies directly anyway
_pin_lock = threading.Lock()
_pin_free = {}  # nbytes -> [ptr, ...], oldest first
_PIN_POOL_BYTES = 512 << 20  # free blocks kept, all sizes together (e.g. four 4096^2 float64 fields)


def _pool_bytes():
    return sum(n * len(v) for n, v in _pin_free.items())


def release_pinned():
    """Give every recycled page-locked block back to the runtime (blocks still held by live
    arrays return to the pool when their arrays go; Context.close() calls this)."""
    with _pin_lock:
        ptrs = [p for v in _pin_free.values() for p in v]
        _pin_free.clear()
    for p in ptrs:
        lib().eik_host_free(p)


class _PinnedBlock:
    def __init__(self, nbytes):
        self.nbytes = nbytes
        with _pin_lock:
            free = _pin_free.get(nbytes)
            ptr = free.pop() if free else None
        if ptr is None:
            p = vp()
            if lib().eik_host_alloc(int(nbytes), C.byref(p)) != EIK_OK:
                raise MemoryError(lib().eik_last_error(None).decode())
            ptr = p.value
        self.ptr = ptr

    def __del__(self):
        try:
            evict = []
            with _pin_lock:
                if self.nbytes > _PIN_POOL_BYTES:
                    evict.append(self.ptr)
                else:
                    _pin_free.setdefault(self.nbytes, []).append(self.ptr)
                    # over the byte budget: free the oldest blocks of the other sizes first
                    while _pool_bytes() > _PIN_POOL_BYTES:
                        n = next((k for k, v in _pin_free.items() if v and k != self.nbytes), self.nbytes)
                        evict.append(_pin_free[n].pop(0))
                        if not _pin_free[n]:
                            del _pin_free[n]
            for p in evict:
                lib().eik_host_free(p)
        except Exception:
            pass


def result_empty(shape, dtype):
    """An uninitialised C-contiguous array for a returned field: page-locked (recycled) when at
    least PINNED_MIN_BYTES, else a plain numpy array."""
    dtype = np.dtype(dtype)
    n = int(np.prod(shape)) * dtype.itemsize
    if n < PINNED_MIN_BYTES:
        return np.empty(shape, dtype)
    blk = _PinnedBlock(n)
    buf = (C.c_byte * n).from_address(blk.ptr)
    buf._owner = blk  # the block lives as long as any view of the array
    return np.frombuffer(buf, dtype=dtype).reshape(shape)


class IpcBuffer:
    """A device buffer other processes of the node can map (eik_ipc_alloc / eik_ipc_open)."""

    def __init__(self, ctx, nbytes):
        self.ctx = ctx
        p = vp()
        h = C.create_string_buffer(64)
        ctx._chk(lib().eik_ipc_alloc(ctx._h, int(nbytes), C.byref(p), h))
        self.ptr, self.handle, self.nbytes = p.value, h.raw, int(nbytes)

    def close(self):
        if getattr(self, "ptr", None):
            lib().eik_ipc_free(self.ctx._h, self.ptr)
            self.ptr = None


def ipc_open(ctx, handle):
    p = vp()
    ctx._chk(lib().eik_ipc_open(ctx._h, C.create_string_buffer(bytes(handle), 64), C.byref(p)))
    return p.value


def ipc_close(ctx, ptr):
    ctx._chk(lib().eik_ipc_close(ctx._h, ptr))


_default = {}


def default_context(device=0):
    """Per-thread default context used by the FastMarching drop-in."""
    key = (threading.get_ident(), device)
    c = _default.get(key)
    if c is None:
        c = Context(device)
        _default[key] = c
    return c


def node_shm_open(name, nbytes, create):
    p = vp()
    rc = lib().eik_node_shm_open(name.encode(), int(nbytes), 1 if create else 0, C.byref(p))
    if rc != EIK_OK:
        raise EikError(rc, f"shared memory segment {name!r} could not be {'created' if create else 'opened'}")
    return p.value


def node_shm_close(addr, nbytes):
    lib().eik_node_shm_close(addr, int(nbytes))


def node_shm_unlink(name):
    lib().eik_node_shm_unlink(name.encode())


def node_allreduce(addr, rank, world, rnd, value, timeout_s=60.0):
    """eik_node_allreduce over a shared-memory segment at host address addr."""
    out = i64(0)
    rc = lib().eik_node_allreduce(addr, int(rank), int(world), int(rnd), int(value), C.byref(out), float(timeout_s))
    if rc != EIK_OK:
        raise EikError(rc, "node all-reduce timed out (a rank stopped voting)")
    return out.value
