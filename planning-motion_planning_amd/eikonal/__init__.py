"""MI355X Eikonal solver: ctypes front-end of libeikonal.so (include/eikonal.h).

This is the host-side runtime the drop-in ``FastMarching`` package (and bench.py) call.  There
is no CPU fallback: if the HIP library is missing or no GPU is visible, every entry point raises.
"""
from ._lib import (EikError, Context, Fim2d, Fim3dLayered, lib, LIB_PATH, EIK_F32, EIK_F64,  # noqa: F401
                   PATH_DONE, PATH_FALLBACK, PATH_ERROR, default_context)
