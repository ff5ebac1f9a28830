"""The partial-field band bracket shared by the early-exit / bidirectional parity tests.

The reference's narrow band (FastMarching3D.py:77-95, FastMarching.py:141-155) holds TENTATIVE
values that depend on its sequential update order; the GPU holds the band cells' final values
(DESIGN.md §3.7), so GPU <= reference always, and reference <= BAND_BRACKET x GPU.  Measured worst
case: 1.5 % on the reference fixtures, 2.6 % on the random end-effector areas of test_gpu_arm.py
(round 3); the bracket is 3 %.  Every failure message reports the measured ratio.  It applies to the
default mode only: EIK_OPT_EXACT_BAND replays the reference's band (tests/test_gpu_bidir_exact.py:
bit-identical; tests/test_gpu_fm3d_exact.py: masks identical, values within 1e-11)."""
import numpy as np

BAND_BRACKET = 1.03


def band_ratio(T, R, mask):
    """max over mask of reference / GPU (1.0 where both are 0)."""
    t, r = T[mask].astype(np.float64), R[mask].astype(np.float64)
    if t.size == 0:
        return 1.0
    with np.errstate(divide="ignore", invalid="ignore"):
        q = np.where(t > 0, r / t, np.where(r > 0, np.inf, 1.0))
    return float(q.max())
