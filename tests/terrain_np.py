"""Small synthetic DEMs for the cost-builder tests (numpy; same spectral recipe as
eikonal/terrain.py, evaluated on the CPU)."""
import numpy as np


def dem(H, W, seed=0, n_waves=60, rms_slope=0.25, res=0.05):
    rng = np.random.default_rng(seed)
    f = np.exp(rng.uniform(np.log(1 / 256), np.log(1 / 12), n_waves))
    th = rng.uniform(0, 2 * np.pi, n_waves)
    ph = rng.uniform(0, 2 * np.pi, n_waves)
    amp = f ** -1.1 * np.sqrt(f)
    kx, ky = 2 * np.pi * f * np.cos(th), 2 * np.pi * f * np.sin(th)
    scale = rms_slope * res / np.sqrt(0.5 * np.sum((amp * np.hypot(kx, ky)) ** 2))
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
    z = np.zeros((H, W))
    for i in range(n_waves):
        z += amp[i] * scale * np.sin(kx[i] * xx + ky[i] * yy + ph[i])
    return z
