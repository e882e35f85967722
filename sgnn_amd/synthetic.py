"""Synthetic Taylor-bar particle trajectories ("Synthetic inputs").

There is no network and no dataset in this image, so every bench and test
runs on lattices laid out like the reference's real data
(`datasets/taylor_impact_2d/README.md:243-251`: 0.5 mm spacing, x = 0.25 +
0.5 i, y = -9.75 + 0.5 j, x-major with y fastest, as the LS-DYNA parser
emits them).  Frames are a smooth impact-like drift plus a seeded random walk
so that velocity / acceleration features are non-trivial.
"""
from __future__ import annotations

import numpy as np


def lattice_2d(nx: int, ny: int, spacing: float = 0.5,
               x0: float = 0.25, y0: float = -9.75) -> np.ndarray:
    """[nx*ny, 2] float32 lattice, particle index = i*ny + j (y fastest)."""
    xs = x0 + spacing * np.arange(nx, dtype=np.float64)
    ys = y0 + spacing * np.arange(ny, dtype=np.float64)
    gx, gy = np.meshgrid(xs, ys, indexing="ij")
    return np.stack([gx.ravel(), gy.ravel()], axis=-1).astype(np.float32)


def lattice_3d(nx: int, ny: int, nz: int, spacing: float = 0.5,
               x0: float = 0.25, y0: float = -9.75, z0: float = -9.75) -> np.ndarray:
    """[nx*ny*nz, 3] float32 lattice, z fastest."""
    xs = x0 + spacing * np.arange(nx, dtype=np.float64)
    ys = y0 + spacing * np.arange(ny, dtype=np.float64)
    zs = z0 + spacing * np.arange(nz, dtype=np.float64)
    gx, gy, gz = np.meshgrid(xs, ys, zs, indexing="ij")
    return np.stack([gx.ravel(), gy.ravel(), gz.ravel()], axis=-1).astype(np.float32)


def trajectory(base: np.ndarray, nframes: int, seed: int = 0,
               impact_speed: float = 0.02, jitter: float = 0.004) -> np.ndarray:
    """[N, nframes, d] float32 positions.

    Impact-like velocity profile v_x = -v0 (1 - x/L) (the bar decelerates
    from its free end towards the wall at x = 0) plus a per-particle random
    walk of std `jitter` per frame.
    """
    rng = np.random.default_rng(seed)
    base = base.astype(np.float64)
    n, d = base.shape
    length = max(float(base[:, 0].max()), 1e-6)
    v = np.zeros((n, d))
    v[:, 0] = -impact_speed * (1.0 - base[:, 0] / length)
    frames = np.empty((n, nframes, d))
    p = base.copy()
    for t in range(nframes):
        frames[:, t] = p
        v = v + rng.normal(0.0, jitter, size=(n, d)) * 0.25
        p = p + v + rng.normal(0.0, jitter, size=(n, d))
    return frames.astype(np.float32)


def normalization_stats(dim: int, noise_std: float = 0.0, identity: bool = False) -> dict:
    """Normalisation stats in the reference's layout (train.py:446-457):
    std = sqrt(std_meta**2 + noise_std**2).  Returned as float32 numpy."""
    if identity:
        acc_mean, acc_std = np.zeros(dim), np.ones(dim)
        vel_mean, vel_std = np.zeros(dim), np.ones(dim)
    else:
        acc_mean = np.array([1.0e-4, -2.0e-4, 5.0e-5][:dim])
        acc_std = np.array([3.0e-3, 4.0e-3, 3.5e-3][:dim])
        vel_mean = np.array([-1.0e-3, 2.0e-3, 1.0e-3][:dim])
        vel_std = np.array([2.0e-2, 3.0e-2, 2.5e-2][:dim])
    f = lambda a, s: np.sqrt(np.asarray(s, np.float32) ** 2 + np.float32(noise_std) ** 2).astype(np.float32)
    return {
        "acceleration": {"mean": np.asarray(acc_mean, np.float32), "std": f(acc_mean, acc_std)},
        "velocity": {"mean": np.asarray(vel_mean, np.float32), "std": f(vel_mean, vel_std)},
    }
