"""Synthetic workloads of BASELINE.json's configs (shared by bench.py and tests).

C1  ArmadilloBack_330 -> _0, Preprocessor([RandomDownsampler(5000)]) (+SOR in the
    reference; SOR is out of scope here), np.random.seed(0).
C2  the same scans densified to 50,000 points each: sample
    50,000 indices WITH replacement (default_rng(2)), add isotropic N(0, 5e-5)
    jitter in raw units to break duplicates; Preprocessor([]) -> RadiusScaler.
C3  bumpy unit sphere r = 1 + 0.1 sin(3θ) cos(2φ), default_rng(3); target =
    index-aligned source·diag(1.1, 0.95, 1.0)·R(20°) + t + N(0, 1e-4).
C5  same surface family, default_rng(5), target = R(10°) x + t + N(0, 1e-4).

The Armadillo scans come from tests/golden/armadillo.npz (parsed from the
reference's sample PLYs by tests/golden/make_golden.py), so nothing here
reads /root/reference at run time.
"""
from __future__ import annotations

import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ARMADILLO = os.path.join(HERE, "tests", "golden", "armadillo.npz")


def armadillo():
    z = np.load(ARMADILLO)
    return z["ArmadilloBack_330"].astype(np.float64), z["ArmadilloBack_0"].astype(np.float64)


def densify(cloud: np.ndarray, n: int, rng: np.random.Generator, sigma: float = 5e-5) -> np.ndarray:
    idx = rng.integers(0, len(cloud), size=n)
    return cloud[idx] + rng.normal(0.0, sigma, size=(n, 3))


def c2_pair(n: int = 50_000):
    src, tgt = armadillo()
    rng = np.random.default_rng(2)
    return densify(src, n, rng), densify(tgt, n, rng)


def rot_xyz(deg_x: float, deg_y: float, deg_z: float) -> np.ndarray:
    ax, ay, az = np.radians([deg_x, deg_y, deg_z])
    Rx = np.array([[1, 0, 0], [0, np.cos(ax), -np.sin(ax)], [0, np.sin(ax), np.cos(ax)]])
    Ry = np.array([[np.cos(ay), 0, np.sin(ay)], [0, 1, 0], [-np.sin(ay), 0, np.cos(ay)]])
    Rz = np.array([[np.cos(az), -np.sin(az), 0], [np.sin(az), np.cos(az), 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def bumpy_sphere(n: int, rng: np.random.Generator) -> np.ndarray:
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    th = np.arccos(np.clip(u[:, 2], -1, 1))
    ph = np.arctan2(u[:, 1], u[:, 0])
    r = 1.0 + 0.1 * np.sin(3 * th) * np.cos(2 * ph)
    return u * r[:, None]


def c3_pair(n: int = 100_000):
    rng = np.random.default_rng(3)
    src = bumpy_sphere(n, rng)
    R = rot_xyz(0, 0, 20)
    tgt = (src * np.array([1.1, 0.95, 1.0])) @ R.T + np.array([0.05, -0.03, 0.02])
    return src, tgt + rng.normal(0, 1e-4, size=tgt.shape)


def c5_pair(n: int = 1_000_000):
    rng = np.random.default_rng(5)
    src = bumpy_sphere(n, rng)
    R = rot_xyz(0, 0, 10)
    tgt = src @ R.T + 0.02
    return src, tgt + rng.normal(0, 1e-4, size=tgt.shape)


def small_pair(n: int = 2000, m: int = None, seed: int = 0, deg=(8.0, -5.0, 6.0), t=(0.03, -0.02, 0.01),
               noise: float = 1e-3):
    """A generic asymmetric surface pair in radius-normalised units."""
    rng = np.random.default_rng(seed)
    m = n if m is None else m
    src = bumpy_sphere(n, rng) * np.array([1.0, 0.8, 0.6])
    base = bumpy_sphere(m, rng) * np.array([1.0, 0.8, 0.6])
    R = rot_xyz(*deg)
    tgt = base @ R.T + np.array(t) + rng.normal(0, noise, size=(m, 3))
    return src, tgt
