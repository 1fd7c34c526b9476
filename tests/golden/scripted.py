"""Deterministic scripted IOptimizer used to pin the Aligner control flow.

Its (T, rmse) are pure numpy functions of the arguments the Aligner passes
(`source_initialized`, `target_scaled`), so driving the reference Aligner and
the build's Aligner with it must produce bit-identical call sequences and
results (golden vector G3).  This is build-side test code.
"""
import numpy as np


def _rot_zyx(a):
    cz, sz = np.cos(a[2]), np.sin(a[2])
    cy, sy = np.cos(a[1]), np.sin(a[1])
    cx, sx = np.cos(a[0]), np.sin(a[0])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1.0]])
    Ry = np.array([[cy, 0, sy], [0, 1.0, 0], [-sy, 0, cy]])
    Rx = np.array([[1.0, 0, 0], [0, cx, -sx], [0, sx, cx]])
    return Rz @ Ry @ Rx


class ScriptedOptimizer:
    """rmse = ||mean|target| - goal||^2 + 1e-3 * (1 + sin(7 * mean(source)_x))."""

    def __init__(self, goal, mode="scripted"):
        self.goal = np.asarray(goal, dtype=np.float64)
        self.mode = mode
        self.calls = []

    def optimize(self, source, target, **kwargs):
        a = np.abs(target).mean(axis=0)
        s0 = source.mean(axis=0)
        if self.mode == "never_improves":
            rmse = 1.0 + 1e-3 * len(self.calls)
        elif self.mode == "constant":
            rmse = 0.5
        else:
            rmse = float(((a - self.goal) ** 2).sum() + 1e-3 * (1.0 + np.sin(7.0 * s0[0])))
        T = np.eye(4)
        T[:3, :3] = _rot_zyx(0.5 * s0)
        T[:3, 3] = 0.1 * s0
        self.calls.append((a.copy(), source[0].copy(), rmse))
        return T, rmse
