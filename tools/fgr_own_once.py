"""One own-features FGR call at C3 after a warm-up (for kernel traces):  python tools/fgr_own_once.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]
import numpy as np  # noqa: E402
from workloads import c3_pair  # noqa: E402
from orpcd_amd import FastGlobalOptimizer  # noqa: E402


def rs(c):
    c0 = c.mean(axis=0, keepdims=True)
    return (c - c0) / np.max(np.linalg.norm(c - c0, axis=1))


s, t = c3_pair(100000)
s, t = rs(s), rs(t)
opt = FastGlobalOptimizer(seed=0, target_features_from_source=False)
for _ in range(3):
    opt.optimize(s, t)
