"""Median set_target / set_source time at C5 (1M points), for KNN A/B builds:
    ORPCD_HIP_LIB=... python tools/knn_time.py [--reps 9]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]
import numpy as np  # noqa: E402
from orpcd_amd import _native  # noqa: E402
from workloads import c5_pair  # noqa: E402

reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 9
src, tgt = c5_pair()
ctx = _native.Context(0)
tt, ts = [], []
for _ in range(reps):
    t0 = time.perf_counter()
    ctx.set_target(tgt, 1e-3, cache=False)
    tt.append(time.perf_counter() - t0)
    t0 = time.perf_counter()
    ctx.set_source(src, cache=False)
    ts.append(time.perf_counter() - t0)
print(f"{os.environ.get('ORPCD_HIP_LIB', 'head')}: set_target {1e3 * np.median(tt[1:]):.3f} ms, "
      f"set_source {1e3 * np.median(ts[1:]):.3f} ms")
