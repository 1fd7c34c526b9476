"""Set-up time (set_target / set_source) of the wave- and lane-per-query KNN at several cloud sizes:
    python tools/knn_sizes.py"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]
from orpcd_amd import _native, Preprocessor
from workloads import c2_pair, bumpy_sphere
ctx = _native.Context(0)
for n in (50_000, 100_000, 200_000, 400_000):
    if n == 50_000:
        s, t = c2_pair(n); s = Preprocessor([]).preprocess(s); t = Preprocessor([]).preprocess(t)
    else:
        rng = np.random.default_rng(n); t = bumpy_sphere(n, rng); s = bumpy_sphere(n, rng)
    for lm in (0, 1):
        ctx.set_option("knn_lane_min", lm)
        tt, ts = [], []
        for _ in range(7):
            t0 = time.perf_counter(); ctx.set_target(t, 1e-3, cache=False); tt.append(time.perf_counter() - t0)
            t0 = time.perf_counter(); ctx.set_source(s, cache=False); ts.append(time.perf_counter() - t0)
        print(f"n={n} {'lane' if lm else 'wave'}: set_target {1e3*np.median(tt[1:]):.3f} ms set_source {1e3*np.median(ts[1:]):.3f} ms", flush=True)
