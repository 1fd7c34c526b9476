"""C3 FGR optimize with the lane- vs wave-per-query KNN threshold (knn_lane_min) interleaved:
    python tools/c3_lane_ab.py"""
import os, sys, time
import numpy as np
REPO = os.getcwd()
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO, os.path.join(REPO, "tools")]
from workloads import c3_pair
from bench_fgr import radius_scale
from orpcd_amd import FastGlobalOptimizer
src, tgt = c3_pair(100_000)
src, tgt = radius_scale(src), radius_scale(tgt)
res = {}
for own in (False, True):
    opt = FastGlobalOptimizer(seed=0, target_features_from_source=not own)
    opt.optimize(src, tgt)
    times = {v: [] for v in (262144, 65536)}
    Ts = {}
    for _ in range(6):
        for v in times:
            opt.context.set_option("knn_lane_min", v)
            t0 = time.perf_counter(); T, r = opt.optimize(src, tgt); times[v].append(time.perf_counter() - t0)
            Ts[v] = T
    for v, t in times.items():
        print(f"own={own} knn_lane_min={v}: {1e3*np.median(t):.3f} ms", "T identical" if np.array_equal(Ts[v], Ts[262144]) else "T DIFFERS", flush=True)
