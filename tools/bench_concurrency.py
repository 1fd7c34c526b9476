"""How well do several multistart batches overlap on one GPU (the speculative
compass)?  Times one C2 multistart batch alone, then k batches (different
target scales, own contexts and streams) through optimize_batch_multi.

    python tools/bench_concurrency.py [--points 50000] [--k 6]
"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=50000)
    ap.add_argument("--k", type=int, default=6)
    ap.add_argument("--waves", type=int, default=32768, help="split target of one batch alone")
    a = ap.parse_args()
    from orpcd_amd import GeneralizedICP, Preprocessor
    from workloads import c2_pair, rot_xyz
    s, t = c2_pair(a.points)
    s = Preprocessor([]).preprocess(s)
    t = Preprocessor([]).preprocess(t)
    rng = np.random.default_rng(1000)
    R0 = np.array([rot_xyz(*rng.uniform(-90, 90, 3)) for _ in range(30)])
    t0 = rng.normal(size=(30, 3)) * 0.1
    opt = GeneralizedICP()
    opt.search_waves = a.waves
    targets = [t * np.array([1.0 + 0.05 * (j % 3 - 1), 1.0, 1.0 + 0.02 * j]) for j in range(a.k)]
    for rep in range(2):  # warm-up round then timed
        t1 = time.perf_counter()
        for tg in targets:
            opt.optimize_batch(s, tg, R0, t0)
        seq = time.perf_counter() - t1
        t1 = time.perf_counter()
        opt.optimize_batch_multi(s, targets, [R0] * a.k, [t0] * a.k)
        par = time.perf_counter() - t1
    print(f"k={a.k}: sequential {seq * 1e3:.1f} ms ({seq / a.k * 1e3:.1f} per batch), concurrent {par * 1e3:.1f} ms, "
          f"overlap gain {seq / par:.2f}x")


if __name__ == "__main__":
    main()
