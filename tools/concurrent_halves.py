"""Would two halves of a C2 multistart overlap on one GPU?  Runs the 30 (or
--starts) starts of tools/one_batch.py as one batch on one context, then as
two halves on two contexts driven from two host threads at once (separate
HIP streams), and reports the wall-clock of each and whether every start's
result is the same (it must be: a start's answer does not depend on its
batch).  A measurement of the idea "hide one half's per-pass floor kernels
behind the other half's search", not a product path.
    python tools/concurrent_halves.py [--starts 30] [--reps 5]"""
import argparse
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]
from orpcd_amd import Preprocessor, _native  # noqa: E402
from workloads import c2_pair, rot_xyz  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--starts", type=int, default=30)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    s, t = c2_pair(50000)
    s = Preprocessor([]).preprocess(s)
    t = Preprocessor([]).preprocess(t)
    rng = np.random.default_rng(1000)
    R0 = np.array([rot_xyz(*rng.uniform(-90, 90, 3)) for _ in range(a.starts)])
    t0 = rng.normal(size=(a.starts, 3)) * 0.1
    one = _native.Context(0)
    two = [_native.Context(0), _native.Context(0)]
    for c in [one] + two:
        c.set_target(t)
        c.set_source(s)
    h = a.starts // 2
    halves = [(R0[:h], t0[:h]), (R0[h:], t0[h:])]
    for c in two:  # the half batches run the uniform dispatch below sched_min_starts: keep the ordered one
        c.set_option("sched_min_starts", 1)
    res_one, res_two = None, [None, None]
    w1, w2 = [], []
    for rep in range(a.reps + 1):
        t_0 = time.perf_counter()
        res_one = one.gicp_batch(R0, t0)
        w1.append(time.perf_counter() - t_0)

        def run(k):
            res_two[k] = two[k].gicp_batch(*halves[k])
        th = [threading.Thread(target=run, args=(k,)) for k in range(2)]
        t_0 = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        w2.append(time.perf_counter() - t_0)
    same = all(np.array_equal(res_one[k], np.concatenate([res_two[0][k], res_two[1][k]]))
               for k in ("T", "rmse", "iters"))
    seq = []
    for rep in range(a.reps):
        t_0 = time.perf_counter()
        two[0].gicp_batch(*halves[0])
        two[1].gicp_batch(*halves[1])
        seq.append(time.perf_counter() - t_0)
    print(f"one batch of {a.starts}: {1e3 * np.median(w1[1:]):.2f} ms; two halves concurrently: "
          f"{1e3 * np.median(w2[1:]):.2f} ms; two halves one after the other: {1e3 * np.median(seq):.2f} ms; "
          f"results identical: {same}", flush=True)


if __name__ == "__main__":
    main()
