"""The zero-code-change drop-in path at C2: the reference-shaped sequential
multistart (one GeneralizedICP.optimize per attempt, Aligner.py:178-202, as
the reference's own Aligner calls the plugin) against the batched multistart
(optimize_batch, one device batch of 30 starts).

    python tools/bench_dropin.py [--reps 3] [--out profiles/r03_dropin.json]

Three legs, same seeds (np.random.seed(1000 + k)), 30 attempts each:
  batched      Aligner -> GeneralizedICP.optimize_batch
  dropin       Aligner over a plugin exposing only optimize(): every call
               hands over source @ R0 + t0; the plugin recognises the rigid
               image of its cached cloud (GeneralizedICP._rigid_image) and runs
               the start on the cached layout / covariances
  dropin_cold  the same with rigid_cache=False: every posed copy uploaded,
               laid out and its KNN-20 covariances recomputed, as Open3D does
Per-start results of the drop-in legs are compared with the batched table.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]


class OnlyOptimize:
    """An IOptimizer with nothing but optimize(): the Aligner takes its
    sequential path (Aligner.py:178-202), exactly the reference's calls."""

    def __init__(self, inner):
        self.inner = inner
        self.rmse = []

    def optimize(self, source, target, **kw):
        T, m = self.inner.optimize(source, target, **kw)
        self.rmse.append(m)
        return T, m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--attempts", type=int, default=30)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor
    from workloads import c2_pair
    s, t = c2_pair(50_000)
    s, t = Preprocessor([]).preprocess(s), Preprocessor([]).preprocess(t)

    def leg(opt, name):
        al = Aligner(Preprocessor([]), Preprocessor([]), opt, attempts=a.attempts)
        np.random.seed(999)
        al.multistart_registration(s, t)  # warm-up
        times, rmse = [], []
        for k in range(a.reps):
            if isinstance(opt, OnlyOptimize):
                opt.rmse = []
            np.random.seed(1000 + k)
            t0 = time.perf_counter()
            al.multistart_registration(s, t)
            times.append(time.perf_counter() - t0)
            rmse.append(np.array(opt.rmse) if isinstance(opt, OnlyOptimize) else al.history[-1]["rmse"])
        print(f"{name}: {np.median(times) * 1e3:.1f} ms per multistart", file=sys.stderr, flush=True)
        return float(np.median(times)), rmse

    tb, rb = leg(GeneralizedICP(), "batched")
    td, rd = leg(OnlyOptimize(GeneralizedICP()), "dropin")
    tc, rc = leg(OnlyOptimize(GeneralizedICP(rigid_cache=False)), "dropin_cold")
    d_warm = max(float(np.abs(x - y).max()) for x, y in zip(rd, rb))
    d_cold = max(float(np.abs(x - y).max()) for x, y in zip(rc, rb))
    res = {"metric": "multistart wall-clock at C2 (30 starts), drop-in sequential vs batched", "unit": "ms",
           "batched_ms": round(tb * 1e3, 2), "dropin_ms": round(td * 1e3, 2), "dropin_cold_ms": round(tc * 1e3, 2),
           "dropin_over_batched": round(td / tb, 2), "dropin_cold_over_batched": round(tc / tb, 2),
           "max_abs_d_rmse_vs_batched": {"dropin": d_warm, "dropin_cold": d_cold},
           "reps": a.reps, "attempts": a.attempts}
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
