"""Where a drop-in multistart's time goes (C2, 30 attempts, the reference-shaped
sequential Aligner over GeneralizedICP.optimize): per multistart, the caller's
loop, the speculative batch, the unspeculated single-start runs, and serving.
    python tools/dropin_breakdown.py [--reps 3]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]
from orpcd_amd import Aligner, GeneralizedICP, Preprocessor, _native  # noqa: E402
from workloads import c2_pair  # noqa: E402


class OnlyOptimize:
    def __init__(self, inner):
        self.inner = inner

    def optimize(self, source, target, **kw):
        return self.inner.optimize(source, target, **kw)


def main():
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 3
    s, t = c2_pair(50_000)
    s, t = Preprocessor([]).preprocess(s), Preprocessor([]).preprocess(t)
    g = GeneralizedICP()
    calls = []  # (starts, seconds, iterations) of every device batch
    orig = _native.Context.gicp_batch

    def timed(self, R0, t0, **kw):
        t_0 = time.perf_counter()
        r = orig(self, R0, t0, **kw)
        calls.append((len(R0), time.perf_counter() - t_0, int(np.sum(r["iters"])), int(np.max(r["iters"]))))
        return r

    _native.Context.gicp_batch = timed
    al = Aligner(Preprocessor([]), Preprocessor([]), OnlyOptimize(g), attempts=30)
    np.random.seed(999)
    al.multistart_registration(s, t)
    np.random.seed(1000)
    for k in range(reps):
        calls.clear()
        t_0 = time.perf_counter()
        al.multistart_registration(s, t)
        el = time.perf_counter() - t_0
        dev = sum(c[1] for c in calls)
        print(f"multistart {k}: {1e3 * el:.1f} ms; device batches {[(c[0], round(1e3 * c[1], 2), c[2], c[3]) for c in calls]} "
              f"(starts, ms, iterations, max iterations) = {1e3 * dev:.1f} ms", flush=True)
    # the same 30 attempts as one batched multistart, for the per-start cost
    np.random.seed(1000)
    alb = Aligner(Preprocessor([]), Preprocessor([]), g, attempts=30)
    for k in range(reps):
        calls.clear()
        t_0 = time.perf_counter()
        alb.multistart_registration(s, t)
        print(f"batched {k}: {1e3 * (time.perf_counter() - t_0):.1f} ms; "
              f"{[(c[0], round(1e3 * c[1], 2), c[2], c[3]) for c in calls]}", flush=True)


if __name__ == "__main__":
    main()
