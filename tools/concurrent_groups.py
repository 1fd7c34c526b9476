"""One C2 multistart (30 starts) split over G device contexts that run concurrently
(one host thread per context, each context on its own HIP stream), against the same
30 starts as one batch on one context.  Per-start results are compared bit for bit.

    python tools/concurrent_groups.py [--groups 1,2,3] [--reps 5] [--split interleave|block]
"""
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]
from orpcd_amd import Preprocessor, _native  # noqa: E402
from workloads import c2_pair, rot_xyz  # noqa: E402


def arg(name, default):
    return sys.argv[sys.argv.index(name) + 1] if name in sys.argv else default


def main():
    groups = [int(g) for g in arg("--groups", "1,2,3").split(",")]
    reps = int(arg("--reps", "5"))
    split = arg("--split", "interleave")
    starts = int(arg("--starts", "30"))
    s, t = c2_pair(50000)
    s = Preprocessor([]).preprocess(s)
    t = Preprocessor([]).preprocess(t)
    rng = np.random.default_rng(1000)
    R0 = np.array([rot_xyz(*rng.uniform(-90, 90, 3)) for _ in range(30)])
    t0 = rng.normal(size=(30, 3)) * 0.1
    R0, t0 = np.resize(R0, (starts, 3, 3)), np.resize(t0, (starts, 3))
    ctxs = []
    for _ in range(max(groups)):
        c = _native.Context(0)
        c.set_target(t)
        c.set_source(s)
        ctxs.append(c)
    ref = ctxs[0].gicp_batch(R0, t0)
    for G in groups:
        if split == "interleave":
            parts = [np.arange(g, starts, G) for g in range(G)]
        else:
            parts = np.array_split(np.arange(starts), G)
        out = [None] * G

        def run(g):
            out[g] = ctxs[g].gicp_batch(R0[parts[g]], t0[parts[g]])

        times = []
        for _ in range(reps + 1):
            th = [threading.Thread(target=run, args=(g,)) for g in range(G)]
            t_0 = time.perf_counter()
            for x in th:
                x.start()
            for x in th:
                x.join()
            times.append(time.perf_counter() - t_0)
        same = True
        for g in range(G):
            for k in ("T", "rmse", "iters"):
                same &= np.array_equal(np.asarray(out[g][k]), np.asarray(ref[k])[parts[g]])
        it = int(sum(int(o["iters"].sum()) for o in out))
        best, med = min(times[1:]), float(np.median(times[1:]))
        print(f"G={G} split={split}: median {1e3 * med:.2f} ms best {1e3 * best:.2f} ms, "
              f"{it / med:.0f} iters/s, identical to one batch: {same}", flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
