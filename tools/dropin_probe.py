"""Which part of the drop-in path makes its device batches slow (VERDICT r03
weak #6)?  Four ways to run the same 30 C2 starts as one batch, 6 times each,
host wall-clock of the batch call (orpcd stats host_batch_ms):

  a  batched: the original source, poses (R0, t0)
  b  rebased: the source is the posed copy of start 0 (as the drop-in path
     caches the first cloud it is given), poses relative to it
  c  a, with the drop-in's host work between batches (29 x the posed copy
     np.dot + rigid-residual check of every point)
  d  b, with that host work

    python tools/dropin_probe.py
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]


def main():
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor, _native
    from workloads import c2_pair
    s, t = c2_pair(50_000)
    s, t = Preprocessor([]).preprocess(s), Preprocessor([]).preprocess(t)
    opt = GeneralizedICP()
    ctx = opt.context
    al = Aligner(Preprocessor([]), Preprocessor([]), opt, attempts=30)
    np.random.seed(1000)
    R0, t0 = al._draw_block(30)
    R0, t0 = np.array(R0), np.array(t0)
    base = np.dot(s, R0[0]) + t0[0]
    Rr = np.array([R0[0].T @ R for R in R0])            # base @ Rr + tr = s @ R0 + t0
    tr = np.array([t0[k] - t0[0] @ Rr[k] for k in range(30)])
    out = {}

    def host_work():
        for k in range(29):
            x = np.dot(s.copy(), R0[k % 30]) + t0[k % 30]
            _native.rigid_residual(base, x, Rr[k % 30], tr[k % 30])

    for mode in ("a", "b", "c", "d", "a"):
        src, R, tt = (s, R0, t0) if mode in "ac" else (base, Rr, tr)
        ctx.set_target(t, 1e-3)
        ctx.set_source(src)
        ctx.gicp_batch(R, tt)  # warm
        ctx.reset_stats()
        walls = []
        for _ in range(6):
            if mode in "cd":
                host_work()
            w = time.perf_counter()
            r = ctx.gicp_batch(R, tt)
            walls.append(time.perf_counter() - w)
        st = ctx.stats()
        nb = st["host_batches"]
        out[mode] = {"wall_ms": round(float(np.median(walls)) * 1e3, 2),
                     "sync_ms": round(st["host_sync_ms"] / nb, 2), "launch_ms": round(st["host_launch_ms"] / nb, 2),
                     "iters": int(r["iters"].sum())}
        print(mode, out[mode], file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
