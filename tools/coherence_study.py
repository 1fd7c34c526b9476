"""How often does a query's nearest target stay provably the same from one ICP
pass to the next?  (Study for a temporal-coherence skip of the search.)

    python tools/coherence_study.py [--points 50000] [--starts 30]

Runs the C2 multistart with max_iteration = k for k = 1..100 (the device
result after k passes is the pose the search of pass k uses), then, per pass
and running start, on the host (scipy cKDTree): d1, d2 = distances to the
nearest and second-nearest target, delta = how far the query moved since the
previous pass.  A query is "certified" when 2*delta < (d2 - d1) at the
previous pass (triangle inequality: its nearest target cannot change).
Prints per pass: running starts, fraction certified, median gap and delta.
"""
import json
import os
import sys

import numpy as np
from scipy.spatial import cKDTree

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]
from orpcd_amd import Preprocessor, _native  # noqa: E402
from workloads import c2_pair, rot_xyz  # noqa: E402


def main():
    points = int(sys.argv[sys.argv.index("--points") + 1]) if "--points" in sys.argv else 50000
    B = int(sys.argv[sys.argv.index("--starts") + 1]) if "--starts" in sys.argv else 30
    s, t = c2_pair(points)
    s = Preprocessor([]).preprocess(s)
    t = Preprocessor([]).preprocess(t)
    rng = np.random.default_rng(1000)
    R0 = np.array([rot_xyz(*rng.uniform(-90, 90, 3)) for _ in range(B)])
    t0 = rng.normal(size=(B, 3)) * 0.1
    ctx = _native.Context(0)
    ctx.set_target(t)
    ctx.set_source(s)
    full = ctx.gicp_batch(R0, t0)
    iters = full["iters"]
    tree = cKDTree(t)
    prev = {}
    rows = []
    for k in range(0, 101):
        if k == 0:
            Ts = np.repeat(np.eye(4)[None], B, axis=0)
        else:
            Ts = ctx.gicp_batch(R0, t0, max_iteration=k)["T"]
        run = [b for b in range(B) if iters[b] >= k]
        cert, tot, gaps, dels = 0, 0, [], []
        for b in run:
            P = s @ R0[b] + t0[b]
            q = P @ Ts[b][:3, :3].T + Ts[b][:3, 3]
            d, j = tree.query(q, k=2)
            inr = d[:, 0] < 0.5
            if b in prev:
                q_old, gap_old, in_old = prev[b]
                delta = np.linalg.norm(q - q_old, axis=1)
                ok = in_old & (2 * delta < gap_old)
                cert += int(ok.sum())
                tot += int(in_old.sum())
                dels.append(np.median(delta))
            gaps.append(np.median(d[inr, 1] - d[inr, 0]) if inr.any() else 0.0)
            prev[b] = (q, d[:, 1] - d[:, 0], inr)
        rows.append(dict(k=k, running=len(run), certified=round(cert / max(tot, 1), 4),
                         median_gap=float(np.median(gaps)) if gaps else None,
                         median_delta=float(np.median(dels)) if dels else None))
        if k % 5 == 0 or k < 5:
            print(json.dumps(rows[-1]), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
