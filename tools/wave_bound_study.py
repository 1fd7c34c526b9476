"""Culling work of a 128-query search wave under two query orders (CPU study).

    python tools/wave_bound_study.py [--points 50000] [--starts 8] [--passes 2,10,30,100]

For a few C2 starts, the oracle's pose after k ICP iterations gives the
queries of pass k; the bound of a query is its exact nearest distance (x1.05,
about what the previous nearest target gives) or r^2 when nothing lies within
r.  Waves of 128 queries are formed
  (A) in source Morton order (the search's order today), or
  (B) after a stable partition of each start's queries by bound class
      (log2 buckets of the bound), Morton order within a class.
Per wave: W = worst bound; counts of super-tiles (4096 targets) and tiles (64
targets, Morton-sorted target) whose box lies within W of the wave's query
box, and of tiles within some query's own bound of that query ("candidates").
"""
import json
import os
import sys

import numpy as np
from scipy.spatial import cKDTree

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO, os.path.join(REPO, "oracle")]
import oracle as O  # noqa: E402
from orpcd_amd import Preprocessor  # noqa: E402
from workloads import c2_pair, rot_xyz  # noqa: E402


def morton_codes(p, lo, hi):
    g = np.clip(((p - lo) / np.maximum(hi - lo, 1e-12) * 1023).astype(np.uint64), 0, 1023)
    code = np.zeros(len(p), np.uint64)
    for bit in range(10):
        for ax in range(3):
            code |= ((g[:, ax] >> np.uint64(bit)) & np.uint64(1)) << np.uint64(3 * bit + ax)
    return code


def boxes(p, n):
    m = (len(p) + n - 1) // n
    pad = np.concatenate([p, np.repeat(p[-1:], m * n - len(p), 0)])
    b = pad.reshape(m, n, 3)
    return b.min(1), b.max(1)


def box_d2(qlo, qhi, lo, hi):
    d = np.maximum(0, np.maximum(lo[None] - qhi[:, None], qlo[:, None] - hi[None]))
    return (d * d).sum(-1)


def wave_stats(q, bound, order, tlo, thi, slo, shi):
    qs, bs = q[order], bound[order]
    n = len(qs) // 128 * 128
    qs, bs = qs[:n].reshape(-1, 128, 3), bs[:n].reshape(-1, 128)
    W = bs.max(1)
    qlo, qhi = qs.min(1), qs.max(1)
    sup = (box_d2(qlo, qhi, slo, shi) < W[:, None]).sum()
    tw = box_d2(qlo, qhi, tlo, thi) < W[:, None]
    cand = 0
    for w in range(len(qs)):
        idx = np.nonzero(tw[w])[0]
        if len(idx):
            d = box_d2(qs[w], qs[w], tlo[idx], thi[idx])  # per query vs tile box
            cand += int((d < bs[w][:, None]).any(0).sum())
    return dict(waves=len(qs), super_per_wave=sup / len(qs), tiles_per_wave=tw.sum() / len(qs),
                cand_per_wave=cand / len(qs), W_median=float(np.median(W)))


def main():
    arg = lambda k, d: sys.argv[sys.argv.index(k) + 1] if k in sys.argv else d  # noqa: E731
    points, B = int(arg("--points", 50000)), int(arg("--starts", 8))
    passes = [int(x) for x in arg("--passes", "2,10,30,100").split(",")]
    s, t = c2_pair(points)
    s = Preprocessor([]).preprocess(s)
    t = Preprocessor([]).preprocess(t)
    lo, hi = t.min(0) - 1, t.max(0) + 1
    t = t[np.argsort(morton_codes(t, lo, hi), kind="stable")]
    tlo, thi = boxes(t, 64)
    slo, shi = boxes(t, 4096)
    s = s[np.argsort(morton_codes(s, s.min(0), s.max(0)), kind="stable")]
    tree = cKDTree(t)
    rng = np.random.default_rng(1000)
    R0 = np.array([rot_xyz(*rng.uniform(-90, 90, 3)) for _ in range(B)])
    t0 = rng.normal(size=(B, 3)) * 0.1
    for k in passes:
        acc = {"A": [], "B": []}
        for b in range(B):
            P = s @ R0[b] + t0[b]
            T = O.gicp(P, t, max_iteration=k)["T"]
            q = P @ T[:3, :3].T + T[:3, 3]
            d, _ = tree.query(q, k=1, workers=8)
            bound = np.where(d < 0.5, np.minimum((d * 1.05) ** 2, 0.25), 0.25)
            qlo_all, qhi_all = q.min(0), q.max(0)
            mort = np.argsort(morton_codes(q, qlo_all, qhi_all), kind="stable")  # q order == source Morton order
            order_a = np.arange(len(q))  # the source's Morton order
            cls = np.floor(np.log2(bound)).astype(int)
            order_b = np.lexsort((np.arange(len(q)), cls))
            del mort
            acc["A"].append(wave_stats(q, bound, order_a, tlo, thi, slo, shi))
            acc["B"].append(wave_stats(q, bound, order_b, tlo, thi, slo, shi))
        out = {"pass": k}
        for key, rows in acc.items():
            out[key] = {f: round(float(np.mean([r[f] for r in rows])), 4) for f in rows[0]}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
