"""Would a per-quarter slab bound (the 16 points' PCA normal n and the range
[lo, hi] of n.t) cull quarters the AABB keeps?  (CPU study.)

    python tools/slab_study.py [--starts 4] [--passes 2,10,30,100]

For a few C2 starts at the oracle's pose after k ICP iterations, per
128-query wave (source Morton order): the quarters (16 Morton-consecutive
targets) that some query of the wave must scan because its lower bound is
below that query's exact nearest distance -- with the AABB bound alone, and
with max(AABB bound, slab bound).  The ratio is what a slab test would save
of the scanned pairs (an upper bound: the scan's running bound is looser).
"""
import json
import os
import sys

import numpy as np
from scipy.spatial import cKDTree

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO, os.path.join(REPO, "oracle"),
                os.path.join(REPO, "tools")]
import oracle as O  # noqa: E402
from orpcd_amd import Preprocessor  # noqa: E402
from wave_bound_study import boxes, morton_codes  # noqa: E402
from workloads import c2_pair, rot_xyz  # noqa: E402


def slabs(t, n):
    m = len(t) // n
    g = t[: m * n].reshape(m, n, 3)
    c = g - g.mean(1, keepdims=True)
    cov = np.einsum("mki,mkj->mij", c, c)
    w, v = np.linalg.eigh(cov)
    nrm = v[:, :, 0]  # smallest eigenvalue's vector
    d = np.einsum("mkj,mj->mk", g, nrm)
    return nrm, d.min(1), d.max(1)


def main():
    arg = lambda k, d: sys.argv[sys.argv.index(k) + 1] if k in sys.argv else d  # noqa: E731
    B = int(arg("--starts", 4))
    passes = [int(x) for x in arg("--passes", "2,10,30,100").split(",")]
    s, t = c2_pair(50000)
    s = Preprocessor([]).preprocess(s)
    t = Preprocessor([]).preprocess(t)
    lo, hi = t.min(0) - 1, t.max(0) + 1
    t = t[np.argsort(morton_codes(t, lo, hi), kind="stable")]
    m = len(t) // 16 * 16
    t16 = t[:m]
    qlo, qhi = boxes(t16, 16)
    nrm, dlo, dhi = slabs(t16, 16)
    s = s[np.argsort(morton_codes(s, s.min(0), s.max(0)), kind="stable")]
    tree = cKDTree(t)
    rng = np.random.default_rng(1000)
    R0 = np.array([rot_xyz(*rng.uniform(-90, 90, 3)) for _ in range(B)])
    t0 = rng.normal(size=(B, 3)) * 0.1
    for k in passes:
        tot_a = tot_s = 0
        for b in range(B):
            P = s @ R0[b] + t0[b]
            T = O.gicp(P, t, max_iteration=k)["T"]
            q = P @ T[:3, :3].T + T[:3, 3]
            d, _ = tree.query(q, k=1, workers=8)
            d2 = np.minimum(d, 0.5) ** 2
            n = len(q) // 128 * 128
            for w in range(0, n, 128):
                qw, dw = q[w:w + 128], d2[w:w + 128]
                W = dw.max()
                blo, bhi = qw.min(0), qw.max(0)
                gap = np.maximum(0, np.maximum(qlo - bhi, blo - qhi))
                cand = np.nonzero((gap * gap).sum(1) < W)[0]
                if not len(cand):
                    continue
                g = np.maximum(0, np.maximum(qlo[cand][None] - qw[:, None], qw[:, None] - qhi[cand][None]))
                ab = (g * g).sum(2)                                  # (128, C) AABB lower bound
                proj = qw @ nrm[cand].T                              # (128, C)
                sl = np.maximum(0, np.maximum(proj - dhi[cand][None], dlo[cand][None] - proj)) ** 2
                need_a = (ab < dw[:, None]).any(0)
                need_s = (np.maximum(ab, sl) < dw[:, None]).any(0)
                tot_a += int(need_a.sum())
                tot_s += int(need_s.sum())
        print(json.dumps({"pass": k, "quarters_aabb": tot_a, "quarters_aabb_slab": tot_s,
                          "ratio": round(tot_s / max(tot_a, 1), 3)}), flush=True)


if __name__ == "__main__":
    main()
