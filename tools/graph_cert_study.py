"""How many queries of a GICP pass can be answered from the target's KNN graph
with a proof of exactness?  (Study for a certified local search.)

    python tools/graph_cert_study.py [--points 50000] [--starts 8] [--passes 60]

CPU only (scipy cKDTree + the oracle's gicp_step).  Per pass and start, for
every query q whose previous-pass nearest target j exists: candidates =
N_k(j), the k nearest targets of t_j (t_j itself included); d* = min over
the candidates of |q - t|.  The answer is certified when
    |q - t_j| + d* < r_k(j)        (r_k(j): distance to the k-th of them)
because every target within d* of q is then within r_k(j) of t_j, i.e. a
candidate.  Prints per pass the certified fraction for several k and checks
that every certified answer equals the exact nearest target.
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
from workloads import c2_pair  # noqa: E402


def arg(name, default):
    return type(default)(sys.argv[sys.argv.index(name) + 1]) if name in sys.argv else default


def main():
    points, B, passes = arg("--points", 50000), arg("--starts", 8), arg("--passes", 60)
    ks = (8, 16, 20, 32, 48)
    s, t = c2_pair(points)
    s = Preprocessor([]).preprocess(s)
    t = Preprocessor([]).preprocess(t)
    tree = cKDTree(t)
    kmax = max(ks)
    dk, nb = tree.query(t, k=kmax)  # nb[:, 0] is the point itself (distinct jittered points)
    _, _, scov = O.estimate_normals(s)
    _, _, tcov = O.estimate_normals(t)
    np.random.seed(1000)
    from orpcd_amd.Aligner.Aligner import Aligner
    R0, t0 = [], []
    for _ in range(B):  # the Aligner's own draws (initialize_rotation)
        R, tt = Aligner._initialize_rotation(np.pi / 2, 0.0, 0.1) if hasattr(Aligner, "_initialize_rotation") else (None, None)
        if R is None:
            ang = np.random.uniform(-np.pi / 2, np.pi / 2, 3)
            cx, cy, cz = np.cos(ang)
            sx, sy, sz = np.sin(ang)
            R = (np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]]) @ np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
                 @ np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]]))
            tt = np.random.normal(0.0, 0.1, 3)
        R0.append(R)
        t0.append(tt)
    T = [np.eye(4) for _ in range(B)]
    prevj = [None] * B
    done = [False] * B
    last_rmse = [None] * B
    for p in range(passes):
        tot = 0
        cert = {k: 0 for k in ks}
        nomatch = 0
        for b in range(B):
            if done[b]:
                continue
            P = s @ R0[b] + t0[b]
            q = P @ T[b][:3, :3].T + T[b][:3, 3]
            d, j = tree.query(q)
            inr = d < 0.5
            if prevj[b] is not None:
                pj = prevj[b]
                ok = pj >= 0
                nomatch += int((~ok).sum())
                tot += len(q)
                qi = q[ok]
                cand = nb[pj[ok]]  # (n, kmax)
                dc = np.linalg.norm(t[cand] - qi[:, None, :], axis=2)
                dqj = dc[:, 0]
                for k in ks:
                    dstar = dc[:, :k].min(axis=1)
                    c = dqj + dstar < dk[pj[ok], k - 1] * (1 - 1e-12)
                    # every certified answer must be the exact nearest target
                    arg_ = cand[np.arange(len(cand)), dc[:, :k].argmin(axis=1)]
                    assert np.all(np.abs(dstar[c] - d[ok][c]) <= 1e-12), k
                    cert[k] += int(c.sum())
                    _ = arg_
            prevj[b] = np.where(inr, j, -1)
            src_cur = q
            R = T[b][:3, :3] @ R0[b].T
            sc = np.einsum("ij,njk,lk->nil", R, scov, R)
            corr = np.where(inr, j, -1).astype(np.int32)
            _, _, upd = O.gicp_step(src_cur, sc, t, tcov, corr)
            T[b] = upd @ T[b]
            rm = np.sqrt(np.mean(d[inr] ** 2)) if inr.any() else 0
            if last_rmse[b] is not None and abs(rm - last_rmse[b]) < 1e-6 * max(rm, 1e-30):
                done[b] = True
            last_rmse[b] = rm
        running = sum(not x for x in done)
        row = dict(p=p, running=running, queries=tot, nomatch=round(nomatch / max(tot, 1), 4),
                   **{f"cert_k{k}": round(cert[k] / max(tot, 1), 4) for k in ks})
        print(json.dumps(row), flush=True)
        if running == 0:
            break


if __name__ == "__main__":
    main()
