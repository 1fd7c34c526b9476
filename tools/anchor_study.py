"""How often can a query's nearest target be certified from its previous
nearest target's neighbour list?  (Study for an anchored local search.)

    python tools/anchor_study.py [--points 50000] [--starts 48] [--ks 16,32,64]

Anchor a = the query's nearest target at the previous pass.  Let L_K(a) be
the K nearest targets of a (a included) and R_K(a) the distance from a to its
(K+1)-th nearest target.  If (2 + eps) * |q - a| < R_K(a), every target p
with |q - p| <= (1 + eps/2) |q - a| satisfies |a - p| < R_K(a), so it is in
L_K(a): the exact nearest target of q (and every near-tie of it) is in the
list.  Prints per pass: running starts, the fraction of in-radius queries
certified for each K, and the fraction of 128-query Morton groups in which
every query is certified (such a group needs no culling at all).
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


def morton_order(p):
    lo, hi = p.min(0), p.max(0)
    g = np.clip(((p - lo) / np.maximum(hi - lo, 1e-12) * 1023).astype(np.uint64), 0, 1023)
    code = np.zeros(len(p), np.uint64)
    for bit in range(10):
        for ax in range(3):
            code |= ((g[:, ax] >> np.uint64(bit)) & np.uint64(1)) << np.uint64(3 * bit + ax)
    return np.argsort(code, kind="stable")


def main():
    arg = lambda k, d: sys.argv[sys.argv.index(k) + 1] if k in sys.argv else d  # noqa: E731
    points, B = int(arg("--points", 50000)), int(arg("--starts", 48))
    ks = [int(x) for x in arg("--ks", "16,32,64").split(",")]
    eps = 1e-3
    s, t = c2_pair(points)
    s = Preprocessor([]).preprocess(s)
    t = Preprocessor([]).preprocess(t)
    s = s[morton_order(s)]
    rng = np.random.default_rng(1000)
    R0 = np.array([rot_xyz(*rng.uniform(-90, 90, 3)) for _ in range(B)])
    t0 = rng.normal(size=(B, 3)) * 0.1
    ctx = _native.Context(0)
    ctx.set_target(t)
    ctx.set_source(s)
    full = ctx.gicp_batch(R0, t0)
    iters = full["iters"]
    tree = cKDTree(t)
    kmax = max(ks)
    dT, _ = tree.query(t, k=kmax + 1, workers=16)
    RK = {k: dT[:, k] for k in ks}  # distance to the (K+1)-th nearest, self included
    prev = {}
    tot_cert = {k: 0 for k in ks}
    tot_q = 0
    for k in range(0, 101):
        Ts = np.repeat(np.eye(4)[None], B, axis=0) if k == 0 else ctx.gicp_batch(R0, t0, max_iteration=k)["T"]
        run = [b for b in range(B) if iters[b] >= k]
        cert = {kk: 0 for kk in ks}
        gcert = {kk: 0 for kk in ks}
        ng, nq = 0, 0
        for b in run:
            P = s @ R0[b] + t0[b]
            q = P @ Ts[b][:3, :3].T + Ts[b][:3, 3]
            d1, j1 = tree.query(q, k=1, workers=16)
            if b in prev:
                a = prev[b]
                da = np.linalg.norm(q - t[a], axis=1)
                inr = d1 < 0.5
                nq += int(inr.sum())
                for kk in ks:
                    ok = (2 + eps) * da + 1e-6 < RK[kk][a]
                    cert[kk] += int((ok & inr).sum())
                    okg = ok | ~inr
                    n = len(okg) // 128 * 128
                    gcert[kk] += int(okg[:n].reshape(-1, 128).all(1).sum())
                ng += len(q) // 128
            prev[b] = j1
        tot_q += nq
        for kk in ks:
            tot_cert[kk] += cert[kk]
        row = dict(k=k, running=len(run), **{f"q{kk}": round(cert[kk] / max(nq, 1), 3) for kk in ks},
                   **{f"g{kk}": round(gcert[kk] / max(ng, 1), 3) for kk in ks})
        if k % 5 == 0 or k < 5:
            print(json.dumps(row), flush=True)
    print(json.dumps({"overall_query_fraction": {kk: round(tot_cert[kk] / max(tot_q, 1), 3) for kk in ks},
                      "R_K_median": {kk: float(np.median(RK[kk])) for kk in ks}}))
    ctx.close()


if __name__ == "__main__":
    main()
