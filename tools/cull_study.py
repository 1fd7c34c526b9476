"""Culling study on the C2 pair (CPU, numpy/scipy): how many 64-target tiles a
128-query Morton group must scan when every query's bound is already its
exact nearest distance (the ideal seed), with the tile test as built (AABB)
and with oriented boxes (PCA frame per tile), and how much of it is owed to
queries with no target within the radius.

    python tools/cull_study.py [--starts 6] [--converged]

--converged poses the source by the start's result instead of its initial
pose (tail passes).  Prints tiles per group and per query.
"""
import os
import sys

import numpy as np
from scipy.spatial import cKDTree

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
from workloads import c2_pair, rot_xyz  # noqa: E402


def normalise(x):
    c = x.mean(0)
    return (x - c) / np.linalg.norm(x - c, axis=1).max()


def morton_order(x):
    lo, hi = x.min(0), x.max(0)
    q = np.clip(((x - lo) / (hi - lo).max() * 1023).astype(np.uint64), 0, 1023)

    def spread(v):
        v = (v | (v << np.uint64(16))) & np.uint64(0x030000FF)
        v = (v | (v << np.uint64(8))) & np.uint64(0x0300F00F)
        v = (v | (v << np.uint64(4))) & np.uint64(0x030C30C3)
        v = (v | (v << np.uint64(2))) & np.uint64(0x09249249)
        return v

    code = spread(q[:, 0]) | (spread(q[:, 1]) << np.uint64(1)) | (spread(q[:, 2]) << np.uint64(2))
    return np.argsort(code, kind="stable")


def tiles_of(t, size=64):
    n = (len(t) + size - 1) // size
    lo = np.array([t[i * size:(i + 1) * size].min(0) for i in range(n)])
    hi = np.array([t[i * size:(i + 1) * size].max(0) for i in range(n)])
    frames, olo, ohi, cen = [], [], [], []
    for i in range(n):
        p = t[i * size:(i + 1) * size]
        c = p.mean(0)
        _, V = np.linalg.eigh(np.cov((p - c).T) if len(p) > 1 else np.eye(3))
        loc = (p - c) @ V
        frames.append(V)
        cen.append(c)
        olo.append(loc.min(0))
        ohi.append(loc.max(0))
    return lo, hi, np.array(frames), np.array(cen), np.array(olo), np.array(ohi)


def box_d2(q, lo, hi):  # q (k,3) vs boxes (m,3) -> (k,m)
    d = np.maximum(0, np.maximum(lo[None] - q[:, None], q[:, None] - hi[None]))
    return (d * d).sum(-1)


def main():
    starts = int(sys.argv[sys.argv.index("--starts") + 1]) if "--starts" in sys.argv else 6
    converged = "--converged" in sys.argv
    s, t = c2_pair(50000)
    s, t = normalise(s), normalise(t)
    t = t[morton_order(t)]
    s = s[morton_order(s)]
    tree = cKDTree(t)
    size = int(sys.argv[sys.argv.index("--tile") + 1]) if "--tile" in sys.argv else 64
    lo, hi, V, C, olo, ohi = tiles_of(t, size)
    rng = np.random.default_rng(7)
    r2 = 0.25
    tot = {"aabb": 0, "obb": 0, "slab": 0, "aabb_matched_only": 0, "obb_matched_only": 0, "groups": 0, "nomatch": 0, "q": 0}
    for _ in range(starts):
        R = rot_xyz(*rng.uniform(-90, 90, 3))
        tt = rng.normal(size=3) * 0.1
        if converged:
            R, tt = np.eye(3), np.zeros(3)  # the pair is roughly aligned as given
        q = s @ R + tt
        d, _ = tree.query(q, distance_upper_bound=0.5)
        bound = np.where(np.isfinite(d), d * d, r2)
        matched = np.isfinite(d)
        tot["nomatch"] += int((~matched).sum())
        tot["q"] += len(q)
        for g in range(0, len(q), 128):
            qq, bb, mm = q[g:g + 128], bound[g:g + 128], matched[g:g + 128]
            qlo, qhi = qq.min(0), qq.max(0)
            W = bb.max()
            dd = np.maximum(0, np.maximum(lo - qhi, qlo - hi))
            cand = np.nonzero((dd * dd).sum(1) < W)[0]
            a = box_d2(qq, lo[cand], hi[cand]) < bb[:, None]
            # oriented boxes: query in each candidate tile's PCA frame
            rel = qq[:, None, :] - C[cand][None]  # (k,m,3)
            locq = np.einsum("kmj,mji->kmi", rel, V[cand])
            dl = np.maximum(0, np.maximum(olo[cand][None] - locq, locq - ohi[cand][None]))
            o = (dl * dl).sum(-1) < bb[:, None]
            o &= a  # both bounds hold: use the tighter
            # slab only: AABB distance and the distance to the tile's plane
            # slab (smallest PCA axis, half-thickness from the points)
            h = np.maximum(-olo[cand][:, 0], ohi[cand][:, 0])
            sd = np.maximum(0, np.abs(locq[..., 0]) - h[None])
            sl = a & (sd * sd < bb[:, None])
            tot["slab"] += int(sl.any(0).sum())
            tot["aabb"] += int(a.any(0).sum())
            tot["obb"] += int(o.any(0).sum())
            tot["aabb_matched_only"] += int((a & mm[:, None]).any(0).sum())
            tot["obb_matched_only"] += int((o & mm[:, None]).any(0).sum())
            tot["groups"] += 1
            # wave-level prefilter: tiles / 64-tile super-tiles within W of
            # the box of K query subgroups (K = 1 as built)
            for K in (1, 4, 8):
                ok_t = np.zeros(len(lo), bool)
                for sub in np.array_split(np.arange(len(qq)), K):
                    slo_, shi_ = qq[sub].min(0), qq[sub].max(0)
                    dd = np.maximum(0, np.maximum(lo - shi_, slo_ - hi))
                    ok_t |= (dd * dd).sum(1) < bb[sub].max()
                tot[f"cand_K{K}"] = tot.get(f"cand_K{K}", 0) + int(ok_t.sum())
                sup = np.unique(np.nonzero(ok_t)[0] // 64)
                tot[f"super_K{K}"] = tot.get(f"super_K{K}", 0) + len(sup)
    G = tot["groups"]
    print(f"starts {starts} converged={converged}: no-match queries {tot['nomatch'] / tot['q']:.3f}")
    for k in ("aabb", "obb", "slab", "aabb_matched_only", "obb_matched_only"):
        print(f"  {k:18s} tiles/group {tot[k] / G:7.2f}  targets/group {tot[k] / G * size:8.1f}")
    for K in (1, 4, 8):
        print(f"  K={K} subgroups: tiles passing the wave test {tot[f'cand_K{K}'] / G:7.2f}, "
              f"super-tiles holding one {tot[f'super_K{K}'] / G:5.2f}")


if __name__ == "__main__":
    main()
