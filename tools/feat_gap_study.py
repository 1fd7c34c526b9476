"""CPU study: could the C3 feature search run its first pass in fp32?


Pass 1 of the feature nearest-neighbour search (fgr_kernels.hip) must flag
every query whose best and runner-up target distances lie within the
expansion's rounding bound; pass 2 re-searches the flagged queries in fp64.
An fp32 pass 1 (the matrix cores' f32 rate is twice the f64 rate) would widen
that bound from ~2e-13 x the norms to ~1e-6 x the norms (|f|^2 is 3e4..1.2e5
for FPFH rows, ~1.6e3 after centring).  This script computes the C3 source
features with the oracle, drops exact duplicate rows (as dedup_rows does),
and prints, for a sample of queries, the fraction whose runner-up gap is
below a range of thresholds: the fraction an fp32 pass 1 would send to the
fp64 pass 2.
    python tools/feat_gap_study.py [--sample 3000]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO, os.path.join(REPO, "oracle"),
                os.path.join(REPO, "tools")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sample", type=int, default=3000)
    args = ap.parse_args()
    import oracle
    from bench_fgr import radius_scale
    from workloads import c3_pair
    s, _ = c3_pair(100_000)
    _, fs = oracle.fpfh(radius_scale(s), 0.1, 20, 0.1, 20)
    _, first = np.unique(fs, axis=0, return_index=True)
    T = fs[np.sort(first)]
    n2 = (fs ** 2).sum(1)
    c = T.mean(0)
    print(f"rows {len(fs)}, distinct {len(T)}; |f|^2 {n2.min():.4g}..{n2.max():.4g}, "
          f"centred median {np.median(((T - c) ** 2).sum(1)):.4g}")
    Q = fs[np.random.default_rng(0).choice(len(fs), args.sample, replace=False)]
    gaps = []
    for b in range(0, len(Q), 100):
        d = ((Q[b:b + 100, None, :] - T[None, :, :]) ** 2).sum(2)
        p = np.partition(d, 1, axis=1)
        gaps.append(p[:, 1] - p[:, 0])
    g = np.concatenate(gaps)
    print(f"queries {len(Q)} (the Q4 pairing: every query's own row is a target, best distance 0)")
    for x in [1e-8, 1e-6, 1e-4, 1e-3, 1e-2, 3e-2, 0.1, 0.3, 1.0]:
        print(f"  runner-up gap < {x:g}: {(g < x).mean():.4f}")


if __name__ == "__main__":
    main()
