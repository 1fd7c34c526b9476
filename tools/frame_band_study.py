"""CPU study: how wide is exact mode's near-tie band, and how wide would it
be with the scan in tile-local fp32 frames?  

The fp32 search's distance differs from the oracle's fp64 one by at most
delta = u (2A + 3.5 d), A = |q32| the query's magnitude in the target's fp32
frame (the bbox centre): the coordinate roundings dominate.  With every tile's
points stored relative to the tile's centre and the query re-centred on it
(q' = (q32 - c) + qlo, qlo the fp64 residual of q32), A becomes the tile's
radius.  This script builds the C2 target's Morton tiles as the library does,
reports the tile radii, and for the 30 bench starts at their initial poses
counts the queries whose second-nearest target lies within the band of the
nearest (those are the queries exact mode re-searches in fp64), for the
current band and for the tile-frame band.
    python tools/frame_band_study.py
"""
import os
import sys

import numpy as np
from scipy.spatial import cKDTree

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]
U = 2.0 ** -24


def morton_tiles(xyz):
    lo = xyz.min(0)
    ext = (xyz.max(0) - lo).max()
    q = np.clip(((xyz - lo) * (1023.0 / ext)).astype(np.int64), 0, 1023)

    def spread(v):
        v = v & 0x3FF
        v = (v | (v << 16)) & 0x030000FF
        v = (v | (v << 8)) & 0x0300F00F
        v = (v | (v << 4)) & 0x030C30C3
        v = (v | (v << 2)) & 0x09249249
        return v

    code = (spread(q[:, 0]) << 2) | (spread(q[:, 1]) << 1) | spread(q[:, 2])
    order = np.argsort(code, kind="stable")
    return order


def band_rel(d, A):
    """exact_band_hi(d^2) / d^2 - 1 for the given A (gicp_kernels.hip)."""
    delta2 = U * (4.04 * A + 7.07 * d)
    return ((d * np.sqrt(1.0000080) + delta2) ** 2 * 1.0000020) / d ** 2 - 1.0


def main():
    from orpcd_amd import Preprocessor
    from orpcd_amd.Aligner.Aligner import draw_block
    from workloads import c2_pair
    s, t = c2_pair(50_000)
    s, t = Preprocessor([]).preprocess(s), Preprocessor([]).preprocess(t)
    order = morton_tiles(t)
    tm = t[order]
    ntiles = (len(tm) + 63) // 64
    org = 0.5 * (t.min(0) + t.max(0))
    rad = np.zeros(ntiles)
    tile_of = np.empty(len(tm), dtype=np.int64)
    for k in range(ntiles):
        p = tm[64 * k:64 * (k + 1)]
        c = 0.5 * (p.min(0) + p.max(0))
        rad[k] = np.linalg.norm(p - c, axis=1).max()
        tile_of[64 * k:64 * (k + 1)] = k
    print(f"tiles {ntiles}: radius median {np.median(rad):.4g}, p99 {np.percentile(rad, 99):.4g}, "
          f"max {rad.max():.4g}; target |x - org| max {np.linalg.norm(t - org, axis=1).max():.4g}")
    tree = cKDTree(tm)
    np.random.seed(1000)
    R0, t0 = draw_block(30, np.pi / 2, 0.0, 0.1)
    tot = cur = new_max = new_tile = 0
    for R, tt in zip(R0, t0):
        q = np.dot(s, R) + tt
        d, j = tree.query(q, k=2)
        d1, d2 = d[:, 0], d[:, 1]
        A = np.linalg.norm(q - org, axis=1)
        gap = d2 ** 2 / np.maximum(d1 ** 2, 1e-300) - 1.0
        tot += len(q)
        cur += int(np.sum(gap <= band_rel(d1, A)))
        new_max += int(np.sum(gap <= band_rel(d1, rad.max())))
        # per-tile radii: the winner's and the runner-up's tiles
        rt = np.maximum(rad[tile_of[j[:, 0]]], rad[tile_of[j[:, 1]]])
        new_tile += int(np.sum(gap <= band_rel(d1, rt)))
    print(f"queries {tot}: near-tie (filed) fraction, current band (A = |q32|) {cur / tot:.5f}, "
          f"tile frames with the global max radius {new_max / tot:.5f}, with per-tile radii {new_tile / tot:.5f}")


if __name__ == "__main__":
    main()
