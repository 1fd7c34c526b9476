"""Where do GPU and oracle GICP part ways at C2 size?  Per pass k the max |dT|
of start 0 (both sides run k passes), and for the pose of pass 0 the
nearest-neighbour mismatches with their relative d^2 gap.

    python tools/diverge_c2.py [--start 0] [--passes 8]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO, os.path.join(REPO, "oracle")]
import oracle  # noqa: E402
from orpcd_amd import Preprocessor, _native  # noqa: E402
from workloads import c2_pair, rot_xyz  # noqa: E402


def main():
    b = int(sys.argv[sys.argv.index("--start") + 1]) if "--start" in sys.argv else 0
    P = int(sys.argv[sys.argv.index("--passes") + 1]) if "--passes" in sys.argv else 8
    s, t = c2_pair(50_000)
    s = Preprocessor([]).preprocess(s)
    t = Preprocessor([]).preprocess(t)
    rng = np.random.default_rng(1000)
    R0 = np.array([rot_xyz(*rng.uniform(-90, 90, 3)) for _ in range(3)])
    t0 = rng.normal(size=(3, 3)) * 0.1
    src = np.dot(s, R0[b]) + t0[b]
    ctx = _native.Context(0)
    gi, gd = ctx.nn1_radius(src, t, 0.5)
    oi, od = oracle.nn1_radius(src, t, 0.5)
    bad = np.nonzero(gi != oi)[0]
    gaps = []
    for i in bad:
        da = ((src[i] - t[oi[i]]) ** 2).sum() if oi[i] >= 0 else np.inf
        db = ((src[i] - t[gi[i]]) ** 2).sum() if gi[i] >= 0 else np.inf
        gaps.append(abs(da - db) / max(da, 1e-300))
    print(f"pass-0 NN mismatches: {len(bad)} of {len(src)}; max relative d^2 gap {max(gaps) if gaps else 0:.2e}")
    ctx.set_target(t)
    ctx.set_source(s)
    for k in range(1, P + 1):
        g = ctx.gicp_batch(R0[b:b + 1], t0[b:b + 1], max_iteration=k)
        o = oracle.gicp(src, t, 0.5, k)
        print(f"passes {k}: max|dT| {np.abs(g['T'][0] - o['T']).max():.3e}  rmse {g['rmse'][0]:.9f} vs "
              f"{o['rmse']:.9f}  ncorr {g['ncorr'][0]} vs {o.get('ncorr')}", flush=True)
    g = ctx.gicp_batch(R0, t0)
    for bb in range(3):
        o = oracle.gicp(np.dot(s, R0[bb]) + t0[bb], t, 0.5, 100)
        print(f"start {bb} converged: iters {g['iters'][bb]} vs {o['iters']}  max|dT| "
              f"{np.abs(g['T'][bb] - o['T']).max():.3e}  rmse {g['rmse'][bb]:.9f} vs {o['rmse']:.9f}", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
