"""A/B of the feature nearest-neighbour search (C3) between library builds.

    ORPCD_HIP_LIB=abl/x.so python tools/fgr_ab.py --tag x [--reps 5]

Runs in the library named by ORPCD_HIP_LIB (or the in-tree one): the C3
source features against themselves (the Q4 pairing FGR uses by default:
a third of the queries hold near-duplicate rows, so the exact pass works), the
source against the target cloud's own features (compat_q4 off), and one
FastGlobalOptimizer.optimize.  Prints the median wall time of each and a
hash of every answer, so builds can be checked for identical results.
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]


def _h(a):
    return hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()[:12]


def _time(fn, reps):
    out, ts = None, []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return out, 1e3 * float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="head")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--points", type=int, default=100_000)
    args = ap.parse_args()
    from workloads import c3_pair
    from orpcd_amd import FastGlobalOptimizer
    from bench_fgr import radius_scale
    src, tgt = c3_pair(args.points)
    src, tgt = radius_scale(src), radius_scale(tgt)
    opt = FastGlobalOptimizer(seed=0)
    opt.optimize(src, tgt)  # warm-up
    ctx = opt.context
    _, fs = ctx.fpfh(src, 0.1, 20, 0.1, 20)
    _, ft = ctx.fpfh(tgt, 0.1, 20, 0.1, 20)
    ctx.feature_nn(fs[:4096], fs)
    line = {"tag": args.tag, "lib": os.environ.get("ORPCD_HIP_LIB", "in-tree")}
    i_ss, line["self_ms"] = _time(lambda: ctx.feature_nn(fs, fs), args.reps)
    i_st, line["cross_ms"] = _time(lambda: ctx.feature_nn(fs, ft), args.reps)
    (T, rmse), line["optimize_ms"] = _time(lambda: opt.optimize(src, tgt), args.reps)
    line["hash"] = {"self": _h(i_ss), "cross": _h(i_st), "T": _h(T), "rmse": repr(float(rmse))}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    sys.path.insert(0, os.path.join(REPO, "tools"))
    main()
