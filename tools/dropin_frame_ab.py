"""Drop-in slowdown: is it the frame the drop-in runs
its batches in?  The drop-in path caches the FIRST posed copy it sees
(base = source @ Rb + tb) and runs later starts relative to it; the batched
path runs on the unposed source.  The same 30 starts (the Aligner's draws,
np.random.seed(1000)) are run here as one gicp_batch on

  plain   the unposed source s with (R0, t0)
  base    base = s @ Rb + tb (the drop-in's first draw, seed 999) with the
          relative poses base @ (Rb^T R0) + (t0 - tb Rb^T R0)

alternately, `reps` times each, with ORPCD_GAPS-style host timing, and the
results compared start by start.
    python tools/dropin_frame_ab.py [--reps 5]
"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from orpcd_amd import Preprocessor, _native
    from orpcd_amd.Aligner.Aligner import draw_block
    from orpcd_amd.utils.constants import __ALIGNER_DEG__, __ALIGNER_MU__, __ALIGNER_STD__
    from workloads import c2_pair

    s, t = c2_pair(50_000)
    s, t = Preprocessor([]).preprocess(s), Preprocessor([]).preprocess(t)
    dm = (__ALIGNER_DEG__, __ALIGNER_MU__, __ALIGNER_STD__)
    np.random.seed(999)
    (Rb,), (tb,) = draw_block(1, *dm)
    np.random.seed(1000)
    R0, t0 = draw_block(30, *dm)
    R0, t0 = np.array(R0), np.array(t0)
    base = np.dot(s, Rb) + tb
    Rr = np.einsum("ji,bjk->bik", Rb, R0)  # Rb^T R0
    tr = t0 - np.einsum("j,bjk->bk", tb, Rr)
    print(f"|tb| = {np.linalg.norm(tb):.4g}, source extent {np.ptp(s, axis=0)}", flush=True)
    ctx = _native.Context(0)
    ctx.set_target(t)
    out = {}
    for rep in range(a.reps):
        for name, src, R, tt in (("plain", s, R0, t0), ("base", base, Rr, tr)):
            ctx.set_source(src)
            st0 = ctx.stats()
            t_0 = time.perf_counter()
            r = ctx.gicp_batch(R, tt)
            dt = time.perf_counter() - t_0
            st = ctx.stats()
            sync = st["host_sync_ms"] - st0["host_sync_ms"]
            print(f"{name:5s} rep {rep}: {dt * 1e3:.2f} ms (device wait {sync:.2f} ms), iters {int(r['iters'].sum())}",
                  flush=True)
            out.setdefault(name, []).append(r)
    p, b = out["plain"][-1], out["base"][-1]
    print("iterations identical:", bool(np.array_equal(p["iters"], b["iters"])),
          "max |d rmse|:", float(np.abs(p["rmse"] - b["rmse"]).max()), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
