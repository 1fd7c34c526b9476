"""Drop-in slowdown: does a batch run slower when the
GPU has been idle (or the host busy) just before it?  The same 30 C2 starts
as one gicp_batch, 6 times per mode:

  b2b    back to back (the batched Aligner's pattern)
  sleep  after the host sleeps `gap` ms (GPU idle)
  numpy  after `gap` ms of host numpy work like the drop-in caller's
         (deepcopy + np.dot of the 50k cloud per attempt)
  munmap after allocating, touching and freeing a 64 MB array (above
         glibc's largest mmap threshold: every free is an munmap)

Per batch: wall time of the call and the stats' device-wait share.
    python tools/idle_ab.py [--gap 20] [--reps 6]
"""
import argparse
import copy
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gap", type=float, default=20.0)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--modes", default="b2b,sleep,numpy,b2b,sleep")
    ap.add_argument("--opt", default="{}")
    a = ap.parse_args()
    from orpcd_amd import Preprocessor, _native
    from orpcd_amd.Aligner.Aligner import draw_block
    from workloads import c2_pair

    s, t = c2_pair(50_000)
    s, t = Preprocessor([]).preprocess(s), Preprocessor([]).preprocess(t)
    np.random.seed(1000)
    R0, t0 = draw_block(30, np.pi / 2, 0.0, 0.1)
    R0, t0 = np.array(R0), np.array(t0)
    ctx = _native.Context(0)
    for k, v in json.loads(a.opt).items():
        ctx.set_option(k, v)
    ctx.set_target(t)
    ctx.set_source(s)
    ctx.gicp_batch(R0, t0)
    res = {}
    for mode in a.modes.split(","):
        walls, syncs = [], []
        for _ in range(a.reps):
            if mode == "sleep":
                time.sleep(a.gap * 1e-3)
            elif mode == "numpy":
                t_end = time.perf_counter() + a.gap * 1e-3
                k = 0
                while time.perf_counter() < t_end:
                    x = copy.deepcopy(s)
                    np.dot(x, R0[k % 30]) + t0[k % 30]
                    k += 1
            elif mode == "munmap":
                x = np.ones(8 << 20)
                del x
            st0 = ctx.stats()
            w = time.perf_counter()
            ctx.gicp_batch(R0, t0)
            walls.append((time.perf_counter() - w) * 1e3)
            syncs.append(ctx.stats()["host_sync_ms"] - st0["host_sync_ms"])
        line = f"{mode:6s} wall ms {np.round(walls, 2).tolist()} (median {np.median(walls):.2f}); " \
               f"device wait median {np.median(syncs):.2f}"
        print(line, flush=True)
        res.setdefault(mode, []).append(round(float(np.median(walls)), 2))
    print(json.dumps({"gap_ms": a.gap, "median_wall_ms": res}))
    ctx.close()


if __name__ == "__main__":
    main()
