"""Is a device batch slower after the GPU sat idle?  (VERDICT r03 weak #6:
the drop-in path's speculative batches -- each preceded by ~17 ms of host-only
work serving the predicted calls -- ran 2x slower than the batched leg's
back-to-back batches of the same size.)

    python tools/idle_gap.py [--gaps 0,2,5,10,20,50] [--reps 6]

Times one C2 30-start batch (GeneralizedICP.optimize_batch, the same starts
every time) after a host-side idle gap of each length (time.sleep, GPU idle),
median over reps; the batch's own wall-clock only.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaps", default="0,1,2,5,10,20,50")
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--spin", type=int, default=0, help="busy-wait instead of sleeping during the gap")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor
    from workloads import c2_pair
    s, t = c2_pair(50_000)
    s, t = Preprocessor([]).preprocess(s), Preprocessor([]).preprocess(t)
    opt = GeneralizedICP()
    al = Aligner(Preprocessor([]), Preprocessor([]), opt, attempts=30)
    np.random.seed(1000)
    R0, t0 = al._draw_block(30)
    R0, t0 = np.array(R0), np.array(t0)
    for _ in range(3):
        opt.optimize_batch(s, t, R0, t0)
    out = {}
    for gap in [float(g) for g in a.gaps.split(",")]:
        ts = []
        for _ in range(a.reps):
            if a.spin:
                e = time.perf_counter() + gap * 1e-3
                while time.perf_counter() < e:
                    pass
            else:
                time.sleep(gap * 1e-3)
            t1 = time.perf_counter()
            opt.optimize_batch(s, t, R0, t0)
            ts.append(time.perf_counter() - t1)
        out[gap] = round(float(np.median(ts)) * 1e3, 3)
        print(f"gap {gap:5.1f} ms: batch {out[gap]:.2f} ms (min {min(ts) * 1e3:.2f}, max {max(ts) * 1e3:.2f})",
              file=sys.stderr, flush=True)
    line = json.dumps({"metric": "C2 30-start batch wall-clock after a host idle gap", "unit": "ms",
                       "spin": bool(a.spin), "batch_ms_by_gap_ms": out})
    print(line)
    if a.out:
        open(a.out, "w").write(line + "\n")


if __name__ == "__main__":
    main()
