"""One warm Aligner.align() at C2 (speculative compass, refine off) for
profiling:  python tools/one_align.py [--attempts 30] [--reps 2]"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--attempts", type=int, default=30)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--points", type=int, default=50_000)
    a = ap.parse_args()
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor
    from workloads import c2_pair
    src, tgt = c2_pair(a.points)
    opt = GeneralizedICP()
    for _ in range(a.reps):
        np.random.seed(0)
        al = Aligner(Preprocessor([]), Preprocessor([]), opt, attempts=a.attempts)
        t0 = time.perf_counter()
        T, m, sf, err = al.align(src.copy(), tgt.copy(), refine_registration=False)
        t = time.perf_counter() - t0
        ms = [round(h["seconds"] * 1e3, 1) for h in al.history]
        print(f"align {t * 1e3:.1f} ms  metric {m:.9g} sf {sf.ravel().tolist()}  multistart ms {ms}", flush=True)


if __name__ == "__main__":
    main()
