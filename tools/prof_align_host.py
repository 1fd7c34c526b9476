"""Host-side profile of one C2 align() with 64 starts per multistart (C4's
workload): cProfile's view of where the Python time goes between and around
the device batches (tottime; the batches themselves show as ctypes calls)."""
import cProfile
import os
import pstats
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]
from orpcd_amd import Aligner, GeneralizedICP, Preprocessor  # noqa: E402
from workloads import c2_pair  # noqa: E402

src, tgt = c2_pair(50_000)
opt = GeneralizedICP()
for _ in range(2):
    np.random.seed(0)
    al = Aligner(Preprocessor([]), Preprocessor([]), opt, attempts=64)
    t0 = time.perf_counter()
    al.align(src, tgt, refine_registration=False)
    print("align", time.perf_counter() - t0, flush=True)
np.random.seed(0)
al = Aligner(Preprocessor([]), Preprocessor([]), opt, attempts=64)
pr = cProfile.Profile()
pr.enable()
al.align(src, tgt, refine_registration=False)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
