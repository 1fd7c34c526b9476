"""Where a bench.py step's time goes (C2, 30 starts): the same K steps
(np.random.seed(1000 + k), Aligner.multistart_registration) timed with the
library's live instrumentation off, with hipEvents only (count_tiles 0), and
with hipEvents + scanned-quarter counters (what bench.py's timed region runs).
    python tools/bench_overhead.py [--steps 10]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]
from orpcd_amd import Aligner, GeneralizedICP, Preprocessor  # noqa: E402
from workloads import c2_pair  # noqa: E402


def main():
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 10
    s, t = c2_pair(50_000)
    s, t = Preprocessor([]).preprocess(s), Preprocessor([]).preprocess(t)
    opt = GeneralizedICP(device=0)
    ctx = opt.context
    al = Aligner(Preprocessor([]), Preprocessor([]), opt, attempts=30)

    def run(k0):
        it = 0
        t0 = time.perf_counter()
        for k in range(steps):
            np.random.seed(1000 + k0 + k)
            al.multistart_registration(s, t)
            it += al.history[-1]["iters"]
        return time.perf_counter() - t0, it

    run(0)  # warm-up
    for rep in range(2):
        for name, prof, cnt in (("off", False, 1), ("events", True, 0), ("events+counters", True, 1)):
            ctx.set_option("count_tiles", cnt)
            ctx.reset_stats()
            ctx.profiling(prof)
            el, it = run(3)
            ctx.profiling(False)
            st = ctx.stats()
            print(f"{name:16s} {1e3 * el / steps:7.3f} ms/step  {it / el:9.1f} it/s  search {st['ms'] / steps:6.3f} "
                  f"ms/step  quarters {st['tiles'] / steps:.4g}", flush=True)
    ctx.set_option("count_tiles", 1)


if __name__ == "__main__":
    main()
