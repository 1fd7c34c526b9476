"""PCIe-inclusive rate of the C2 multistart: the boundary hands over host
float64 clouds (orpcd_set_target / orpcd_set_source: upload, Morton layout, KNN-20
covariances) and host R0/t0; bench.py's `value` is measured with the clouds already
resident.  This times both, uncached, beside the resident multistart.

    python tools/pcie_inclusive.py [--reps 5]
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]
from orpcd_amd import Preprocessor, _native  # noqa: E402
from workloads import c2_pair, rot_xyz  # noqa: E402


def main():
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 5
    s, t = c2_pair(50000)
    s = Preprocessor([]).preprocess(s)
    t = Preprocessor([]).preprocess(t)
    rng = np.random.default_rng(1000)
    R0 = np.array([rot_xyz(*rng.uniform(-90, 90, 3)) for _ in range(30)])
    t0 = rng.normal(size=(30, 3)) * 0.1
    ctx = _native.Context(0)
    ctx.set_target(t)
    ctx.set_source(s)
    ctx.gicp_batch(R0, t0)  # warm-up (allocations)
    setup, batch, iters = [], [], 0
    for _ in range(reps):
        a = time.perf_counter()
        ctx.set_target(t, cache=False)
        ctx.set_source(s, cache=False)
        b = time.perf_counter()
        r = ctx.gicp_batch(R0, t0)
        c = time.perf_counter()
        setup.append(b - a)
        batch.append(c - b)
        iters = int(r["iters"].sum())
    su, ba = float(np.median(setup)), float(np.median(batch))
    out = dict(points=50000, starts=30, gicp_iterations=iters, setup_ms=round(1e3 * su, 3),
               multistart_resident_ms=round(1e3 * ba, 3),
               resident_iters_per_s=round(iters / ba, 1),
               pcie_inclusive_iters_per_s=round(iters / (su + ba), 1),
               host_bytes_in=int(s.nbytes + t.nbytes + R0.nbytes + t0.nbytes),
               note="setup = both clouds uploaded as float64 and laid out, covariances computed; "
                    "an align() pays it once per compass scale for the target and once for the source")
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
