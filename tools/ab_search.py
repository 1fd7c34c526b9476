"""Interleaved A/B of runtime options on one multistart (C2 pair, 30 starts).

    python tools/ab_search.py '{"super_cull":0}' '{"super_cull":1}' ... [--rounds 5]

Each round runs every config once (same starts), so clock/thermal drift hits
all variants alike (cdna_hip_programming.md §5.4 rule 24).  Prints median
and min ms per multistart and GICP iterations (must be equal across configs).
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
    args = [a for a in sys.argv[1:] if a.startswith("{")]
    rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 5
    points = int(sys.argv[sys.argv.index("--points") + 1]) if "--points" in sys.argv else 50000
    B = int(sys.argv[sys.argv.index("--starts") + 1]) if "--starts" in sys.argv else 30
    configs = [json.loads(a) for a in args] or [{}]
    s, t = c2_pair(points)
    s = Preprocessor([]).preprocess(s)
    t = Preprocessor([]).preprocess(t)
    rng = np.random.default_rng(1000)
    R0 = np.array([rot_xyz(*rng.uniform(-90, 90, 3)) for _ in range(B)])
    t0 = rng.normal(size=(B, 3)) * 0.1
    ctx = _native.Context(0)
    ctx.set_target(t)
    ctx.set_source(s)
    ctx.gicp_batch(R0, t0)  # warm-up (code objects, allocations)
    times = {i: [] for i in range(len(configs))}
    iters = {}
    Ts = {}
    filed = {}  # exact mode: queries re-searched in fp64 over the batch
    for _ in range(rounds):
        for i, cfg in enumerate(configs):
            for k, v in cfg.items():  # over the library defaults (options persist: give each config every key varied)
                ctx.set_option(k, v)
            ctx.reset_stats()
            t1 = time.perf_counter()
            r = ctx.gicp_batch(R0, t0)
            times[i].append((time.perf_counter() - t1) * 1e3)
            iters[i] = int(r["iters"].sum())
            Ts[i] = r["T"]
            filed[i] = ctx.stats().get("exact_filed", 0.0)
    for i, cfg in enumerate(configs):
        a = np.array(times[i])
        dT = float(np.abs(Ts[i] - Ts[0]).max())
        print(f"{json.dumps(cfg):50s} median {np.median(a):8.2f} ms  min {a.min():8.2f} ms  iters {iters[i]}  "
              f"max|dT| vs first {dT:.1e}  re-searched {filed[i]:.0f}")


if __name__ == "__main__":
    main()
