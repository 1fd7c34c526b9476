"""Full Aligner.align() at C2 size on the GPU and on the CPU oracle: the
BASELINE metric's "final RMSE vs ref" leg.

    python tools/align_c2_parity.py [--points 50000] [--out profiles/r01_c2_align_parity.json]

Same inputs as bench.py's align() line (C2 pair, Preprocessor([]) =
RadiusScaler only, np.random.seed(0), 30 attempts, refine off).  The oracle
Aligner (the reference's control flow restated, C++/OpenMP GICP) runs the
complete align() on the host cores.  Reported: both wall-clocks, scale
factors, final RMSE and T, and the per-multistart metrics side by side.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO, os.path.join(REPO, "oracle")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=50_000)
    ap.add_argument("--attempts", type=int, default=30)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import oracle as O
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor
    from workloads import c2_pair
    src, tgt = c2_pair(a.points)

    opt = GeneralizedICP()
    for _ in range(2):  # the second run is the timed one (code objects, contexts warm)
        np.random.seed(0)
        al = Aligner(Preprocessor([]), Preprocessor([]), opt, attempts=a.attempts)
        t0 = time.perf_counter()
        T, m, sf, errors = al.align(src, tgt, refine_registration=False)
        tg = time.perf_counter() - t0
    np.random.seed(0)
    oal = O.OracleAligner(O.OracleGeneralizedICP(), attempts=a.attempts)
    t0 = time.perf_counter()
    To, mo, sfo, erro = oal.align(src, tgt)
    tc = time.perf_counter() - t0
    res = {"metric": "Aligner.align() at C2 (50k<->50k): GPU vs CPU oracle, final RMSE", "unit": "s",
           "gpu": {"seconds": round(tg, 3), "rmse": float(m), "scale_factors": sf.ravel().tolist(),
                   "multistarts": len(al.history), "compass_errors": [float(x) for x in errors]},
           "cpu_baseline": {"value": round(tc, 1), "unit": "s", "cores": O.num_threads(), "kind": "port",
                            "sample": "the complete align() on the host cores", "optimize_calls": len(oal.calls),
                            "rmse": float(mo), "scale_factors": np.asarray(sfo).ravel().tolist(),
                            "compass_errors": [float(x) for x in erro]},
           "speedup": round(tc / tg, 1),
           "parity": {"scale_factors_identical": bool(np.array_equal(sf, sfo)), "d_rmse": abs(float(m) - mo),
                      "max_abs_dT": float(np.abs(T - To).max()),
                      "compass_errors_max_abs_diff": float(np.max(np.abs(np.asarray(errors) - np.asarray(erro))))
                      if len(errors) == len(erro) else None}}
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
