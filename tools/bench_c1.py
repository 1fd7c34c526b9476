"""C1 end to end: Aligner.align() on the reference's own CPU-runnable case.

    python tools/bench_c1.py [--attempts 30] [--cpu 1] [--out profiles/r01_c1.json]

ArmadilloBack_330 -> ArmadilloBack_0 (tests/golden/armadillo.npz, parsed from
the reference's sample PLYs), Preprocessor([RandomDownsampler(5000), SOR()])
for both clouds (RadiusScaler auto-inserted), np.random.seed(0), GICP
defaults, refine_registration=False (BASELINE.json configs[0]).  The GPU
Aligner (SOR and every GICP on the MI355X) runs it once for warm-up and once
timed; the CPU oracle Aligner (C++/OpenMP GICP, the same Python control flow
and RNG stream) runs the COMPLETE align() once.  Reported: both wall-clocks,
GICP iterations, and parity (scale factors identical, |dRMSE|, |dT|).
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
    ap.add_argument("--attempts", type=int, default=30)
    ap.add_argument("--cpu", type=int, default=1)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor
    from orpcd_amd.Preprocessor.Downsamplers import RandomDownsampler
    from orpcd_amd.Preprocessor.Outliers import SOR
    from workloads import armadillo
    src, tgt = armadillo()

    def run_gpu(exact=False):
        np.random.seed(0)
        al = Aligner(Preprocessor([RandomDownsampler(5000), SOR()]), Preprocessor([RandomDownsampler(5000), SOR()]),
                     GeneralizedICP(exact_nn=exact), attempts=a.attempts)
        t0 = time.perf_counter()
        T, m, sf, errors = al.align(src, tgt, refine_registration=False)
        return time.perf_counter() - t0, T, m, sf, errors, al

    run_gpu()  # warm-up: code objects, allocations
    tg, T, m, sf, errors, al = run_gpu()
    run_gpu(True)
    tx, Tx, mx, sfx, errx, alx = run_gpu(True)  # exact_nn: the oracle's correspondences
    iters = int(sum(h["iters"] for h in al.history))
    res = {"metric": "Aligner.align() wall-clock (C1: Armadillo 330->0, Random(5000)+SOR, GICP)", "unit": "s",
           "value": round(tg, 3), "higher_is_better": False, "n_gpus": 1,
           "data": "ArmadilloBack_330 / _0 scans of the reference (armadillo.npz), np.random.seed(0)",
           "config": {"workload": "C1", "attempts": a.attempts, "refine_registration": False},
           "gpu": {"seconds": round(tg, 3), "rmse": float(m), "scale_factors": sf.ravel().tolist(),
                   "multistarts": len(al.history), "gicp_iters": iters, "compass_errors": len(errors)}}
    if a.cpu:
        import oracle as O

        def pre(c):
            x = O.random_downsample(O.radius_scale(c)[0], 5000)
            return x[O.sor(x, 64, 2)[0]]
        np.random.seed(0)
        oal = O.OracleAligner(O.OracleGeneralizedICP(), attempts=a.attempts, preprocess=pre)
        t0 = time.perf_counter()
        To, mo, sfo, erro = oal.align(src, tgt)
        tc = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(tc, 2), "unit": "s", "cores": O.num_threads(), "kind": "port",
                               "sample": "the complete align() (every optimize call) on the host cores",
                               "optimize_calls": len(oal.calls)}
        res["speedup"] = round(tc / tg, 1)
        res["parity"] = {"scale_factors_identical": bool(np.array_equal(sf, sfo)), "d_rmse": abs(float(m) - mo),
                         "max_abs_dT": float(np.abs(T - To).max()), "compass_errors_identical_len": len(errors) == len(erro)}
        res["exact_nn"] = {"seconds": round(tx, 3), "rmse": float(mx),
                           "parity": {"scale_factors_identical": bool(np.array_equal(sfx, sfo)),
                                      "d_rmse": abs(float(mx) - mo), "max_abs_dT": float(np.abs(Tx - To).max()),
                                      "compass_errors_max_abs_diff": float(np.max(np.abs(np.asarray(errx) - np.asarray(erro))))
                                      if len(errx) == len(erro) else None}}
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
