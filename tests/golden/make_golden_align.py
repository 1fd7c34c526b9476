"""Golden fixtures g7: the CPU oracle's COMPLETE Aligner.align() at C1 and C2.

    python tests/golden/make_golden_align.py [--which c1,c2]

TEST INFRASTRUCTURE.  Runs the oracle Aligner (the reference's control flow,
Aligner.py:228-317, restated in oracle/oracle.py and pinned by g3; GICP by the
C++/OpenMP restatement of Open3D 0.18, oracle/orpcd_oracle.cpp) on:

* C1: ArmadilloBack_330 -> _0, Preprocessor([RandomDownsampler(5000), SOR()])
  for both clouds (RadiusScaler auto-inserted), np.random.seed(0), 30 attempts,
  refine off (BASELINE.json configs[0]);
* C2: the same scans densified to 50k points each (workloads.c2_pair),
  Preprocessor([]) (RadiusScaler only), np.random.seed(0), 30 attempts, refine
  off (configs[1]);
* C4: C2 with 64 attempts per multistart (configs[3]: the north_star's
  64-start pattern search that bench.py --gpus N times at every N).

Stored per config (g7_align_<cfg>.npz): the final T, metric, scale factors and
compass errors, and for every optimize call in call order its (R0, t0), the
returned row-convention T, rmse, fitness and iteration count.  The GPU test
(tests/test_gpu_align.py) and bench.py's align line compare against these.
C2 takes several minutes on 8 host cores (the complete run, every call).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]


class RecordingGICP:
    """OracleGeneralizedICP that keeps every call's full result."""

    def __init__(self, O):
        self.O = O
        self.inner = O.OracleGeneralizedICP()
        self.rec = []
        self.t0 = time.perf_counter()

    def optimize(self, source, target, **kw):
        T, m = self.inner.optimize(source, target, **kw)
        r = self.inner.last
        self.rec.append((T.copy(), float(m), float(r["fitness"]), int(r["iters"])))
        if len(self.rec) % 30 == 0:
            print(f"  {len(self.rec)} optimize calls, {time.perf_counter() - self.t0:.0f} s", file=sys.stderr,
                  flush=True)
        return T, m


def run(cfg):
    import oracle as O
    from workloads import armadillo, c2_pair

    if cfg == "c1":
        src, tgt = armadillo()

        def pre(c):  # Preprocessor([RandomDownsampler(5000), SOR()]) with RadiusScaler first
            x = O.random_downsample(O.radius_scale(c)[0], 5000)
            return x[O.sor(x, 64, 2)[0]]
    else:
        src, tgt = c2_pair(50_000)
        pre = None
    attempts = 64 if cfg == "c4" else 30
    opt = RecordingGICP(O)
    np.random.seed(0)
    al = O.OracleAligner(opt, attempts=attempts, preprocess=pre)
    t0 = time.perf_counter()
    T, metric, sf, errors = al.align(src, tgt)
    el = time.perf_counter() - t0
    calls = al.calls
    out = dict(
        T=np.asarray(T), metric=np.float64(metric), sf=np.asarray(sf, dtype=np.float64).reshape(1, 3),
        errors=np.asarray(errors, dtype=np.float64),
        R0=np.array([c[0] for c in calls]), t0=np.array([c[1] for c in calls]),
        call_T=np.array([r[0] for r in opt.rec]), call_rmse=np.array([r[1] for r in opt.rec]),
        call_fitness=np.array([r[2] for r in opt.rec]), call_iters=np.array([r[3] for r in opt.rec], np.int32))
    np.savez_compressed(os.path.join(HERE, f"g7_align_{cfg}.npz"), **out)
    meta = {"config": cfg, "attempts": attempts, "seconds": round(el, 1), "cores": O.num_threads(),
            "optimize_calls": len(calls),
            "gicp_iterations": int(out["call_iters"].sum()), "metric": float(metric),
            "scale_factors": out["sf"].ravel().tolist()}
    with open(os.path.join(HERE, f"g7_align_{cfg}.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(json.dumps(meta), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="c1,c2")
    a = ap.parse_args()
    for cfg in a.which.split(","):
        run(cfg)


if __name__ == "__main__":
    main()
