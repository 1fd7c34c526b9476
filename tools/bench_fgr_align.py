"""The reference's README usage end to end: Aligner + FastGlobalOptimizer.

    python tools/bench_fgr_align.py [--attempts 30] [--cpu-seconds 15] [--out profiles/r05_fgr_align.json]

ArmadilloBack_330 -> ArmadilloBack_0 (tests/golden/armadillo.npz),
Preprocessor([RandomDownsampler(5000), SOR()]) for both clouds (RadiusScaler
auto-inserted), FastGlobalOptimizer() with its defaults, np.random.seed(0),
refine_registration=False (README.md:37-40 with the visualiser off).

Timed on the GPU: the batched Aligner (optimize_batch_multi: every multistart
and the speculative compass's candidates as orpcd_fgr_optimize_batch calls)
and the reference-shaped sequential Aligner calling optimize() once per
attempt (Aligner.py:164-204); both warm.  Their results must be identical bit
for bit (scale factors, compass errors, T, metric, RNG position).  CPU
baseline: the oracle's FastGlobalOptimizer (C++/OpenMP restatement of Open3D's
FPFH + FGR) on the sequential run's first posed copies for --cpu-seconds,
extrapolated per call to the align()'s calls.
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
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from orpcd_amd import Aligner, FastGlobalOptimizer, Preprocessor
    from orpcd_amd.Optimizer.iOptimizer import IOptimizer
    from orpcd_amd.Preprocessor.Downsamplers import RandomDownsampler
    from orpcd_amd.Preprocessor.Outliers import SOR
    from workloads import armadillo

    class PerCall(IOptimizer):
        """optimize() only, recording the posed copies (the reference's Aligner path)"""

        def __init__(self):
            self.inner = FastGlobalOptimizer()
            self.calls = []

        def optimize(self, source, target, **kwargs):
            if len(self.calls) < 64:
                self.calls.append((source.copy(), target.copy()))
            else:
                self.calls.append(None)
            return self.inner.optimize(source, target)

    src, tgt = armadillo()

    def run(opt):
        np.random.seed(0)
        pp = lambda: Preprocessor([RandomDownsampler(5000), SOR()])  # noqa: E731
        al = Aligner(pp(), pp(), opt, attempts=a.attempts)
        t0 = time.perf_counter()
        T, m, sf, errors = al.align(src, tgt, refine_registration=False)
        return dict(seconds=time.perf_counter() - t0, T=T, metric=float(m), sf=np.asarray(sf).copy(),
                    errors=list(map(float, errors)), rng=np.random.uniform(size=3), al=al)

    out = {"workload": "README.md:37-40: Aligner(Preprocessor([RandomDownsampler(5000), SOR()]) x2, "
                       "FastGlobalOptimizer()) on ArmadilloBack_330 -> ArmadilloBack_0, seed 0, refine off",
           "attempts": a.attempts}
    run(FastGlobalOptimizer())  # warm-up (code objects, device buffers)
    bat = run(FastGlobalOptimizer())
    seq_opt = PerCall()
    run(seq_opt)
    seq_opt.calls.clear()
    seq = run(seq_opt)
    al = bat["al"]
    out["batched"] = dict(seconds=round(bat["seconds"], 4), multistarts=len(al.history),
                          speculative_extra_multistarts=len(al.speculative_history),
                          starts_run=int(a.attempts * (len(al.history) + len(al.speculative_history))))
    out["sequential_per_call"] = dict(seconds=round(seq["seconds"], 4), optimize_calls=len(seq_opt.calls),
                                      ms_per_call=round(1e3 * seq["seconds"] / max(len(seq_opt.calls), 1), 3))
    out["speedup_batched_vs_per_call"] = round(seq["seconds"] / bat["seconds"], 2)
    out["identical"] = dict(scale_factors=bool(np.array_equal(bat["sf"], seq["sf"])),
                            errors=bat["errors"] == seq["errors"], T=bool(np.array_equal(bat["T"], seq["T"])),
                            metric=bat["metric"] == seq["metric"], rng_after=bool(np.array_equal(bat["rng"], seq["rng"])))
    out["result"] = dict(metric=bat["metric"], scale_factors=bat["sf"].ravel().tolist(), errors=bat["errors"])
    s0, t0_ = seq_opt.calls[0]
    out["clouds"] = dict(source_points=len(s0), target_points=len(t0_))
    if a.cpu_seconds > 0:
        import oracle as O
        from bench import usable_cpus
        cores, how = usable_cpus()
        O.set_num_threads(cores)
        oo = O.OracleFastGlobalOptimizer(seed=0)
        t_0 = time.perf_counter()
        k, match = 0, 0
        for c in seq_opt.calls:
            if c is None or time.perf_counter() - t_0 > a.cpu_seconds:
                break
            To, ro = oo.optimize(c[0], c[1])
            Tg, rg = FastGlobalOptimizer().optimize(c[0], c[1])
            match += int(np.abs(To - Tg).max() <= 1e-8 and abs(ro - rg) <= 1e-9)
            k += 1
        el = time.perf_counter() - t_0
        per = el / max(k, 1)  # includes the GPU re-run (~ms), negligible against the oracle
        out["cpu_baseline"] = dict(kind="port", cores=cores, cores_how=how, calls_timed=k,
                                   seconds_per_call=round(per, 4),
                                   align_seconds_extrapolated=round(per * len(seq_opt.calls), 1),
                                   speedup_batched=round(per * len(seq_opt.calls) / bat["seconds"], 1),
                                   parity_calls_within_1e8=f"{match}/{k}")
    print(json.dumps(out, indent=1))
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
