"""The zero-code-change drop-in path at C2: the reference-shaped sequential
multistart (one GeneralizedICP.optimize per attempt, Aligner.py:178-202, as
the reference's own Aligner calls the plugin) against the batched multistart
(optimize_batch, one device batch of 30 starts).

    python tools/bench_dropin.py [--reps 3] [--out profiles/r03_dropin.json]

Multistart legs: np.random.seed(1000) once, then `reps` consecutive
multistarts (the stream continues, as between the multistarts of an
align()), 30 attempts each, timed per multistart (median):
  batched      Aligner -> GeneralizedICP.optimize_batch
  dropin       Aligner over a plugin exposing only optimize(): every call
               hands over source @ R0 + t0; the plugin recognises the rigid
               image of its cached cloud (GeneralizedICP._rigid_image), runs
               the start on the cached layout / covariances, and from the
               second call on runs the predicted next attempts ahead as one
               batch (GeneralizedICP speculate=29, the default)
  dropin_nospec  the same with speculate=0: one device batch per call
  dropin_cold  the same with rigid_cache=False: every posed copy uploaded,
               laid out and its KNN-20 covariances recomputed, as Open3D does
Per-start results of the drop-in legs are compared with the batched table.
align legs: the complete C2 align() (refine off, np.random.seed(0)) through
the batched Aligner and through the reference-shaped sequential Aligner over
the drop-in plugin (second of two runs each).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]


class OnlyOptimize:
    """An IOptimizer with nothing but optimize(): the Aligner takes its
    sequential path (Aligner.py:178-202), exactly the reference's calls."""

    def __init__(self, inner):
        self.inner = inner
        self.rmse = []
        self.inside = 0.0  # seconds inside the plugin's optimize()

    def optimize(self, source, target, **kw):
        t0 = time.perf_counter()
        T, m = self.inner.optimize(source, target, **kw)
        self.inside += time.perf_counter() - t0
        self.rmse.append(m)
        return T, m


class Constant:
    """A plugin that returns at once: the reference loop's own cost per
    multistart (deepcopy, initialize_rotation, np.dot per attempt)."""

    def optimize(self, source, target, **kw):
        return np.eye(4), 1.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--attempts", type=int, default=30)
    ap.add_argument("--out", default=None)
    ap.add_argument("--opt", default="{}", help="runtime options (orpcd_set_option), JSON")
    ap.add_argument("--events", type=int, default=0, help="time the search launches with hipEvents (stats ms)")
    ap.add_argument("--legs", default="caller_only,batched,dropin,dropin_nospec,dropin_cold,align",
                    help="comma-separated subset of the legs to run")
    a = ap.parse_args()
    legs = set(a.legs.split(","))
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor
    from workloads import c2_pair
    s, t = c2_pair(50_000)
    s, t = Preprocessor([]).preprocess(s), Preprocessor([]).preprocess(t)

    from orpcd_amd import _native
    ctx = _native.default_context(None)
    for k, v in json.loads(a.opt).items():
        ctx.set_option(k, v)

    def leg(opt, name):
        al = Aligner(Preprocessor([]), Preprocessor([]), opt, attempts=a.attempts)
        np.random.seed(999)
        al.multistart_registration(s, t)  # warm-up
        ctx.reset_stats()
        if a.events:
            ctx.set_option("count_tiles", 0)
            ctx.profiling(True)
        times, rmse, inside = [], [], []
        np.random.seed(1000)
        for k in range(a.reps):
            if isinstance(opt, OnlyOptimize):
                opt.rmse = []
                opt.inside = 0.0
            t0 = time.perf_counter()
            al.multistart_registration(s, t)
            times.append(time.perf_counter() - t0)
            if isinstance(opt, OnlyOptimize):
                inside.append(opt.inside)
            rmse.append(np.array(opt.rmse) if isinstance(opt, OnlyOptimize) else
                        al.history[-1]["rmse"] if hasattr(al, "history") and al.history else None)
        print(f"{name}: {np.median(times) * 1e3:.1f} ms per multistart"
              + (f" ({np.median(inside) * 1e3:.1f} ms inside optimize())" if inside else ""), file=sys.stderr, flush=True)
        leg.inside[name] = round(float(np.median(inside)) * 1e3, 2) if inside else None
        ctx.profiling(False)
        st = ctx.stats()
        nb = max(st["host_batches"], 1)
        leg.host[name] = {k: round(st[k] / nb, 3) for k in ("host_batch_ms", "host_launch_ms", "host_sync_ms")}
        if a.events:
            leg.host[name]["search_ms_per_batch"] = round(st["ms"] / nb, 3)
            leg.host[name]["search_launches_per_batch"] = round(st["launches"] / nb, 1)
        leg.host[name]["batches"] = int(st["host_batches"])
        print(f"  {name} per batch: {leg.host[name]}", file=sys.stderr, flush=True)
        return float(np.median(times)), rmse

    leg.inside = {}
    leg.host = {}

    nan = (float("nan"), None)
    tk, _ = leg(Constant(), "caller_only") if "caller_only" in legs else nan
    tb, rb = leg(GeneralizedICP(), "batched") if "batched" in legs else nan
    spec = GeneralizedICP()
    td, rd = leg(OnlyOptimize(spec), "dropin") if "dropin" in legs else nan
    tn, rn = leg(OnlyOptimize(GeneralizedICP(speculate=0)), "dropin_nospec") if "dropin_nospec" in legs else nan
    tc, rc = leg(OnlyOptimize(GeneralizedICP(rigid_cache=False)), "dropin_cold") if "dropin_cold" in legs else nan
    from workloads import c2_pair as pair

    def align_leg(opt, name):
        src_raw, tgt_raw = pair(50_000)
        for _ in range(2):
            np.random.seed(0)
            al = Aligner(Preprocessor([]), Preprocessor([]), opt, attempts=a.attempts)
            t0 = time.perf_counter()
            T, m, sf, err = al.align(src_raw.copy(), tgt_raw.copy(), refine_registration=False)
            dt = time.perf_counter() - t0
        print(f"{name} align: {dt:.3f} s, rmse {m:.12g}", file=sys.stderr, flush=True)
        return dt, float(m)

    spec_al = GeneralizedICP()
    if "align" in legs:
        ta_b, ma_b = align_leg(GeneralizedICP(), "batched")
        ta_d, ma_d = align_leg(OnlyOptimize(spec_al), "dropin")
    else:
        ta_b = ma_b = ta_d = ma_d = float("nan")

    def dmax(r):
        return max(float(np.abs(x - y).max()) for x, y in zip(r, rb)) if r is not None and rb is not None else None
    d_warm, d_cold, d_nospec = dmax(rd), dmax(rc), dmax(rn)
    res = {"metric": "multistart wall-clock at C2 (30 starts), drop-in sequential vs batched", "unit": "ms",
           "batched_ms": round(tb * 1e3, 2), "dropin_ms": round(td * 1e3, 2), "dropin_cold_ms": round(tc * 1e3, 2),
           "dropin_nospec_ms": round(tn * 1e3, 2), "speculation": spec.spec_stats,
           "caller_only_ms": round(tk * 1e3, 2), "inside_optimize_ms": leg.inside, "host_per_batch": leg.host,
           "dropin_over_batched": round(td / tb, 2), "dropin_cold_over_batched": round(tc / tb, 2),
           "max_abs_d_rmse_vs_batched": {"dropin": d_warm, "dropin_nospec": d_nospec, "dropin_cold": d_cold},
           "align": {"batched_s": round(ta_b, 4), "dropin_s": round(ta_d, 4),
                     "dropin_over_batched": round(ta_d / ta_b, 2), "d_rmse": abs(ma_d - ma_b),
                     "speculation": spec_al.spec_stats},
           "reps": a.reps, "attempts": a.attempts}
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
