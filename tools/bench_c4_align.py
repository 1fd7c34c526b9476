"""C4 as BASELINE.json configs[3] words it: the Aligner's multi-start pattern
search -- the whole align() (speculative compass, refine off) with 64 starts
per multistart -- on one GPU, and its strong-scaling projection to G ranks.

    python tools/bench_c4_align.py [--attempts 64] [--ranks 8] [--points 50000] [--out FILE]

1. T1: align() on this GPU with world size 1.  Every multistart's gathered
   table of per-start records is kept, in call order.
2. Rank r of G (r = 0..G-1): the same align() (same seed, hence the same
   control flow and RNG stream) with parallel.world() -> (r, G): the rank
   runs only its contiguous block of every device batch's flat list of
   starts (parallel.shard) on this GPU, alone, with the speculative depth
   the G-rank run would choose (auto: 2, i.e. each batch also holds the next
   compass iteration along the "all six fail" path; --depth overrides).  The
   all-gather is replayed from step 1's rows of every multistart (keyed by
   RNG block and target scale) after checking that the rank's own rows are
   bit-identical to them (sharding never changes a start's result); a
   multistart step 1 never ran was speculated past the reference's path and
   is never selected.  Each rank's time per device batch (_run_tables call)
   is recorded.
3. Projection: the ranks synchronise at every all-gather, so
   T_G = sum over calls of max over ranks of that call's time
       + every all-gather at `--allgather-us` (one RCCL all-gather of
         G x (attempts/G) x 160 B over xGMI is latency-bound)
       + the host time outside the calls (max over ranks).
   speedup = T1 / T_G.  A projection from one GPU, not an 8-GPU measurement:
   the ranks share nothing but the all-gathers.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--attempts", type=int, default=64)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--points", type=int, default=50_000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--allgather-us", type=float, default=50.0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--depth", type=int, default=None, help="speculative_depth of the ranks (default: auto)")
    ap.add_argument("--interleave", action="store_true", help="ranks shard the flat start list attempt-major")
    ap.add_argument("--profile-rank", type=int, default=None, help="cProfile this rank's align() (host time)")
    a = ap.parse_args()
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor, parallel
    from workloads import c2_pair

    src, tgt = c2_pair(a.points)
    opt = GeneralizedICP()
    real_world, real_gather = parallel.world, parallel.allgather_records
    orig_run_tables = Aligner._run_tables
    calls = []  # per _run_tables call: seconds
    cur_keys = []  # the multistarts of the running call

    def timed_run_tables(self, source, targets, draws, keys=None):
        cur_keys[:] = keys
        t0 = time.perf_counter()
        r = orig_run_tables(self, source, targets, draws, keys=keys)
        calls.append(time.perf_counter() - t0)
        return r

    Aligner._run_tables = timed_run_tables

    def align_once(depth=None):
        np.random.seed(a.seed)
        al = Aligner(Preprocessor([]), Preprocessor([]), opt, attempts=a.attempts, speculative_depth=depth,
                     shard_interleave=a.interleave and parallel.world()[1] > 1)
        calls.clear()
        t0 = time.perf_counter()
        T, m, sf, err = al.align(src.copy(), tgt.copy(), refine_registration=False)
        wall = time.perf_counter() - t0
        iters = sum(h["iters"] for h in al.history) + sum(h["iters"] for h in al.speculative_history)
        return wall, list(calls), dict(T=np.asarray(T).tolist(), metric=float(m), sf=sf.ravel().tolist(), n_err=len(err)), iters

    # ---- 1. one GPU (warm-up run first: contexts, covariances, code objects)
    align_once()
    rows = {}  # (block, scale) -> the multistart's gathered rows
    ngather = [0]

    def positions(K, interleave):  # as Aligner._positions
        return [k + K * np.arange(a.attempts) if interleave else k * a.attempts + np.arange(a.attempts)
                for k in range(K)]

    def recording_gather(local, B):
        t = real_gather(local, B)
        for key, p in zip(cur_keys, positions(len(cur_keys), False)):  # the 1-GPU run: target-major
            rows[key] = t[p].copy()
        ngather[0] += 1
        return t

    parallel.allgather_records = recording_gather
    t1, calls1, res1, iters1 = align_once()
    n1 = ngather[0]
    # ---- 2. every rank's shard alone; the all-gather returns the 1-GPU rows
    # of every multistart (a multistart the 1-GPU run never evaluated was
    # speculated past the reference's path: its rows are never selected and
    # are filled with rmse = inf)
    rank_wall, rank_calls, rank_gathers, rank_iters = [], [], [], []
    for r in range(a.ranks):
        k = [0]
        its = []  # per call: (max, sum) of this rank's starts' iterations

        def replay(local, B, r=r):
            full = np.zeros((B, parallel.REC))
            known = np.zeros(B, bool)
            for key, p in zip(cur_keys, positions(len(cur_keys), a.interleave)):
                if key in rows:
                    full[p] = rows[key]
                    known[p] = True
                else:
                    full[p, 0] = np.inf
            lo, hi = parallel.shard(B, r, a.ranks)
            its.append((int(local[:, 2].max()) if len(local) else 0, int(local[:, 2].sum())))
            m = known[lo:hi]
            assert np.array_equal(local[m], full[lo:hi][m]), f"rank {r} call {k[0]}: sharded rows differ"
            full[lo:hi] = local
            k[0] += 1
            return full

        parallel.world = lambda r=r: (r, a.ranks)
        parallel.allgather_records = replay
        if a.profile_rank == r:
            import cProfile
            import pstats
            pr = cProfile.Profile()
            pr.enable()
        w, c, res, _ = align_once(a.depth)
        if a.profile_rank == r:
            pr.disable()
            pstats.Stats(pr, stream=sys.stderr).sort_stats("tottime").print_stats(25)
        assert res["sf"] == res1["sf"] and res["metric"] == res1["metric"], (r, res, res1)
        rank_wall.append(w)
        rank_calls.append(c)
        rank_gathers.append(k[0])
        rank_iters.append(its)
    parallel.world, parallel.allgather_records = real_world, real_gather
    Aligner._run_tables = orig_run_tables
    ncalls = len(rank_calls[0])
    assert all(len(c) == ncalls for c in rank_calls)
    per_call_max = [max(rc[i] for rc in rank_calls) for i in range(ncalls)]
    host_outside = max(w - sum(c) for w, c in zip(rank_wall, rank_calls))
    ag = rank_gathers[0] * a.allgather_us * 1e-6
    tG = sum(per_call_max) + ag + host_outside
    # the same projection if every call's work were spread evenly over the
    # ranks (the bound a perfect re-deal could reach)
    per_call_mean = [float(np.mean([rc[i] for rc in rank_calls])) for i in range(ncalls)]
    t_bal = sum(per_call_mean) + ag + host_outside
    # what sets a rank's call time: its starts' largest iteration count (the
    # passes it runs) or their summed iterations (its work)
    xs = np.array([[rank_iters[r][i][0], rank_iters[r][i][1], rank_calls[r][i]] for r in range(a.ranks)
                   for i in range(min(ncalls, len(rank_iters[r])))], float)
    corr = {"max_iters": round(float(np.corrcoef(xs[:, 0], xs[:, 2])[0, 1]), 3) if len(xs) > 2 else None,
            "sum_iters": round(float(np.corrcoef(xs[:, 1], xs[:, 2])[0, 1]), 3) if len(xs) > 2 else None}
    out = {
        "metric": f"C4 Aligner.align() pattern search wall-clock, {a.attempts} starts/multistart, "
                  f"{a.points // 1000}k<->{a.points // 1000}k (1-GPU measurement + {a.ranks}-rank projection)",
        "attempts": a.attempts, "ranks": a.ranks, "seed": a.seed,
        "t_1gpu_s": round(t1, 4),
        "gicp_iters_1gpu": int(iters1),
        "gicp_iters_per_s_1gpu": round(iters1 / t1, 1),
        "calls_1gpu": len(calls1), "calls_ranks": ncalls, "allgathers": rank_gathers[0],
        "t_projected_s": round(tG, 4),
        "t_projected_parts_s": {"sum_per_call_max": round(sum(per_call_max), 4), "allgathers": round(ag, 4),
                                "host_outside_calls": round(host_outside, 4)},
        "rank_wall_s": [round(w, 4) for w in rank_wall],
        "per_call_1gpu_s": [round(x, 5) for x in calls1],
        "per_call_rank_s": [[round(x, 5) for x in c] for c in rank_calls],

        "per_call_rank_iters_max_sum": rank_iters,
        "call_time_correlation": corr,
        "projected_speedup": round(t1 / tG, 2),
        "projected_speedup_balanced": round(t1 / t_bal, 2),
        "speculative_depth": {"1gpu": "auto", "ranks": a.depth or "auto"}, "shard_interleave": a.interleave,
        "result": res1,
        "note": "every rank's shard timed alone on one MI355X (same seed, same control flow); its rows were "
                "checked bit-identical to the 1-GPU table; all-gathers replayed and charged",
    }
    print(json.dumps(out))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
