"""C4 as BASELINE.json configs[3] words it: the Aligner's multi-start pattern
search -- the whole align() (speculative compass, refine off) with 64 starts
per multistart -- on one GPU, and its strong-scaling projection to G ranks.

    python tools/bench_c4_align.py [--attempts 64] [--ranks 8] [--points 50000] [--out FILE]

1. T1: align() on this GPU with world size 1.  Every multistart's gathered
   table of per-start records is kept, in call order.
2. Rank r of G (r = 0..G-1): the same align() (same seed, hence the same
   control flow and RNG stream) with parallel.world() -> (r, G): the rank
   runs only its contiguous block of every call's starts (parallel.shard of
   the initial multistart, or of a compass iteration's six candidates as one
   flat list) on this GPU, alone.  The all-gather is replayed from
   step 1's tables after checking that the rank's own rows are bit-identical
   to them (sharding never changes a start's result).  Each rank's time per
   _run_tables call (one compass iteration's six candidate shards, or the
   initial multistart) is recorded.
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
    a = ap.parse_args()
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor, parallel
    from workloads import c2_pair

    src, tgt = c2_pair(a.points)
    opt = GeneralizedICP()
    real_world, real_gather = parallel.world, parallel.allgather_records
    orig_run_tables = Aligner._run_tables
    calls = []  # per _run_tables call: seconds

    def timed_run_tables(self, source, targets, draws):
        t0 = time.perf_counter()
        r = orig_run_tables(self, source, targets, draws)
        calls.append(time.perf_counter() - t0)
        return r

    Aligner._run_tables = timed_run_tables

    def align_once():
        np.random.seed(a.seed)
        al = Aligner(Preprocessor([]), Preprocessor([]), opt, attempts=a.attempts)
        calls.clear()
        t0 = time.perf_counter()
        T, m, sf, err = al.align(src.copy(), tgt.copy(), refine_registration=False)
        wall = time.perf_counter() - t0
        iters = sum(h["iters"] for h in al.history) + sum(h["iters"] for h in al.speculative_history)
        return wall, list(calls), dict(T=np.asarray(T).tolist(), metric=float(m), sf=sf.ravel().tolist(), n_err=len(err)), iters

    # ---- 1. one GPU (warm-up run first: contexts, covariances, code objects)
    align_once()
    tables = []

    def recording_gather(local, B):
        t = real_gather(local, B)
        tables.append(t.copy())
        return t

    parallel.allgather_records = recording_gather
    t1, calls1, res1, iters1 = align_once()
    # ---- 2. every rank's shard alone
    rank_wall, rank_calls = [], []
    for r in range(a.ranks):
        k = [0]

        def replay(local, B, r=r):
            full = tables[k[0]]
            lo, hi = parallel.shard(B, r, a.ranks)
            assert np.array_equal(local, full[lo:hi]), f"rank {r} call {k[0]}: sharded rows differ"
            k[0] += 1
            return full

        parallel.world = lambda r=r: (r, a.ranks)
        parallel.allgather_records = replay
        w, c, res, _ = align_once()
        assert res["sf"] == res1["sf"] and res["metric"] == res1["metric"], (r, res, res1)
        assert k[0] == len(tables)
        rank_wall.append(w)
        rank_calls.append(c)
    parallel.world, parallel.allgather_records = real_world, real_gather
    Aligner._run_tables = orig_run_tables
    ncalls = len(calls1)
    assert all(len(c) == ncalls for c in rank_calls)
    per_call_max = [max(rc[i] for rc in rank_calls) for i in range(ncalls)]
    host_outside = max(w - sum(c) for w, c in zip(rank_wall, rank_calls))
    ag = len(tables) * a.allgather_us * 1e-6
    tG = sum(per_call_max) + ag + host_outside
    out = {
        "metric": f"C4 Aligner.align() pattern search wall-clock, {a.attempts} starts/multistart, "
                  f"{a.points // 1000}k<->{a.points // 1000}k (1-GPU measurement + {a.ranks}-rank projection)",
        "attempts": a.attempts, "ranks": a.ranks, "seed": a.seed,
        "t_1gpu_s": round(t1, 4),
        "gicp_iters_1gpu": int(iters1),
        "gicp_iters_per_s_1gpu": round(iters1 / t1, 1),
        "multistart_calls": ncalls, "allgathers": len(tables),
        "t_projected_s": round(tG, 4),
        "t_projected_parts_s": {"sum_per_call_max": round(sum(per_call_max), 4), "allgathers": round(ag, 4),
                                "host_outside_calls": round(host_outside, 4)},
        "rank_wall_s": [round(w, 4) for w in rank_wall],
        "projected_speedup": round(t1 / tG, 2),
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
