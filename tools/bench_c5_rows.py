"""C5 row sharding projected to G GPUs from one MI355X (VERDICT r03 missing
#3): one GICP on the 1M<->1M pair (BASELINE.json configs[4]) with the source
rows split over G ranks (parallel.gicp_rows_sharded: every rank holds the
whole target and rows [lo, hi) of the source; per ICP pass each rank sums its
29 normal-equation terms, one all-reduce of 232 B combines them, every rank
applies the same update).

    python tools/bench_c5_rows.py [--ranks 1,2,4,8,16] [--iters 10] [--allreduce-us 30] [--out FILE]

Set-up per rank: rank r times orpcd_set_target_rows (the
whole target's layout and seed grid, the KNN-20 covariance pass over its 1/G
of the Morton rows) and orpcd_set_source_rows (the source layout, KNN-24 with
boundary ties for its rows only), warm (a second set-up on the same
context).  The all-gather that completes the target's covariances (m x 3
doubles) is charged at --allgather-gbs (RCCL all-gather over xGMI); in this
one-GPU projection the rows are assembled on the host, outside the timing.

For each G, G contexts on this GPU each hold one rank's rows (the full
target in each); every pass runs rank by rank, each rank's orpcd_gicp_shard_
pass timed alone (host wall-clock around the synchronous call: the rank has
the whole GPU, as it would on its own), the sums added on the host as the
all-reduce would, and every rank's orpcd_gicp_shard_update timed.  A
G-GPU pass then takes
    max over ranks of the pass + max over ranks of the update + one all-reduce
(--allreduce-us: a 232-B RCCL all-reduce over xGMI is latency-bound), and
T_G = the sum over the passes.  Every rank's final T is checked identical
across ranks and within 1e-9 of G = 1.  The per-pass floor is the pass time
as G grows (the launches of a pass over few rows).  A projection from one GPU,
not a G-GPU measurement.
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
    ap.add_argument("--points", type=int, default=1_000_000)
    ap.add_argument("--ranks", default="1,2,4,8,16")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--allreduce-us", type=float, default=30.0)
    ap.add_argument("--allgather-gbs", type=float, default=100.0)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from orpcd_amd import _native, parallel
    from workloads import c5_pair
    src, tgt = c5_pair(a.points)
    params = dict(max_correspondence_distance=0.5, max_iteration=a.iters)
    res = {}
    T_ref = None
    for G in [int(x) for x in a.ranks.split(",")]:
        ctxs = []
        t_setup, t_tgt, t_src, parts = [], [], [], []
        for r in range(G):
            c = _native.Context(0)
            lo, hi = parallel.shard(len(src), r, G)
            for rep in range(2):  # cold, then warm (the reported one)
                t0 = time.perf_counter()
                tlo, thi = c.set_target_rows(tgt, r, G, 1e-3)
                t1 = time.perf_counter()
                c.set_source_rows(src, lo, hi)
                t2 = time.perf_counter()
            t_tgt.append(t1 - t0)
            t_src.append(t2 - t1)
            t_setup.append(t2 - t0)
            parts.append(c.target_cov_rows(tlo, thi) if G > 1 else None)
            ctxs.append(c)
        if G > 1:  # the all-gather, on the host here (outside the timing)
            cov = np.concatenate(parts)
            for c in ctxs:
                c.set_target_cov(cov)
            allgather_s = cov.nbytes * (G - 1) / G / (a.allgather_gbs * 1e9)
        else:
            allgather_s = 0.0

        def run(timed):
            for c in ctxs:
                c.shard_begin(np.eye(3), np.zeros(3), n_total=len(src), **params)
            per_pass, per_upd, n_pass = [], [], 0
            while True:
                sums, tp, act = [], [], []
                for c in ctxs:
                    t0 = time.perf_counter()
                    s_, a_ = c.shard_pass()
                    tp.append(time.perf_counter() - t0)
                    sums.append(s_)
                    act.append(a_)
                assert len(set(act)) == 1
                if not act[0]:
                    break
                n_pass += 1
                total = np.sum(sums, axis=0)
                tu, done = [], []
                for c in ctxs:
                    t0 = time.perf_counter()
                    done.append(c.shard_update(total))
                    tu.append(time.perf_counter() - t0)
                per_pass.append(tp)
                per_upd.append(tu)
                assert len(set(done)) == 1
                if done[0]:
                    break
            return np.array(per_pass), np.array(per_upd), n_pass

        run(False)  # warm-up
        pp, pu, n_pass = run(True)
        rs = [c.shard_result() for c in ctxs]
        for r in rs[1:]:
            assert np.array_equal(r["T"], rs[0]["T"]) and r["iters"] == rs[0]["iters"]
        if T_ref is None:
            T_ref = rs[0]["T"]
        t_G = float(pp.max(axis=1).sum() + pu.max(axis=1).sum() + (a.allreduce_us * 1e-6 * n_pass if G > 1 else 0))
        rank_alone = pp.sum(axis=0) + pu.sum(axis=0)
        res[G] = {"passes": n_pass, "iters": int(rs[0]["iters"]), "T_seconds": round(t_G, 5),
                  "ms_per_pass": round(t_G / max(n_pass, 1) * 1e3, 4),
                  "rank_pass_ms_mean": round(float(pp.mean()) * 1e3, 4),
                  "rank_pass_ms_max": round(float(pp.max(axis=1).mean()) * 1e3, 4),
                  "update_ms_max": round(float(pu.max(axis=1).mean()) * 1e3, 4),
                  "slowest_rank_over_mean": round(float(rank_alone.max() / rank_alone.mean()), 4),
                  "max_abs_dT_vs_1": float(np.abs(rs[0]["T"] - T_ref).max()),
                  "rmse": rs[0]["rmse"],
                  "setup_rank_s": {"target_rows_max": round(max(t_tgt), 4), "source_rows_max": round(max(t_src), 4),
                                   "allgather_model": round(allgather_s, 5),
                                   "total_max": round(max(t_setup) + allgather_s, 4)},
                  "call_s": round(max(t_setup) + allgather_s + t_G, 4)}
        print(f"G={G}: {res[G]}", file=sys.stderr, flush=True)
        for c in ctxs:
            c.close()
    g1 = res.get(1, {}).get("T_seconds")
    for G, r in res.items():
        r["speedup_vs_1"] = round(g1 / r["T_seconds"], 3) if g1 else None
        r["iters_per_s"] = round(r["iters"] / r["T_seconds"], 2)
    floor = min(r["ms_per_pass"] for r in res.values())
    line = {"metric": "C5 GICP (1M<->1M, one start) with source rows over G GPUs, projected from one MI355X",
            "unit": "s", "allreduce_us": a.allreduce_us, "per_rank_projection": res,
            "per_pass_floor_ms": floor, "allgather_gbs": a.allgather_gbs,
            "note": "pass times measured rank by rank, each alone on the GPU; the all-reduce charged at "
            "--allreduce-us per pass; set-up per rank warm (target rows + source rows) plus the covariance "
            "all-gather at --allgather-gbs; call_s = set-up + iterations"}
    s = json.dumps(line)
    print(s)
    if a.out:
        open(a.out, "w").write(s + "\n")


if __name__ == "__main__":
    main()
