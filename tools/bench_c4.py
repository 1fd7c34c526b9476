"""C4 on one GPU: the Aligner's multistart with 64 starts (BASELINE configs[3]),
and the per-rank work of the same multistart sharded over G ranks.

    python tools/bench_c4.py [--attempts 64] [--ranks 8] [--steps 5] [--out FILE]

Each step draws the 64 starts from np.random exactly as Aligner does (seed
2000 + k).  Measured:
  * T1  = one device batch of all 64 starts (the 1-GPU run);
  * T_r = the batch of rank r's contiguous block of 64/G starts
    (parallel.shard), each timed alone on this GPU;
and the record all-gather of parallel.allgather_records
is charged at 0.1 ms (an RCCL all-gather of 64 x 160 B is latency-bound).
Projected G-GPU time per multistart = max_r T_r + all-gather; projected
strong-scaling speedup = T1 / that.  A projection from one GPU, not an
8-GPU measurement: the ranks share nothing but the all-gather
(SURVEY.md §8e), so their batches run as they do here, alone on a GPU.
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
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--points", type=int, default=50_000)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor, parallel
    from workloads import c2_pair

    s, t = c2_pair(a.points)
    s = Preprocessor([]).preprocess(s)
    t = Preprocessor([]).preprocess(t)
    opt = GeneralizedICP()
    al = Aligner(Preprocessor([]), Preprocessor([]), opt, attempts=a.attempts)

    def draws(k):
        np.random.seed(2000 + k)
        R0, t0 = zip(*[al.initialize_rotation() for _ in range(a.attempts)])
        return np.array(R0), np.array(t0).reshape(a.attempts, 3)

    def timed(R0, t0):
        t1 = time.perf_counter()
        r = opt.optimize_batch(s, t, R0, t0)
        return time.perf_counter() - t1, r

    timed(*draws(-1))  # warm-up (contexts, covariances)
    timed(*draws(-2))
    t_one, t_ranks, iters = [], [], 0
    for k in range(a.steps):
        R0, t0 = draws(k)
        el, r = timed(R0, t0)
        t_one.append(el)
        iters += int(np.sum(r["iters"]))
        per = []
        for rank in range(a.ranks):
            lo, hi = parallel.shard(a.attempts, rank, a.ranks)
            per.append(timed(R0[lo:hi], t0[lo:hi])[0])
        t_ranks.append(per)
    # the all-gather cannot be timed on one GPU: one RCCL all-gather of
    # 8 x 8 x 160 B over xGMI is latency-bound (tens of us); 0.1 ms is charged
    ag = 1e-4
    T1 = float(np.median(t_one))
    Tr = float(np.median([max(p) for p in t_ranks]))
    out = {
        "metric": "C4 multistart wall-clock, 64 starts, 50k<->50k (1-GPU measurement + 8-rank projection)",
        "attempts": a.attempts, "ranks": a.ranks, "steps": a.steps,
        "t_1gpu_ms": round(T1 * 1e3, 2),
        "t_rank_max_ms": round(Tr * 1e3, 2),
        "t_rank_each_ms_step0": [round(x * 1e3, 2) for x in t_ranks[0]],
        "allgather_ms_charged": round(ag * 1e3, 3),
        "projected_speedup": round(T1 / (Tr + ag), 2),
        "gicp_iters_per_s_1gpu": round(iters / sum(t_one), 1),
        "note": "projection: each rank's shard timed alone on one MI355X; ranks share only the all-gather",
    }
    print(json.dumps(out))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
