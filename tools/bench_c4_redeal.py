"""C4's 8-rank projection with a one-time re-deal of the running starts
(VERDICT r04 item 8), from the device batches C4's align() really issues.

    python tools/bench_c4_redeal.py [--ranks 8] [--passes 16,24,32] [--out FILE]

1. align() with 64 starts per multistart runs as rank 0 of G (world patched,
   the all-gathers replayed from a 1-GPU run as in tools/bench_c4_align.py);
   every device batch (Aligner._run_tables call) is recorded: its targets and
   its flat list of K x 64 starts.  The control flow is the same on every
   rank, so this is every rank's sequence of batches.
2. Per batch and rank r (each alone on this GPU, as bench_c4_align times
   them): (a) its contiguous block of the flat list run to completion -- the
   shipped sharding; (b) with re-deal at pass P: the block over passes
   [0, P) (orpcd_gicp_batch_window), then -- after the (replayed) all-gather
   of every rank's states -- an even contiguous share of ALL ranks' still
   running starts resumed from pass P.  The re-dealt results are checked
   bit-identical to (a).
3. T_G = sum over batches of max over ranks of (a), versus sum of
   (max over ranks of phase 1 + max of phase 2 + one more all-gather at
   --allgather-us); both plus the host time outside the batches from
   profiles (--host-s).  Reported against T1 (--t1-s, the 1-GPU align()).
4. --move-layouts 1 (round 6): in phase 2 a rank ADOPTS the device layouts of
   the targets its share needs (orpcd_set_target_layouts, written once by
   their phase-1 owner with orpcd_get_target_layout) instead of building them
   again; the layouts it did not own are charged at --xgmi-gbps, and each
   owner's serialisation time is added to its phase 1.
A projection from one GPU, not an 8-GPU measurement.
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
    ap.add_argument("--passes", default="16,24,32")
    ap.add_argument("--allgather-us", type=float, default=50.0)
    ap.add_argument("--move-layouts", type=int, default=1)
    ap.add_argument("--xgmi-gbps", type=float, default=50.0,
                    help="point-to-point rate charged for a moved layout (one xGMI link, conservative)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor, _native, parallel
    from workloads import c2_pair

    src, tgt = c2_pair(a.points)
    opt = GeneralizedICP()
    real_world, real_gather = parallel.world, parallel.allgather_records
    orig_run_tables = Aligner._run_tables
    cur = {}
    calls = []

    def rec_run_tables(self, source, targets, draws, keys=None):
        cur["keys"] = keys
        K = len(draws)
        cur["call"] = dict(source=source, targets=targets(list(range(K))) if callable(targets) else list(targets),
                           draws=[(np.array(d[0]), np.array(d[1])) for d in draws], pos=self._positions(K))
        return orig_run_tables(self, source, targets, draws, keys=keys)

    Aligner._run_tables = rec_run_tables

    def align_once():
        np.random.seed(a.seed)
        al = Aligner(Preprocessor([]), Preprocessor([]), opt, attempts=a.attempts)
        t0 = time.perf_counter()
        al.align(src.copy(), tgt.copy(), refine_registration=False)
        return time.perf_counter() - t0

    # 1-GPU run: warm-up, then the timed one recording every multistart's rows
    align_once()
    rows = {}

    def recording_gather(local, B):
        t = real_gather(local, B)
        for key, p in zip(cur["keys"], cur["call"]["pos"]):
            rows[key] = t[p].copy()
        return t
    parallel.allgather_records = recording_gather
    t1 = align_once()
    # rank 0 of G: the batch sequence
    parallel.world = lambda: (0, a.ranks)

    def replay(local, B):
        full = np.zeros((B, parallel.REC))
        for key, p in zip(cur["keys"], cur["call"]["pos"]):
            if key in rows:
                full[p] = rows[key]
            else:
                full[p, 0] = np.inf
        lo, hi = parallel.shard(B, 0, a.ranks)
        full[lo:hi] = local
        calls.append(cur["call"])
        return full
    parallel.allgather_records = replay
    align_once()
    parallel.world, parallel.allgather_records = real_world, real_gather
    Aligner._run_tables = orig_run_tables

    ctx = _native.Context(0)
    prm = dict(max_correspondence_distance=0.5, max_iteration=100)

    def run(call, idx, pass_begin=0, pass_end=1 << 30, state=None):
        """Starts idx (flat positions) of one batch: set-up as the Aligner's rank does, timed."""
        flat_k, flat_R, flat_t = call["flat"]
        ks = sorted(set(flat_k[idx].tolist()))
        t0 = time.perf_counter()
        ctx.set_targets([call["targets"][k] for k in ks], 1e-3)
        ctx.set_source(call["source"])
        tids = np.searchsorted(ks, flat_k[idx]).astype(np.int32)
        r = ctx.gicp_batch_window(flat_R[idx], flat_t[idx], tids, pass_begin=pass_begin, pass_end=pass_end,
                                  state=state, **prm)
        return time.perf_counter() - t0, r

    builder = _native.Context(0)  # the phase-1 owners' contexts, as far as their layouts go

    def layouts_for(call):
        """Every target's device layout of one batch, as its phase-1 owner writes it: (tensor, ptr, bytes,
        seconds to write)."""
        if "lay" not in call:
            builder.set_targets(call["targets"], 1e-3, cache=False)
            lay = []
            for k in range(len(call["targets"])):
                n = builder.target_layout_bytes(k)
                ptr = builder.device_alloc(n)
                t0 = time.perf_counter()
                builder.get_target_layout(k, ptr, n)
                lay.append((None, ptr, n, time.perf_counter() - t0))
            call["lay"] = lay
        return call["lay"]

    def run_adopt(call, idx, owned, pass_begin, state):
        """Phase 2 of one rank with moved layouts: adopt, then resume; plus the charged transfer."""
        flat_k, flat_R, flat_t = call["flat"]
        ks = sorted(set(flat_k[idx].tolist()))
        lay = layouts_for(call)
        moved = sum(lay[k][2] for k in ks if k not in owned)
        t0 = time.perf_counter()
        ctx.set_target_layouts([lay[k][1] for k in ks])
        ctx.set_source(call["source"])
        tids = np.searchsorted(ks, flat_k[idx]).astype(np.int32)
        r = ctx.gicp_batch_window(flat_R[idx], flat_t[idx], tids, pass_begin=pass_begin, state=state, **prm)
        return time.perf_counter() - t0 + moved / (a.xgmi_gbps * 1e9), r, moved

    for call in calls:
        K = len(call["draws"])
        B = a.attempts
        flat_k = np.zeros(K * B, np.int64)
        flat_R = np.zeros((K * B, 3, 3))
        flat_t = np.zeros((K * B, 3))
        for k in range(K):
            p = call["pos"][k]
            flat_k[p] = k
            flat_R[p] = call["draws"][k][0]
            flat_t[p] = call["draws"][k][1]
        call["flat"] = (flat_k, flat_R, flat_t)
    G = a.ranks
    run(calls[0], np.arange(G))  # warm the kernels
    base = []   # per call: per rank seconds
    ref = []    # per call: full records by position
    for call in calls:
        n = len(call["flat"][0])
        ts, rec = [], {}
        for r in range(G):
            lo, hi = parallel.shard(n, r, G)
            dt, res = run(call, np.arange(lo, hi))
            ts.append(dt)
            for i, f in enumerate(range(lo, hi)):
                rec[f] = tuple(np.asarray(res[k][i]).tobytes() for k in ("T", "rmse", "iters"))
        base.append(ts)
        ref.append(rec)
    out = {"metric": f"C4 per-batch projection to {G} ranks, with and without a re-deal of the running starts",
           "batches": len(calls), "t1_s": round(t1, 4), "allgather_us": a.allgather_us,
           "no_redeal": {"sum_batch_max_s": round(sum(max(t) for t in base), 4),
                         "rank_s": [[round(x, 5) for x in t] for t in base]}}
    for P in [int(x) for x in a.passes.split(",")]:
        ph1, ph2, moved, identical, moved_bytes = [], [], [], True, []
        for call, rec in zip(calls, ref):
            n = len(call["flat"][0])
            t_1, done, state, owned = [], np.zeros(n, bool), np.zeros((n, 18)), []
            for r in range(G):
                lo, hi = parallel.shard(n, r, G)
                dt, res = run(call, np.arange(lo, hi), pass_end=P)
                own = set(call["flat"][0][lo:hi].tolist())
                owned.append(own)
                if a.move_layouts:  # the owner writes its targets' layouts for the others
                    dt += sum(layouts_for(call)[k][3] for k in own)
                t_1.append(dt)
                done[lo:hi] = res["done"]
                state[lo:hi] = res["state"]
                for i, f in enumerate(range(lo, hi)):
                    if res["done"][i]:
                        identical &= rec[f] == tuple(np.asarray(res[k][i]).tobytes() for k in ("T", "rmse", "iters"))
            U = np.nonzero(~done)[0]
            t_2 = []
            for r in range(G):
                lo, hi = parallel.shard(len(U), r, G)
                idx = U[lo:hi]
                if len(idx) == 0:
                    t_2.append(0.0)
                    continue
                if a.move_layouts:
                    dt, res, mb = run_adopt(call, idx, owned[r], P, state[idx])
                    moved_bytes.append(mb)
                else:
                    dt, res = run(call, idx, pass_begin=P, state=state[idx])
                t_2.append(dt)
                for i, f in enumerate(idx):
                    identical &= rec[f] == tuple(np.asarray(res[k][i]).tobytes() for k in ("T", "rmse", "iters"))
            ph1.append(t_1)
            ph2.append(t_2)
            moved.append(int(len(U)))
        tot = sum(max(x) for x in ph1) + sum(max(x) for x in ph2) + len(calls) * a.allgather_us * 1e-6
        out[f"redeal_P{P}"] = {"sum_s": round(tot, 4), "phase1_max_s": [round(max(x), 5) for x in ph1],
                               "phase2_max_s": [round(max(x), 5) for x in ph2], "running_at_P": moved,
                               "bit_identical": bool(identical), "move_layouts": bool(a.move_layouts),
                               "moved_layout_mb_per_rank_max": round(max(moved_bytes, default=0) / 1e6, 2)}
        print(f"P={P}: {tot:.4f} s vs {out['no_redeal']['sum_batch_max_s']:.4f} s, identical {identical}",
              file=sys.stderr, flush=True)
    s = json.dumps(out)
    print(s)
    if a.out:
        open(a.out, "w").write(s + "\n")


if __name__ == "__main__":
    main()
