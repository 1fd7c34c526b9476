"""C5 measurement: one GICP on the 1M<->1M synthetic pair (max_iterations=30).

    python tools/bench_c5.py [--points 1000000] [--iters 30] [--cpu-iters 2] [--out FILE]
    torchrun --nproc-per-node N tools/bench_c5.py ...   # source rows sharded over N GPUs

Reports GICP iterations/s of the single start (each iteration = one exact
nearest-neighbour pass over all 1M source points + the 6x6 solve), the
nn_search kernel's roofline on evaluated pairs (8 FLOP/pair, fp32 peak), the
one-time covariance cost, and the CPU oracle timed on a bounded number of
iterations of the same problem.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]
FP32_PEAK_TF = 157.3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--cpu-iters", type=int, default=2)
    ap.add_argument("--parity", type=int, default=1, help="also run the full oracle GICP and compare")
    ap.add_argument("--out", default=None)
    ap.add_argument("--opt", default="{}", help="runtime options (orpcd_set_option), JSON")
    ap.add_argument("--path", choices=["auto", "rows", "batch"], default="auto",
                    help="rows: the row-sharded pass API (a host all-reduce every pass); batch: orpcd_gicp_batch "
                         "with one start (host sync every sync_every passes; bit-identical at one rank); "
                         "auto: batch on one GPU, rows on several")
    ap.add_argument("--device-collectives", type=int, default=0,
                    help="rows path: target all-gather and per-pass all-reduce on the library's RCCL communicator")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        import torch
        import torch.distributed as dist
        # ORPCD_BENCH_BACKEND=gloo / ORPCD_BENCH_DEVICE=0: rehearsal of the multi-rank path on a one-GPU box
        torch.cuda.set_device(int(os.environ.get("ORPCD_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0"))))
        dist.init_process_group(os.environ.get("ORPCD_BENCH_BACKEND", "nccl"))
    from orpcd_amd import _native, parallel
    from workloads import c5_pair
    src, tgt = c5_pair(args.points)
    t_ctx = time.perf_counter()
    ctx = _native.Context(int(os.environ.get("ORPCD_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0"))) if world > 1
                          else None)
    ctx_create_s = time.perf_counter() - t_ctx  # the process's first context: GPU runtime init + warm-up
    for k, v in json.loads(args.opt).items():
        ctx.set_option(k, v)
    params = dict(max_correspondence_distance=0.5, max_iteration=args.iters)

    path = args.path if args.path != "auto" else ("batch" if world == 1 else "rows")
    if path == "batch" and world > 1:
        raise SystemExit("--path batch runs one GPU")
    lo, hi = parallel.shard(len(src), rank, world)

    def setup():
        """The call's set-up, as registration_generalized_icp does it
        (generalizedICP.py:59-70 builds both KD-trees and covariances inside
        the call): target and source uploaded, laid out, KNN-20 covariances.
        Returns (target s, source s)."""
        t_0 = time.perf_counter()
        if path == "rows":  # the target's covariance pass split by rows, one all-gather
            parallel.target_rows_sharded(ctx, tgt, 1e-3, device_collectives=bool(args.device_collectives))
        else:
            ctx.set_target(tgt, 1e-3, cache=False)
        t_1 = time.perf_counter()
        if path == "batch":
            ctx.set_source(src, cache=False)
        else:
            ctx.set_source_rows(src, lo, hi)
        return t_1 - t_0, time.perf_counter() - t_1

    cold_target_s, cold_source_s = setup()  # first call of the process: allocations, code objects
    setup_s = cold_target_s + cold_source_s

    def run_rows(prm):
        ctx.shard_begin(np.eye(3), np.zeros(3), n_total=len(src), **prm)
        if args.device_collectives:
            parallel.device_comm(ctx)
            ctx.shard_run()
            return ctx.shard_result()
        while True:
            sums, act = ctx.shard_pass()
            if not act or ctx.shard_update(parallel.allreduce_sum(sums)):
                break
        return ctx.shard_result()

    def run_batch(prm):
        b = ctx.gicp_batch(np.eye(3)[None], np.zeros((1, 3)), **prm)
        return {k: (v[0] if k == "T" else v[0].item()) for k, v in b.items()}

    def run(prm=params):
        return run_batch(prm) if path == "batch" else run_rows(prm)

    t0 = time.perf_counter()
    run(dict(params, max_iteration=1))  # warm-up (code objects, allocations) on a short run
    cold_first_run_s = time.perf_counter() - t0
    # the whole call warm: set-up + iterations, as one registration_generalized_icp call
    warm = []
    for _ in range(3):
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        ts, ss = setup()
        t1 = time.perf_counter()
        run()
        warm.append((ts, ss, t1 - t0, time.perf_counter() - t0))
    warm.sort(key=lambda w: w[3])
    warm_t, warm_s, warm_setup, warm_call = warm[len(warm) // 2]

    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    r = run()
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # a second, HIP-event-timed run for the kernel roofline (its host syncs
    # for the tile counters are kept out of the timed run above)
    ctx.profiling(True)
    ctx.reset_stats()
    run()
    ctx.profiling(False)
    st = ctx.stats()
    passes = r["iters"] + 1
    line = {
        "metric": "GICP iterations/s, one start, 1M<->1M (C5)",
        "value": round(r["iters"] / elapsed, 3), "unit": "GICP iterations/s", "higher_is_better": True,
        "n_gpus": world, "scaling": "strong", "dtype": "f32+f64",
        "data": "synthetic C5 (bumpy sphere, default_rng(5), target = R(10deg) x + 0.02 + N(0,1e-4))",
        "config": {"workload": "C5: GeneralizedICP max_iterations=30 from identity", "points": len(src),
                   "parallelism": (f"source rows over {world} GPU(s), all-reduce of 29 f64 per pass" if path == "rows"
                                   else "one start, orpcd_gicp_batch (bit-identical to the one-rank row path)"),
                   "path": path},
        "ms_per_iteration": round(1e3 * elapsed / max(passes, 1), 3),
        "setup_s": round(setup_s, 4),
        # one registration_generalized_icp call end to end (its KD-trees / covariances included, as the
        # CPU baseline's): set-up + iterations, median of 3 warm calls; cold = the process's first
        "call_s": {"warm": round(warm_call, 4), "warm_setup": round(warm_setup, 4),
                   "warm_setup_target": round(warm_t, 4), "warm_setup_source": round(warm_s, 4),
                   "warm_iterations": round(warm_call - warm_setup, 4),
                   "cold": round(setup_s + cold_first_run_s + elapsed, 4), "cold_setup": round(setup_s, 4),
                   "cold_setup_target": round(cold_target_s, 4), "cold_setup_source": round(cold_source_s, 4),
                   "ctx_create": round(ctx_create_s, 4),
                   "lazy_code_objects": bool(os.environ.get("ORPCD_LAZY_CODE_OBJECTS")),
                   "note": "cold = first set-up + the 1-iteration warm-up run + the timed run, on a fresh context; "
                           "ctx_create = the process's first orpcd_ctx_create (HIP runtime init, code-object "
                           "loads and the synthetic set-up warm-up, profiles/r06_c5_cold.md)"},
        "value_end_to_end": round(r["iters"] / warm_call, 3),
        "result": {"rmse": r["rmse"], "fitness": r["fitness"], "iters": r["iters"], "ncorr": r["ncorr"]},
    }
    if st["launches"] > 0:
        avg_ms = st["ms"] / st["launches"]
        achieved = st["pairs"] / st["launches"] * 8 / (avg_ms * 1e-3) / 1e12
        line["roofline"] = {"bound": "valu_fp32", "kernel": "nn_search_kernel", "achieved": round(achieved, 3),
                            "peak": FP32_PEAK_TF, "unit": "TFLOP/s", "frac": round(achieved / FP32_PEAK_TF, 4),
                            "avg_launch_ms": round(avg_ms, 4),
                            "pairs_vs_bruteforce": round(st["pairs"] / st["launches"] / (hi - lo) / len(tgt), 6)}
    if rank == 0 and world == 1 and args.cpu_iters > 0:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle
        t0 = time.perf_counter()
        o = oracle.gicp(src, tgt, 0.5, args.cpu_iters)
        cpu_s = time.perf_counter() - t0
        line["cpu_baseline"] = {"value": round(o["iters"] / cpu_s, 4), "unit": "GICP iterations/s",
                                "cores": oracle.num_threads(), "kind": "port",
                                "sample": f"first {o['iters']} iterations of the same GICP (incl. its KD-trees "
                                          f"and covariances), {cpu_s:.1f} s"}
        if args.parity:
            o = oracle.gicp(src, tgt, 0.5, args.iters)
            line["parity"] = {"oracle_iters": o["iters"], "max_abs_dT": float(np.abs(o["T"] - r["T"]).max()),
                              "d_rmse": abs(o["rmse"] - r["rmse"]), "d_fitness": abs(o["fitness"] - r["fitness"])}
    if rank == 0:
        s = json.dumps(line)
        print(s, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(s + "\n")
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
