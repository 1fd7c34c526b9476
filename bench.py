"""Benchmark: GICP iterations/s of the MI355X inner registration loop (C2).

    python bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[1]): ArmadilloBack_330 ->
ArmadilloBack_0 densified to 50,000 points each (synthetic: sampling with
replacement + 5e-5 jitter, workloads.c2_pair), RadiusScaler-normalised
(Preprocessor([])), GICP defaults (max_corr 0.5, 100 iterations).

One step = one Aligner.multistart_registration over the pair at scale (1,1,1)
with `--attempts` (default 30, the reference's default) starts PER GPU, i.e.
Aligner(attempts = 30 * N): the starts are drawn from the global numpy RNG
exactly as the reference draws them, each is a full GICP run, the starts of a
rank run as ONE device batch (one process per GPU, torch.distributed with
RCCL), and one all-gather of a 160-byte record per start lets every rank
replay the reference's argmin.  Per-GPU work is fixed as N grows (weak
scaling: the multistart is partitioned into independent starts; the only
collective is that all-gather).

value = GICP iterations completed (all starts, all ranks) / max-over-ranks
wall time of the K timed steps, in the default (exact) correspondence mode:
every correspondence is the fp64 KD-tree answer Open3D would return
(GeneralizedICP(exact_nn=True)), so each start's trajectory is
the oracle's.  Also reported (rank 0, N=1): the dominant kernel's roofline
(live hipEvent timing inside the library on its own stream), the same steps
with every cloud re-uploaded (setup-inclusive rate) and in the fp32-answer
mode (exact_nn=False), a CPU baseline (the oracle: C++/OpenMP KD-tree GICP on
the host cores, bounded sample of the same starts) with per-start parity, and
one full Aligner.align() wall-clock compared with the committed complete
oracle align() (tests/golden/g7_align_c2.npz).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "multi-scale-pointcloud-registration_amd"))
sys.path.insert(0, REPO)

FP32_PEAK_TFLOPS = 157.3    # MI355X FP32 VALU (packed v_pk_* math), MI355X_MICROARCH.md
# VALU issue roof: 1024 SIMDs (256 CUs x 4) x 2.4 GHz (MI355X_MICROARCH.md max clock); gfx950's SIMDs
# are SIMD-32 and issue a wave64 VALU instruction every 2 cycles at throughput (MI355X_MICROARCH.md
# "Wave scheduling" and the v_fma_f32 row of its cycle constants; rounds 1-4 used the SIMD-16 figure
# of 4 cycles, which halved this roof)
VALU_ISSUE_PEAK_GINST = 1024 * 2.4 / 2  # G wave-instructions/s
WAVE_SLOTS = 256 * 4 * 5    # search waves resident at most: 5 per SIMD (amdgpu_waves_per_eu(5), 94 VGPRs)
FLOP_PER_PAIR = 8           # 3 sub + 3 mul/fma(=5) per query-target distance


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one process per GPU); N > 1 without WORLD_SIZE spawns the N rank processes "
                         "itself (default: WORLD_SIZE when launched by torch.distributed.run, else 1)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--points", type=int, default=50_000)
    ap.add_argument("--attempts", type=int, default=30, help="multistart starts per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="CPU baseline sample budget (0 = skip)")
    ap.add_argument("--align", type=int, default=1, help="also time one full align() on rank 0 (N=1)")
    ap.add_argument("--c4", type=int, default=1,
                    help="also time C4 at every N: align() with --c4-attempts starts per multistart, sharded over "
                         "the N ranks (strong scaling: the same total work at every N)")
    ap.add_argument("--c4-attempts", type=int, default=64)
    return ap.parse_args()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """`--gpus N` (N > 1) started without a launcher: start the N rank
    processes here, one per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N,
    rendezvous on 127.0.0.1), exactly as `python -m torch.distributed.run
    --nproc-per-node N bench.py --gpus N ...` would.  This parent never
    imports torch or touches a GPU; it forwards nothing but waits, and exits
    with the first non-zero rank status (the other ranks are then stopped), so
    a failed rank fails the run.  Rank 0 prints the JSON line."""
    import signal
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env))
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                print(f"bench.py: rank {procs.index(p)} exited with {rc}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                for q in live:
                    q.send_signal(signal.SIGTERM)
        if live:
            time.sleep(0.05)
    return status


def _bench_optimizer(device):
    """The optimizer the bench drives: the build's GeneralizedICP (HIP) -- or,
    for the CPU rehearsal of the multi-rank launch only (tests/test_bench_launch.py),
    the class named by ORPCD_BENCH_OPTIMIZER="file.py:Class", which must
    provide the same optimize_batch / context surface."""
    spec = os.environ.get("ORPCD_BENCH_OPTIMIZER")
    if not spec:
        from orpcd_amd import GeneralizedICP
        return GeneralizedICP(device=device)
    import importlib.util
    path, cls = spec.rsplit(":", 1)
    m = importlib.util.spec_from_file_location("orpcd_bench_optimizer", path)
    mod = importlib.util.module_from_spec(m)
    m.loader.exec_module(mod)
    return getattr(mod, cls)(device=device)


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus is not None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(env_world or "1")
    if args.gpus is not None and args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU "
              f"(--nproc-per-node {args.gpus}) or drop --gpus", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # ORPCD_BENCH_BACKEND=gloo / ORPCD_BENCH_DEVICE=0: rehearsal of the
    # multi-rank path on a one-GPU box (production: nccl = RCCL, GPU = LOCAL_RANK)
    device = int(os.environ.get("ORPCD_BENCH_DEVICE", local_rank))
    on_gpu = not os.environ.get("ORPCD_BENCH_OPTIMIZER")
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist

        if on_gpu:
            torch.cuda.set_device(device)
        dist.init_process_group(os.environ.get("ORPCD_BENCH_BACKEND", "nccl"), init_method="env://")

    from orpcd_amd import Aligner, Preprocessor
    from workloads import c2_pair

    src_raw, tgt_raw = c2_pair(args.points)
    source = Preprocessor([]).preprocess(src_raw)
    target = Preprocessor([]).preprocess(tgt_raw)

    opt = _bench_optimizer(device)
    ctx = opt.context
    devices = [device]
    if dist is not None:
        devices = [None] * world
        dist.all_gather_object(devices, device)
    total_attempts = args.attempts * world
    aligner = Aligner(Preprocessor([]), Preprocessor([]), opt, attempts=total_attempts)

    def barrier():
        if dist is not None:
            import torch
            if on_gpu:
                torch.cuda.synchronize()
            dist.barrier()

    def step(k, al=aligner):
        np.random.seed(1000 + k)  # identical draws on every rank
        al.multistart_registration(source, target)
        return al.history[-1]["iters"]

    for k in range(args.warmup):
        step(k)
    h0 = aligner.history[0] if args.warmup > 0 else None  # seed 1000's starts
    rmse_step0 = np.array(h0["rmse"]) if h0 else None
    iters_step0 = np.array(h0["iters_per_start"]) if h0 and "iters_per_start" in h0 else None
    # the timed region runs with the library's live hipEvent timing (the search
    # launches' durations) but without its scanned-quarter counters: their
    # atomics cost 7-14% of a step (tools/bench_overhead.py); the counts come
    # from a replay of the same steps below
    ctx.reset_stats()
    ctx.set_option("count_tiles", 0)
    ctx.profiling(True)
    barrier()
    t0 = time.perf_counter()
    iters = 0
    for k in range(args.steps):
        iters += step(args.warmup + k)
    barrier()
    elapsed = time.perf_counter() - t0
    ctx.profiling(False)
    st = ctx.stats()
    # replay (untimed): the same seeds, so the same starts and trajectories;
    # only the scan counters are taken from it
    ctx.reset_stats()
    ctx.set_option("count_tiles", 1)
    ctx.profiling(True)
    for k in range(args.steps):
        step(args.warmup + k)
    ctx.profiling(False)
    rp = ctx.stats()
    st["pairs"], st["tiles"], st["passes"] = rp["pairs"], rp["tiles"], rp["passes"]
    replay_ms = rp["ms"]
    ctx.reset_stats()
    if dist is not None:
        import torch
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        s = torch.tensor([st["ms"], st["launches"], st["pairs"], st["sched_launches"]], dtype=torch.float64,
                         device=dev)
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        st["ms"], st["launches"], st["pairs"], st["sched_launches"] = (float(x) for x in s.tolist())

    value = iters / elapsed
    # the search kernel that ran: the ordered dispatch for batches of >= 16
    # starts (option sched_min_starts), else the uniform-split kernel
    kname = "nn_search_sched_kernel" if st["sched_launches"] * 2 > st["launches"] else "nn_search_kernel"
    # the instantiation that ran: <true> in exact mode (the default), <false> otherwise
    traffic, traffic_src = pmc_traffic("orpcd::" + kname, bool(getattr(opt, "_exact_nn", True)))
    valu_insts = pmc_counter("orpcd::" + kname, bool(getattr(opt, "_exact_nn", True)), "SQ_INSTS_VALU")
    avg_ms = st["ms"] / max(st["launches"], 1)
    flops_per_launch = st["pairs"] / max(st["launches"], 1) * FLOP_PER_PAIR
    achieved = flops_per_launch / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0

    cpu = None
    align_s = None
    parity = None
    fast = None
    setup = None
    if rank == 0 and world == 1 and on_gpu:
        setup = setup_inclusive_run(ctx, step, args)
        o = o_iters = None
        if args.cpu_seconds > 0:
            cpu = cpu_baseline(source, target, args)
            # "final RMSE vs ref" per start: the GPU's inlier RMSE of step 0 against the
            # oracle's on the same starts (exact mode: identical iterations, |d rmse| ~1e-13)
            o = np.array(cpu.pop("oracle_rmse"))
            o_iters = np.array(cpu.pop("oracle_iters"))
            if rmse_step0 is not None and len(o):
                d = np.abs(rmse_step0[: len(o)] - o)
                parity = {"starts": int(len(o)), "max_abs_d_rmse": float(d.max()),
                          "within_1e-9": int((d <= 1e-9).sum()),
                          "multistart_min_rmse_gpu": float(rmse_step0[: len(o)].min()),
                          "multistart_min_rmse_oracle": float(o.min())}
                if iters_step0 is not None:
                    parity["iterations_identical"] = int((iters_step0[: len(o)] == o_iters).sum())
        fast = fast_mode_run(source, target, args, local_rank, o, o_iters)
        if args.align:
            # one cold align() (device contexts of the speculative compass created
            # inside it), then the same align() warm: the figure reported
            cold = None
            for _ in range(2):
                np.random.seed(0)
                al = Aligner(Preprocessor([]), Preprocessor([]), opt, attempts=args.attempts)
                t1 = time.perf_counter()
                T, metric, sf, errors = al.align(src_raw, tgt_raw, refine_registration=False)
                cold = cold if cold is not None else time.perf_counter() - t1
            align_s = dict(seconds=round(time.perf_counter() - t1, 3), seconds_cold=round(cold, 3), rmse=float(metric),
                           scale_factors=[round(float(x), 6) for x in sf.ravel()],
                           multistarts=len(al.history), gicp_iters=int(sum(h["iters"] for h in al.history)),
                           speculative_extra_multistarts=len(al.speculative_history))
            align_s.update(align_vs_fixture(T, metric, sf, errors, align_s["seconds"]))

    c4 = c4_run(opt, src_raw, tgt_raw, args, barrier, dist) if args.c4 else None

    if rank == 0:
        line = {
            "metric": "GICP iters/sec (Aligner multistart, 50k<->50k)",
            "value": round(value, 3),
            "unit": "GICP iterations/s",
            "n_gpus": world,
            "devices": devices,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32+f64",
            "data": "synthetic (Armadillo 330->0 densified to 50k, jitter 5e-5; seeds fixed)",
            "config": {"workload": "C2: Armadillo pair @50k pts, GeneralizedICP defaults, one multistart/step",
                       "points": args.points, "attempts_per_step": total_attempts,
                       "attempts_per_gpu": args.attempts,
                       "parallelism": f"multistart starts sharded over {world} GPU(s), one all-gather per step"},
            "roofline": {"bound": "valu_fp32", "achieved": round(achieved, 3), "peak": FP32_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved / FP32_PEAK_TFLOPS, 4), "traffic": traffic,
                         "traffic_source": traffic_src,
                         # the binding resource: VALU instructions issued per launch (committed SQ_INSTS_VALU,
                         # same command) over the live launch time, against the VALU issue roof -- most
                         # issued instructions are culling and bookkeeping, not pair FLOPs
                         "valu_issue": None if not valu_insts or avg_ms <= 0 else {
                             "insts_per_launch": round(valu_insts),
                             "achieved_ginst_s": round(valu_insts / (avg_ms * 1e-3) / 1e9, 1),
                             "peak_ginst_s": VALU_ISSUE_PEAK_GINST,
                             "frac": round(valu_insts / (avg_ms * 1e-3) / 1e9 / VALU_ISSUE_PEAK_GINST, 3)},
                         # where the search's wave-cycles go (committed SQ counters of the same command):
                         # parked on memory / issue-stalled / issuing, and the average resident waves
                         "stalls": pmc_stalls("orpcd::" + kname, bool(getattr(opt, "_exact_nn", True))),
                         "note": "achieved = 8 FLOP x pairs the culled search evaluates; it falls whenever "
                                 "culling improves (round 4's 8-point in-tile boxes: 39% fewer pairs per "
                                 "launch in a 4% shorter launch). Neither roof binds: the stall breakdown "
                                 "(latency: waves parked on memory and dependency chains) does, DESIGN.md §6",
                         "kernel": kname, "avg_launch_ms": round(avg_ms, 4),
                         "search_kernel_ms_total": round(st["ms"], 3),
                         "launches": int(st["launches"]), "flop_per_pair": FLOP_PER_PAIR,
                         "pairs_source": "replay of the timed steps with the scan counters on "
                                         f"(its search time {replay_ms:.1f} ms vs {st['ms']:.1f} ms timed)",
                         "pairs_per_launch": round(st["pairs"] / max(st["launches"], 1)),
                         "pairs_vs_bruteforce": round(st["pairs"] / max(st["passes"] * len(source) * len(target), 1),
                                                      5),
                         # SURVEY §8d's brute-force count (8*N*M per start per pass) over the same kernel
                         # time: what a brute-force search would have to sustain to match (not a roofline)
                         "bruteforce_equivalent_tflops": round(
                             8.0 * st["passes"] * len(source) * len(target) / max(st["launches"], 1)
                             / (avg_ms * 1e-3) / 1e12, 1) if avg_ms > 0 else None},
            "cpu_baseline": cpu,
            "parity_vs_oracle": parity,
            "setup_inclusive": setup,
            "fast_mode": fast,
            "gicp_iterations": int(iters),
            "align": align_s,
            "c4": c4,
        }
        fixture_iters = align_s.pop("_fixture_iterations", 0) if align_s is not None else 0
        if align_s is not None and cpu is not None and cpu.get("seconds_per_iteration"):
            # the CPU align() on THIS host: the oracle's measured seconds per GICP iteration (the step-0
            # sample above, per-call set-up included) times the complete align()'s iterations (fixture)
            est = cpu["seconds_per_iteration"] * fixture_iters
            if est > 0:
                align_s["cpu_seconds_same_host_extrapolated"] = round(est, 1)
                align_s["speedup_vs_cpu_same_host"] = round(est / align_s["seconds"], 1)
        if cpu is not None:
            cpu["seconds_per_iteration"] = round(cpu["seconds_per_iteration"], 6)
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


def setup_inclusive_run(ctx, step, args):
    """The timed steps again with both clouds re-uploaded before every step
    (host float64 -> HBM, Morton layout, tile boxes, KNN-20 covariances): the
    rate a caller sees when every multistart brings new clouds.  `value`
    keeps the clouds resident, as the Aligner does within one align()."""
    k = max(1, args.steps // 2)
    t0 = time.perf_counter()
    iters = 0
    for j in range(k):
        ctx._target_key = ctx._source_key = None  # forget the content-hash cache: upload again
        iters += step(args.warmup + j)
    el = time.perf_counter() - t0
    return {"value": round(iters / el, 3), "unit": "GICP iterations/s", "ms_per_step": round(el / k * 1e3, 3),
            "steps": k, "note": "source and target uploaded, laid out and covariances recomputed every step"}


def fast_mode_run(source, target, args, device, oracle_rmse, oracle_iters):
    """The same steps with GeneralizedICP(exact_nn=False): the fp32 search's
    answer (near-ties within 2^-17 relative resolved by Morton position, not
    the KD-tree's fp64 order).  Its rate, and step 0's starts against the
    oracle (stated tolerance of this mode: converged RMSE within 1e-5)."""
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor

    opt = GeneralizedICP(device=device, exact_nn=False)
    al = Aligner(Preprocessor([]), Preprocessor([]), opt, attempts=args.attempts)
    np.random.seed(1000)
    al.multistart_registration(source, target)  # step 0 (warm-up and parity)
    r0 = np.array(al.history[-1]["rmse"])
    t0 = time.perf_counter()
    iters = 0
    for k in range(args.steps):
        np.random.seed(1000 + args.warmup + k)
        al.multistart_registration(source, target)
        iters += al.history[-1]["iters"]
    el = time.perf_counter() - t0
    out = {"value": round(iters / el, 3), "unit": "GICP iterations/s", "ms_per_step": round(el / args.steps * 1e3, 3),
           "steps": args.steps, "gicp_iterations": int(iters)}
    if oracle_rmse is not None and len(oracle_rmse):
        n = len(oracle_rmse)
        d = np.abs(r0[:n] - oracle_rmse)
        out["parity_vs_oracle"] = {"starts": int(n), "max_abs_d_rmse": float(d.max()),
                                   "within_1e-5": int((d <= 1e-5).sum())}
    GeneralizedICP(device=device).context  # the shared context back in the default (exact) mode
    return out


def align_vs_fixture(T, metric, sf, errors, gpu_seconds):
    """The GPU align() against the committed COMPLETE CPU-oracle align() at C2
    (tests/golden/g7_align_c2.npz, made by tests/golden/make_golden_align.py:
    every optimize call on the oracle, same inputs and RNG stream)."""
    path = os.path.join(REPO, "tests", "golden", "g7_align_c2.npz")
    if not os.path.exists(path):
        return {"parity_vs_oracle": None}
    z = np.load(path)
    meta = json.load(open(path.replace(".npz", ".json")))
    e = np.asarray(errors, dtype=np.float64)
    out = {"parity_vs_oracle": {
        "scale_factors_identical": bool(np.array_equal(np.asarray(sf).reshape(1, 3), z["sf"])),
        "d_rmse": abs(float(metric) - float(z["metric"])), "max_abs_dT": float(np.abs(np.asarray(T) - z["T"]).max()),
        "compass_errors_max_abs_diff": float(np.abs(e - z["errors"]).max()) if len(e) == len(z["errors"]) else None,
        "oracle_rmse": float(z["metric"]), "fixture": "tests/golden/g7_align_c2.npz"},
        "_fixture_iterations": int(z["call_iters"].sum())}
    return out


def c4_run(opt, src_raw, tgt_raw, args, barrier, dist):
    """C4 (BASELINE.json configs[3], the north_star's strong-scaling case): one
    complete Aligner.align() (Aligner.py:228-317, refine off) on the C2 pair
    with --c4-attempts (64) starts per multistart, the starts of every device
    batch sharded over the N ranks (one all-gather per batch).  The total work
    is the same at every N, so T1 / TN is the strong-scaling speedup.  One
    cold run (device buffers grown), then the timed run; the wall-clock is the
    max over ranks between barriers.  The result is checked against the
    committed complete-oracle C4 align() (tests/golden/g7_align_c4.npz)
    when present."""
    from orpcd_amd import Aligner, Preprocessor

    world = dist.get_world_size() if dist is not None else 1
    out = None
    for timed in (False, True):
        np.random.seed(0)
        al = Aligner(Preprocessor([]), Preprocessor([]), opt, attempts=args.c4_attempts)
        barrier()
        t0 = time.perf_counter()
        T, metric, sf, errors = al.align(src_raw, tgt_raw, refine_registration=False)
        barrier()
        el = time.perf_counter() - t0
        if timed:
            mine = el
            if dist is not None:
                import torch
                dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
                t = torch.tensor([el], dtype=torch.float64, device=dev)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                el = float(t.item())
            iters = int(sum(h["iters"] for h in al.history))
            spec = int(sum(h["iters"] for h in al.speculative_history))
            out = {"workload": f"C4: Aligner.align() on the C2 pair, {args.c4_attempts} starts per multistart, "
                               f"starts sharded over {world} GPU(s) (strong scaling)",
                   "seconds": round(el, 4), "seconds_rank0": round(mine, 4), "n_gpus": world,
                   "attempts": args.c4_attempts, "multistarts": len(al.history),
                   "gicp_iterations": iters, "gicp_iterations_per_s": round(iters / el, 1),
                   "speculative_gicp_iterations": spec,
                   "rmse": float(metric), "scale_factors": [float(x) for x in np.asarray(sf).ravel()]}
            path = os.path.join(REPO, "tests", "golden", "g7_align_c4.npz")
            if os.path.exists(path):
                z = np.load(path)
                e = np.asarray(errors, dtype=np.float64)
                rmse = np.concatenate([h["rmse"] for h in al.history])
                its = np.concatenate([h["iters_per_start"] for h in al.history])
                same = len(rmse) == len(z["call_rmse"])
                out["parity_vs_oracle"] = {
                    "fixture": "tests/golden/g7_align_c4.npz",
                    "scale_factors_identical": bool(np.array_equal(np.asarray(sf).reshape(1, 3), z["sf"])),
                    "d_rmse": abs(float(metric) - float(z["metric"])),
                    "max_abs_dT": float(np.abs(np.asarray(T) - z["T"]).max()),
                    "compass_errors_identical_count": bool(len(e) == len(z["errors"])),
                    "starts": int(len(rmse)), "starts_oracle": int(len(z["call_rmse"])),
                    "iterations_identical": int((its == z["call_iters"]).sum()) if same else None,
                    "max_abs_d_rmse_per_start": float(np.abs(rmse - z["call_rmse"]).max()) if same else None}
    return out


def pmc_counter(kernel, exact, counter):
    """Per-launch value of an SQ counter for `kernel` from the newest committed
    profiles/rNN_pmc.json (rocprofv3 --pmc on this same bench command)."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc.json")))
    if not files:
        return None
    d = json.load(open(files[-1]))
    inst = kernel + ("<true" if exact else "<false")
    key = kernel if kernel in d else next((k for k in sorted(d) if k.startswith(inst)), None)
    return None if key is None else d[key].get(counter)


def pmc_stalls(kernel, exact):
    """Wave-cycle breakdown of `kernel` per launch from the newest committed
    SQ counters (profiles/rNN_pmc.json) and the same round's kernel-trace
    average duration (rNN_kernel_stats.csv): SQ_WAIT_ANY (parked: s_waitcnt on
    memory / barrier), SQ_WAIT_INST_ANY (issue stalls: dependencies, pipe
    busy), the rest (issuing), all over SQ_WAVE_CYCLES (quad-cycles,
    MI355X_MICROARCH.md §rocprofv3 PMC slots), and the average resident waves
    = wave-cycles / (launch duration x clock) against the 5120 slots the
    kernel's register budget allows.  The clock is GRBM_GUI_ACTIVE / 8 / the
    launch time when that counter was collected, else 2.4 GHz."""
    import csv
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc.json")))
    if not files:
        return None
    d = json.load(open(files[-1]))
    inst = kernel + ("<true" if exact else "<false")
    key = kernel if kernel in d else next((k for k in sorted(d) if k.startswith(inst)), None)
    if key is None or "SQ_WAVE_CYCLES" not in d[key]:
        return None
    c = d[key]
    rnd = os.path.basename(files[-1]).split("_")[0]
    avg_ns = None
    ks = os.path.join(REPO, "profiles", f"{rnd}_kernel_stats.csv")
    if os.path.exists(ks):
        for r in csv.DictReader(open(ks)):
            if r["Name"].replace("void ", "").startswith(inst):
                avg_ns = float(r["AverageNs"])
    wc = c["SQ_WAVE_CYCLES"]
    out = {"source": f"{os.path.basename(files[-1])} + {rnd}_kernel_stats.csv",
           "wait_any_frac": round(c.get("SQ_WAIT_ANY", 0) / wc, 3),
           "wait_inst_any_frac": round(c.get("SQ_WAIT_INST_ANY", 0) / wc, 3)}
    if "SQ_ACTIVE_INST_ANY" in c:
        out["active_inst_any_frac"] = round(c["SQ_ACTIVE_INST_ANY"] / wc, 3)
    out["waves_per_launch"] = round(c.get("SQ_WAVES", 0))
    if avg_ns:
        ghz = c["GRBM_GUI_ACTIVE"] / 8 / avg_ns if "GRBM_GUI_ACTIVE" in c else 2.4
        res = wc * 4 / (avg_ns * ghz)
        out.update(avg_launch_us_profiled=round(avg_ns / 1e3, 2), clock_ghz=round(ghz, 3),
                   avg_resident_waves=round(res), resident_frac_of_slots=round(res / WAVE_SLOTS, 3),
                   avg_wave_us=round(wc * 4 / max(c.get("SQ_WAVES", 1), 1) / ghz / 1e3, 2))
    return out


def pmc_traffic(kernel, exact=True):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/rNN_hbm.json: FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md
    §HBM), collected by rocprofv3 --pmc on this same bench command."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_hbm.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    # the instantiation of the templated search kernel that ran: "name<true>" (exact_nn) or "name<false>"
    inst = kernel + ("<true" if exact else "<false")
    key = kernel if kernel in d else next((k for k in sorted(d) if k.startswith(inst)), None)
    if key is None:
        return None, None
    return d[key]["hbm_bytes_per_launch_corrected"], os.path.basename(files[-1])


def cpu_baseline(source, target, args):
    """The oracle (C++/OpenMP, KD-tree 1-NN, fp64) on the same starts as step 0,
    attempt by attempt until the time budget is spent."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O

    cores, how = usable_cpus()  # the host cores this process may run on (all of them)
    O.set_num_threads(cores)
    np.random.seed(1000)
    al = O.OracleAligner(None, attempts=args.attempts)
    starts = [al.initialize_rotation() for _ in range(args.attempts)]
    t0 = time.perf_counter()
    iters = 0
    done = 0
    oracle_rmse, oracle_iters = [], []
    for R0, t0_ in starts:
        r = O.gicp(np.dot(source, R0) + t0_, target, 0.5, 100)
        iters += r["iters"]
        oracle_rmse.append(float(r["rmse"]))
        oracle_iters.append(int(r["iters"]))
        done += 1
        if time.perf_counter() - t0 > args.cpu_seconds:
            break
    el = time.perf_counter() - t0
    return {"oracle_rmse": oracle_rmse, "oracle_iters": oracle_iters, "value": round(iters / el, 3),
            "unit": "GICP iterations/s", "seconds_per_iteration": el / max(iters, 1),
            "cores": O.num_threads(),
            "cpu_model": cpu_model(),
            "kind": "port",
            "sample": f"{done} of {args.attempts} starts of step 0 (same R0,t0), {iters} GICP iterations, "
                      f"{el:.1f} s; OpenMP threads = the {cores} cpus this process may use ({how}; "
                      f"{os.cpu_count()} host cpus visible)"}


def usable_cpus():
    """CPUs this process can actually run on: its affinity mask, capped by the
    cgroup CPU quota (a container granted 16 of 256 cpus sees all 256 in its
    mask; 256 OpenMP threads on a 16-cpu quota run ~50x slower than 16)."""
    n = len(os.sched_getaffinity(0))
    how = f"affinity mask {n}"
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            q = max(1, -(-int(quota) // int(period)))
            if q < n:
                n, how = q, how + f", cgroup cpu quota {q}"
    except (OSError, ValueError):
        pass
    return n, how


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


if __name__ == "__main__":
    main()
