"""Measurement of the rows either side of the hot path on 1 GPU.

    python tools/bench_prep.py [--points 50000] [--repeat 5] [--cpu 1] [--out profiles/r01_prep.json]

Workloads (the C2 pair: Armadillo 330 -> 0 densified to 50k, RadiusScaler-
normalised, workloads.c2_pair):
  refine  Aligner.refine_registration(PointToPoint) from a perturbed pose
          (R(3,-2,4), t(0.01,0,-0.02)): registration_icp, <= 200 iterations;
  sor     SOR() (nb_neighbours 64, std_ratio 2) on the source;
  voxel   VoxelDownsampler(2000).process (compass search over the voxel size);
  fps     FarthestDownsampler(4096).process (the reference's default size).
GPU times: wall-clock of the plugin call with host inputs (as the reference's
callers hand them over), median of `repeat` after one warm-up.  CPU baseline:
the oracle restatement of the same call (C++/OpenMP for refine/sor/voxel; the
numpy restatement of farthestDownsampler.py for fps, i.e. the reference's own
algorithm), timed once on the host cores.  Every GPU result is checked
against the CPU result (identical / within the parity tolerances).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO, os.path.join(REPO, "oracle")]


def radius_scale(c):
    center = c.mean(axis=0, keepdims=True)
    return (c - center) / np.max(np.linalg.norm(c - center, axis=1))


def timed(fn, repeat):
    fn()
    ts = []
    out = None
    for _ in range(repeat):
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=50_000)
    ap.add_argument("--repeat", type=int, default=5)
    ap.add_argument("--cpu", type=int, default=1)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import oracle as O
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor
    from orpcd_amd.Preprocessor.Downsamplers import FarthestDownsampler, VoxelDownsampler
    from orpcd_amd.Preprocessor.Outliers import SOR
    from workloads import c2_pair, rot_xyz

    src_raw, tgt_raw = c2_pair(args.points)
    src, tgt = radius_scale(src_raw), radius_scale(tgt_raw)
    res = {"metric": "preprocessing + refinement wall-clock (C2 pair, 50k pts)", "unit": "ms", "n_gpus": 1,
           "higher_is_better": False, "data": "synthetic C2 (Armadillo 330->0 densified to 50k)",
           "cpu_cores": O.num_threads(), "rows": {}}

    # ---- refine (PointToPoint ICP)
    al = Aligner(Preprocessor([]), Preprocessor([]), GeneralizedICP(), attempts=1)
    T0 = np.eye(4)
    T0[:3, :3] = rot_xyz(3, -2, 4)
    T0[:3, 3] = [0.01, 0.0, -0.02]
    t, (T, rmse) = timed(lambda: al.refine_registration(src, tgt, T0, icp_type="PointToPoint"), args.repeat)
    row = {"gpu_ms": round(t * 1e3, 3), "iters": al.last_refine["iters"], "rmse": rmse}
    row["gpu_iters_per_s"] = round(al.last_refine["iters"] / t, 1)
    if args.cpu:
        t0 = time.perf_counter()
        o = O.icp_p2p(src, tgt, 0.5, T0, 200)
        tc = time.perf_counter() - t0
        row.update(cpu_ms=round(tc * 1e3, 1), cpu_iters=o["iters"], speedup=round(tc / t, 1),
                   max_abs_dT=float(np.abs(T - o["T"]).max()), d_rmse=abs(rmse - o["rmse"]))
    res["rows"]["refine_p2p"] = row

    # ---- SOR
    sor = SOR()
    t, kept = timed(lambda: sor.process(src), args.repeat)
    row = {"gpu_ms": round(t * 1e3, 3), "kept": len(kept)}
    if args.cpu:
        t0 = time.perf_counter()
        oi, _ = O.sor(src, 64, 2.0)
        tc = time.perf_counter() - t0
        row.update(cpu_ms=round(tc * 1e3, 1), speedup=round(tc / t, 1), identical=bool(np.array_equal(kept, src[oi])))
    res["rows"]["sor"] = row

    # ---- voxel compass
    def vox():
        v = VoxelDownsampler(2000)
        out = v.process(src)
        return out, v.voxel_size
    t, (vout, vsize) = timed(vox, args.repeat)
    row = {"gpu_ms": round(t * 1e3, 3), "voxel_size": vsize, "points": len(vout)}
    if args.cpu:
        t0 = time.perf_counter()
        cur, delta, metric = 0.01, 0.01, abs(2000 - O.voxel_down_sample(src, 0.01, True))
        best = cur
        while delta >= 0.0005:
            moved = False
            for d in (delta, -delta):
                v = cur + d if cur + d > 0.0001 else 0.0001
                m = abs(2000 - O.voxel_down_sample(src, v, True))
                if m < metric:
                    cur, metric, best, moved = v, m, v, True
                    break
            if not moved:
                delta /= 2
        ov = O.voxel_down_sample(src, best)
        tc = time.perf_counter() - t0
        row.update(cpu_ms=round(tc * 1e3, 1), speedup=round(tc / t, 1),
                   identical=bool(vsize == best and np.array_equal(vout, ov)))
    res["rows"]["voxel_compass"] = row

    # ---- FPS
    fps = FarthestDownsampler(4096)
    np.random.seed(0)
    t, pts = timed(lambda: fps.process(src), args.repeat)
    row = {"gpu_ms": round(t * 1e3, 3), "samples": 4096, "us_per_step": round(t / 4095 * 1e6, 2)}
    if args.cpu:
        np.random.seed(0)
        first = np.random.randint(0, len(src))
        np.random.seed(0)
        gp = fps.process(src)
        t0 = time.perf_counter()
        oi = O.farthest_downsample(src, 4096, first)
        tc = time.perf_counter() - t0
        row.update(cpu_ms=round(tc * 1e3, 1), cpu_kind="numpy restatement of farthestDownsampler.py (1 core)",
                   speedup=round(tc / t, 1), identical=bool(np.array_equal(gp, src[oi])))
    res["rows"]["fps"] = row

    line = json.dumps(res)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
