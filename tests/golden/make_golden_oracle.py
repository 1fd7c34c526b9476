"""Regression fixtures G4 / G5, produced by the CPU ORACLE
(oracle/, the Open3D 0.18 restatement) — they pin the restatement against
itself across rounds and give the GPU tests fixed expected values; they are
NOT outputs of Open3D (absent from this image: parity with it is unpinned).

    python tests/golden/make_golden_oracle.py

G4  GICP per-iteration trace (correspondence count, fitness, rmse) and final
    (T, rmse, iters) on (a) the 300 <-> 300 synthetic pair small_pair(300,
    seed=0) and (b) C1: ArmadilloBack_330 -> _0 after RadiusScaler +
    RandomDownsampler(5000) + SOR(64, 2) (np.random.seed(0); source then
    target, as Aligner.align preprocesses them), from identity.
G5  FPFH (Hybrid r=0.1, k=20) of a 2,000-point index-aligned synthetic pair and
    FGR on those features (seed 0): features, mutual-match / tuple counts, T.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "oracle"), REPO]


def c1_pair():
    import oracle as O
    from workloads import armadillo
    src, tgt = armadillo()
    np.random.seed(0)
    s = O.random_downsample(O.radius_scale(src)[0], 5000)
    s = s[O.sor(s, 64, 2)[0]]
    t = O.random_downsample(O.radius_scale(tgt)[0], 5000)
    t = t[O.sor(t, 64, 2)[0]]
    return s, t


def g5_pair():
    from workloads import bumpy_sphere, rot_xyz
    rng = np.random.default_rng(21)
    src = bumpy_sphere(2000, rng)
    tgt = src @ rot_xyz(0, 0, 15).T + np.array([0.02, -0.01, 0.03]) + rng.normal(0, 1e-4, size=src.shape)
    return src, tgt


def main():
    import oracle as O
    from workloads import small_pair
    out = {}
    for name, (s, t) in {"p300": small_pair(300, seed=0), "c1": c1_pair()}.items():
        r = O.gicp(s, t, 0.5, 100, trace=True)
        out[f"g4_{name}_T"] = r["T"]
        out[f"g4_{name}_rmse"] = np.array(r["rmse"])
        out[f"g4_{name}_iters"] = np.array(r["iters"])
        out[f"g4_{name}_trace_ncorr"] = r["trace_ncorr"]
        out[f"g4_{name}_trace_rmse"] = r["trace_rmse"]
    s, t = g5_pair()
    ns, fs = O.fpfh(s)
    nt, ft = O.fpfh(t)
    r = O.fgr(s, t, fs, ft, seed=0)
    out.update(g5_src_feat=fs, g5_tgt_feat=ft, g5_T=r["T"], g5_rmse=np.array(r["rmse"]),
               g5_n_mutual=np.array(r["n_mutual"]), g5_n_tuple=np.array(r["n_tuple_corr"]))
    np.savez_compressed(os.path.join(HERE, "g45_oracle.npz"), **out)
    print("wrote g45_oracle.npz", {k: np.shape(v) for k, v in out.items()})


if __name__ == "__main__":
    main()
