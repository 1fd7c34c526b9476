"""Golden fixtures for the FarthestDownsampler (G6), produced by the
REFERENCE class itself (farthestDownsampler.py:26-54 — numpy + scipy cdist,
no open3d).  Run in the build container (reads /root/reference):

    python tests/golden/make_golden_fps.py

Cases (inputs regenerated from the stored seeds / shapes by the tests):
  rand   3,000 N(0,1) points (default_rng(11)), sample 257, np.random.seed(5)
  grid   integer lattice 12x10x8 (exact distance ties), sample 200, seed 6
  dup    600 points drawn with replacement from 150 (duplicates), sample 150,
         seed 7
  arm    ArmadilloBack_0 RadiusScaler-normalised (tests/golden/armadillo.npz),
         sample 512, seed 8
The fixture stores the chosen points (the reference returns cloud[index_list])
and the first index drawn from np.random.
"""
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = "/root/reference/src"
sys.path.insert(0, HERE)


def cases():
    rng = np.random.default_rng(11)
    rand = rng.normal(size=(3000, 3))
    g = np.stack(np.meshgrid(np.arange(12.0), np.arange(10.0), np.arange(8.0), indexing="ij"), -1).reshape(-1, 3)
    base = np.random.default_rng(12).normal(size=(150, 3))
    dup = base[np.random.default_rng(13).integers(0, 150, size=600)]
    z = np.load(os.path.join(HERE, "armadillo.npz"))
    a = z["ArmadilloBack_0"].astype(np.float64)
    c = a.mean(axis=0)
    arm = (a - c) / np.max(np.linalg.norm(a - c, axis=1))
    return {"rand": (rand, 257, 5), "grid": (g, 200, 6), "dup": (dup, 150, 7), "arm": (arm, 512, 8)}


def main():
    from make_golden import _name_only_open3d
    work = tempfile.mkdtemp(prefix="orpcd_golden_")
    os.makedirs(os.path.join(work, "cwd"))
    os.chdir(os.path.join(work, "cwd"))
    _name_only_open3d()
    sys.path.insert(0, REF_SRC)
    import logging
    logging.disable(logging.CRITICAL)
    from or_pcd.Preprocessor.Downsamplers.farthestDownsampler import FarthestDownsampler
    out = {}
    for name, (cloud, k, seed) in cases().items():
        np.random.seed(seed)
        first = np.random.randint(low=0, high=cloud.shape[0])
        np.random.seed(seed)
        pts = FarthestDownsampler(sample_size=k).process(cloud)
        out[name + "_points"] = pts
        out[name + "_first"] = np.array(first)
        out[name + "_after"] = np.array(np.random.random())  # RNG position after process()
    np.savez_compressed(os.path.join(HERE, "g6_fps.npz"), **out)
    print("wrote g6_fps.npz:", {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
