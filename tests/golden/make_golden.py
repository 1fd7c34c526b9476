"""Generate the committed golden fixtures under tests/golden/.

Run in the build container (NOT on the GPU box — it reads /root/reference):

    python tests/golden/make_golden.py

What it pins:
  G1  RNG replay: Aligner.initialize_rotation (Aligner.py:125-162) x64 for
      seeds {0, 1, 42}, drawn by the REFERENCE class.
  G2  RadiusScaler (+auto-insert, preprocessor.py:19-23) + RandomDownsampler
      (randomDownsampler.py:35-37) on ArmadilloBack_330 / _0, seed 0,
      run by the REFERENCE classes.
  G3  Aligner.align control flow (Aligner.py:228-317, refine off) driven by a
      deterministic scripted IOptimizer, run by the REFERENCE Aligner.
  DATA the two Armadillo scans the configs use, parsed from the reference's
      sample PLYs (binary big-endian float x,y,z) into float32 .npz — input
      data for C1/C2 (the GPU box has no /root/reference).

The reference imports `open3d` at module scope; open3d is absent here, so a
module exposing only the attribute NAMES the imports touch is placed in
sys.modules.  No computation is attributed to it: every fixture below comes
from code paths of the reference that never call open3d.
"""
import json
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = "/root/reference/src"
REF_DATA = "/root/reference/data"


def _name_only_open3d():
    o3d = types.ModuleType("open3d")
    o3d.geometry = types.SimpleNamespace(PointCloud=object, KDTreeSearchParamHybrid=object)
    o3d.pipelines = types.SimpleNamespace(
        registration=types.SimpleNamespace(Feature=object, RegistrationResult=object))
    o3d.utility = types.SimpleNamespace(Vector3dVector=list)
    sys.modules["open3d"] = o3d


def read_ply_xyz(path):
    """Binary big-endian PLY with a leading `vertex` element of float x,y,z."""
    raw = open(path, "rb").read()
    end = raw.index(b"end_header\n") + len(b"end_header\n")
    header = raw[:end].decode("ascii").splitlines()
    assert "format binary_big_endian 1.0" in header
    nv = int([h for h in header if h.startswith("element vertex")][0].split()[-1])
    props = []
    for h in header[header.index(f"element vertex {nv}") + 1:]:
        if not h.startswith("property"):
            break
        props.append(h.split()[-1])
    assert props == ["x", "y", "z"], props
    return np.frombuffer(raw, dtype=">f4", count=nv * 3, offset=end).reshape(nv, 3).astype(np.float32)


def main():
    work = tempfile.mkdtemp(prefix="orpcd_golden_")
    os.makedirs(os.path.join(work, "cwd"))
    os.chdir(os.path.join(work, "cwd"))  # reference loggers write to <cwd>/../logs
    _name_only_open3d()
    sys.path.insert(0, REF_SRC)
    sys.path.insert(0, HERE)
    from or_pcd.Aligner.Aligner import Aligner
    from or_pcd.Preprocessor.preprocessor import Preprocessor
    from or_pcd.Preprocessor.Downsamplers.randomDownsampler import RandomDownsampler
    from scripted import ScriptedOptimizer
    import logging
    logging.disable(logging.CRITICAL)

    # ---------------------------------------------------------------- DATA
    clouds = {}
    for name in ("ArmadilloBack_330", "ArmadilloBack_0"):
        clouds[name] = read_ply_xyz(os.path.join(REF_DATA, name + ".ply"))
    np.savez_compressed(os.path.join(HERE, "armadillo.npz"), **clouds)

    # ---------------------------------------------------------------- G1
    g1 = {}
    for seed in (0, 1, 42):
        np.random.seed(seed)
        al = Aligner(Preprocessor([]), Preprocessor([]), ScriptedOptimizer([1, 1, 1]))
        Rs, ts = [], []
        for _ in range(64):
            R, t = al.initialize_rotation()
            Rs.append(R)
            ts.append(t)
        g1[f"R_{seed}"] = np.array(Rs)
        g1[f"t_{seed}"] = np.array(ts)
    np.savez_compressed(os.path.join(HERE, "g1_rng.npz"), **g1)

    # ---------------------------------------------------------------- G2
    g2 = {}
    for name, cloud in clouds.items():
        np.random.seed(0)
        pp = Preprocessor([RandomDownsampler(5000)])
        out = pp.preprocess(cloud.astype(np.float64))
        scaler = pp.preprocessor_blocks[0]
        g2[f"{name}_out"] = out
        g2[f"{name}_mean"] = np.asarray(scaler.mean)
        g2[f"{name}_scale"] = np.asarray(scaler.scale)
    np.savez_compressed(os.path.join(HERE, "g2_preprocess.npz"), **g2)

    # ---------------------------------------------------------------- G3
    rng = np.random.default_rng(123)
    src = rng.normal(size=(60, 3)) * np.array([1.0, 0.7, 0.4])
    tgt = rng.normal(size=(50, 3)) * np.array([0.9, 0.8, 0.5])
    tgt_pre = (tgt - tgt.mean(0, keepdims=True))
    tgt_pre = tgt_pre / np.max(np.linalg.norm(tgt_pre, axis=1))
    goal = np.abs(tgt_pre).mean(0) * np.array([1.2, 0.8, 1.05])
    g3 = {"src": src, "tgt": tgt, "goal": goal}
    meta = {}
    for mode, attempts, seed in (("scripted", 4, 7), ("never_improves", 30, 0), ("constant", 2, 3)):
        np.random.seed(seed)
        opt = ScriptedOptimizer(goal, mode=mode)
        al = Aligner(Preprocessor([]), Preprocessor([]), opt, attempts=attempts)
        T, metric, sf, errors = al.align(src.copy(), tgt.copy(), refine_registration=False)
        g3[f"{mode}_T"] = T
        g3[f"{mode}_metric"] = np.asarray(metric)
        g3[f"{mode}_sf"] = sf
        g3[f"{mode}_errors"] = np.asarray(errors)
        g3[f"{mode}_call_a"] = np.array([c[0] for c in opt.calls])
        g3[f"{mode}_call_s0"] = np.array([c[1] for c in opt.calls])
        g3[f"{mode}_call_rmse"] = np.array([c[2] for c in opt.calls])
        g3[f"{mode}_rng_after"] = np.random.uniform(size=4)
        g3[f"{mode}_delta_after"] = np.asarray(al._delta)
        meta[mode] = dict(attempts=attempts, seed=seed, n_calls=len(opt.calls))
    np.savez_compressed(os.path.join(HERE, "g3_aligner_trace.npz"), **g3)
    with open(os.path.join(HERE, "g3_meta.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("golden fixtures written:", meta)


if __name__ == "__main__":
    main()
