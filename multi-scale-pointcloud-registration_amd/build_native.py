"""Build liborpcd_hip.so for gfx950 in-tree (hipcc, no cmake/ninja).

    python multi-scale-pointcloud-registration_amd/build_native.py [--force]

Each csrc/*.hip unit is compiled to an object (incremental on mtime of the
unit and every header), then linked into orpcd_amd/_lib/liborpcd_hip.so.
The .so is git-ignored but travels to the GPU box with the snapshot.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build", "obj")
LIBDIR = os.path.join(HERE, "orpcd_amd", "_lib")
LIB = os.environ.get("ORPCD_BUILD_LIB", os.path.join(LIBDIR, "liborpcd_hip.so"))
EXTRA = os.environ.get("ORPCD_EXTRA_FLAGS", "").split()  # e.g. -DORPCD_PHASES (instrumented variant)
ARCH = os.environ.get("ORPCD_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXXFLAGS = EXTRA + ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
            "-munsafe-fp-atomics", f"-I{os.path.join(REPO, 'include')}", f"-I{CSRC}"]


def _headers():
    return glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(REPO, "include", "*.h"))


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


# instrumented variants (ORPCD_EXTRA_FLAGS) keep objects of their own per flag set
OBJ_DIR = OBJ + ("_" + "".join(c if c.isalnum() else "_" for c in "".join(EXTRA)) if EXTRA else "")


def _compile(src, force):
    obj = os.path.join(OBJ_DIR, os.path.basename(src) + ".o")
    if force or _stale(obj, [src] + _headers()):
        cmd = [HIPCC] + CXXFLAGS + ["-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OBJ_DIR, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    if force or _stale(LIB, objs):
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-fPIC", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    if verbose:
        print("built", LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
