"""Build liborpcd_hip.so for gfx950 in-tree (hipcc, no cmake/ninja).

    python multi-scale-pointcloud-registration_amd/build_native.py [--force]

Each csrc/*.hip unit is compiled to an object (incremental on mtime of the
unit and every header), then linked into orpcd_amd/_lib/liborpcd_hip.so.
The .so is git-ignored but travels to the GPU box with the snapshot.
"""
from __future__ import annotations

import glob
import hashlib
import json
import os
import subprocess
import sys
import time
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


def source_id() -> str:
    """sha256 (first 16 hex) over every source the library is built from
    (csrc/*.hip, csrc/*.h, include/*.h, by name and content).  The library
    embeds it (orpcd_build_id) and orpcd_amd._native refuses a library whose
    id differs from the sources beside it: a stale prebuilt .so fails loudly."""
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h"))
                   + glob.glob(os.path.join(REPO, "include", "*.h")))
    for f in files:
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def _build_id_object(force):
    """A one-function host unit returning the source id and the extra flags."""
    sid = source_id()
    flags = json.dumps(" ".join(EXTRA))  # a C string literal: quotes and backslashes escaped
    src = os.path.join(OBJ_DIR, "build_id.cpp")
    text = (f'extern "C" const char* orpcd_build_id(void) {{ return "{sid}"; }}\n'
            f'extern "C" const char* orpcd_build_flags(void) {{ return {flags}; }}\n')
    old = open(src).read() if os.path.exists(src) else None
    if old != text:
        with open(src, "w") as fh:
            fh.write(text)
    obj = src + ".o"
    if force or _stale(obj, [src]):
        r = subprocess.run([HIPCC, "-O2", "-fPIC", "-c", "-x", "c++", src, "-o", obj], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on build_id.cpp:\n{r.stdout}\n{r.stderr}")
    return obj


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


# instrumented variants (ORPCD_EXTRA_FLAGS) keep objects of their own per flag set
OBJ_DIR = OBJ + ("_" + "".join(c if c.isalnum() else "_" for c in "".join(EXTRA)) if EXTRA else "")


def _compile(src, force):
    """(object path, whether it was compiled now)"""
    obj = os.path.join(OBJ_DIR, os.path.basename(src) + ".o")
    if force or _stale(obj, [src] + _headers()):
        cmd = [HIPCC] + CXXFLAGS + ["-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stdout}\n{r.stderr}")
        return obj, True
    return obj, False


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile what is stale, relink if needed.  Every call records what it
    did (units recompiled, relinked or not, source id, seconds) in
    build/last_build.json and, with verbose, prints it: the build is observed,
    not assumed."""
    t0 = time.perf_counter()
    os.makedirs(OBJ_DIR, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        res = list(ex.map(lambda s: _compile(s, force), srcs))
    objs = [o for o, _ in res]
    objs.append(_build_id_object(force))
    linked = force or _stale(LIB, objs)
    if linked:
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-fPIC", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    rec = {"library": os.path.relpath(LIB, REPO), "source_id": source_id(), "extra_flags": " ".join(EXTRA),
           "units": len(srcs), "recompiled": [os.path.basename(s) for s, (_, c) in zip(srcs, res) if c],
           "relinked": bool(linked), "seconds": round(time.perf_counter() - t0, 1),
           "when": time.strftime("%Y-%m-%dT%H:%M:%S")}
    with open(os.path.join(OBJ_DIR, "last_build.json"), "w") as fh:
        json.dump(rec, fh, indent=1)
    if verbose:
        print(f"built {LIB}: {len(rec['recompiled'])} of {rec['units']} units recompiled "
              f"({', '.join(rec['recompiled']) or 'none'}), relinked: {'yes' if linked else 'no'}, "
              f"source id {rec['source_id']}, {rec['seconds']} s")
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
