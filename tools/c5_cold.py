"""Where C5's cold set-up goes: the first orpcd_set_target
of a fresh process on the 1M-point target, split into context creation, the
first launches of the library's kernels (code objects; on a tiny cloud) and
the 1M-point allocations, against the warm call.

    python tools/c5_cold.py [--order tiny-first|direct] [--out FILE]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multi-scale-pointcloud-registration_amd"), REPO]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--order", choices=["tiny-first", "direct"], default="tiny-first")
    ap.add_argument("--points", type=int, default=1_000_000)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from orpcd_amd import _native
    from workloads import c5_pair, small_pair
    src, tgt = c5_pair(a.points)
    tiny_s, tiny_t = small_pair(1500, 1700, seed=0)
    out = {"order": a.order, "points": a.points,
           "lazy_code_objects": bool(os.environ.get("ORPCD_LAZY_CODE_OBJECTS"))}
    t0 = time.perf_counter()
    ctx = _native.Context(0)
    out["ctx_create_s"] = time.perf_counter() - t0
    if a.order == "tiny-first":
        t0 = time.perf_counter()
        ctx.set_target(tiny_t, 1e-3, cache=False)
        out["first_set_target_tiny_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        ctx.set_target(tiny_t, 1e-3, cache=False)
        out["second_set_target_tiny_s"] = time.perf_counter() - t0
    for k in range(3):
        t0 = time.perf_counter()
        ctx.set_target(tgt, 1e-3, cache=False)
        out[f"set_target_1M_{k}_s"] = time.perf_counter() - t0
    for k in range(2):
        t0 = time.perf_counter()
        ctx.set_source(src, cache=False)
        out[f"set_source_1M_{k}_s"] = time.perf_counter() - t0
    out = {k: (round(v, 5) if isinstance(v, float) else v) for k, v in out.items()}
    s = json.dumps(out)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
