"""Per-launch counters of the search kernels from tools/pmc_waves.sh runs.

    python tools/pmc_compare.py OUTDIR name:lib ...  -> JSON on stdout
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_profile import counters, newest_run, short  # noqa: E402


def main():
    out_dir, variants = sys.argv[1], [v.split(":")[0] for v in sys.argv[2:]]
    res = {}
    for n in variants:
        d = {}
        st = newest_run(glob.glob(os.path.join(out_dir, n, "kt", "**", "*kernel_stats.csv"), recursive=True))
        for r in csv.DictReader(open(st[0])) if st else []:
            k = short(r["Name"])
            if "nn_search" in k or "accum" in k or "solve" in k or "xform" in k:
                d.setdefault(k, {}).update(calls=int(r["Calls"]), avg_us=round(float(r["AverageNs"]) / 1e3, 2))
        for sub in ("tcc", "tcp"):
            for (k, c), (cnt, s) in counters(os.path.join(out_dir, n, sub)).items():
                if k in d:
                    d[k][c] = s / cnt
        for k, v in d.items():
            if "TCC_EA0_RDREQ_sum" in v:
                # FETCH_SIZE = RDREQ x 64 B; x2 for wide coalesced reads (MI355X_MICROARCH.md §HBM)
                v["fetch_size_MB_per_launch"] = round(v["TCC_EA0_RDREQ_sum"] * 64 / 1e6, 2)
            if "TCC_HIT_sum" in v and "TCC_MISS_sum" in v:
                v["l2_hit_rate"] = round(v["TCC_HIT_sum"] / max(v["TCC_HIT_sum"] + v["TCC_MISS_sum"], 1), 4)
        res[n] = d
    json.dump(res, sys.stdout, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
