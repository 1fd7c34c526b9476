"""Summarise rocprofv3 CSV output into profiles/ (committed evidence).

    python tools/summarize_profile.py --round r01 --kt DIR [--fetch DIR] [--write DIR] [--pmc DIR ...] [--out-dir D]

Writes profiles/<round>_kernel_stats.csv (rocprofv3 --kernel-trace --stats),
profiles/<round>_hbm.json (per-kernel FETCH_SIZE / WRITE_SIZE per launch with
the gfx950 correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE counts half of
the bytes of wide (16 B/lane) coalesced reads -> x2; WRITE_SIZE exact for
16 B/lane stores) and profiles/<round>_profile.md (a readable table).
"""
import argparse
import csv
import glob
import json
import os
import shutil

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


def newest_run(paths):
    """The files of the newest rocprofv3 run among `paths` (gpurun merges each
    call's outputs into the same local directory, so older runs accumulate):
    the run is the file name's process-id prefix."""
    if not paths:
        return []
    runs = {}
    for p in paths:
        runs.setdefault(os.path.basename(p).split("_")[0], []).append(p)
    last = max(runs, key=lambda r: max(os.path.getmtime(p) for p in runs[r]))
    return runs[last]


def counters(d):
    out = {}
    for path in newest_run(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(path)):
            k = (short(r["Kernel_Name"]), r["Counter_Name"])
            n, s = out.get(k, (0, 0.0))
            out[k] = (n + 1, s + float(r["Counter_Value"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", required=True)
    ap.add_argument("--kt", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--pmc", nargs="*", default=[])
    ap.add_argument("--out-dir", default=os.path.join(REPO, "profiles"),
                    help="where the summaries go (on the GPU box: under gpurun_out/, so they come back)")
    a = ap.parse_args()
    prof = a.out_dir
    os.makedirs(prof, exist_ok=True)
    stats = newest_run(glob.glob(os.path.join(a.kt, "**", "*kernel_stats.csv"), recursive=True))[0]
    shutil.copy(stats, os.path.join(prof, f"{a.round}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    hbm = {}
    if a.fetch and a.write:
        f, w = counters(a.fetch), counters(a.write)
        for (k, c), (n, s) in f.items():
            if c != "FETCH_SIZE":
                continue
            wn, ws = w.get((k, "WRITE_SIZE"), (1, 0.0))
            fk, wk = s / n, ws / max(wn, 1)
            hbm[k] = {"launches": n, "FETCH_SIZE_KB": round(fk, 1), "WRITE_SIZE_KB": round(wk, 1),
                      "hbm_bytes_per_launch_corrected": int((2 * fk + wk) * 1024)}
        json.dump(hbm, open(os.path.join(prof, f"{a.round}_hbm.json"), "w"), indent=1, sort_keys=True)
    extra = {}
    for d in a.pmc:
        for (k, c), (n, s) in counters(d).items():
            extra.setdefault(k, {})[c] = s / n
    if extra:
        json.dump(extra, open(os.path.join(prof, f"{a.round}_pmc.json"), "w"), indent=1, sort_keys=True)
    with open(os.path.join(prof, f"{a.round}_profile.md"), "w") as fh:
        fh.write(f"# {a.round} rocprofv3 summary\n\n| kernel | calls | total ms | avg us | % | HBM MB/launch (corrected) |\n|---|---|---|---|---|---|\n")
        for r in rows:
            k = short(r["Name"])
            h = hbm.get(k, {}).get("hbm_bytes_per_launch_corrected")
            fh.write(f"| {k} | {r['Calls']} | {float(r['TotalDurationNs'])/1e6:.2f} | "
                     f"{float(r['AverageNs'])/1e3:.1f} | {float(r['Percentage']):.1f} | "
                     f"{'' if h is None else f'{h/1e6:.2f}'} |\n")
    print("wrote", prof)


if __name__ == "__main__":
    main()
