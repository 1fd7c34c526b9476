"""Where a bench step's time goes by the number of running starts: from a
rocprofv3 kernel trace (csv) of bench.py, group the passes (one per
gicp_accum_kernel launch; its grid y = running starts) by running starts and
print, per group, passes, GICP iterations (= running starts), GPU time of each
kernel and wall time between consecutive passes.

    python tools/tail_profile.py gpurun_out/<dir>/<host>/<pid>_kernel_trace.csv
"""
import csv
import sys
from collections import defaultdict


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    acc = [i for i, r in enumerate(rows) if "gicp_accum_kernel" in r["Kernel_Name"]]
    bins = [(1, 1), (2, 4), (5, 8), (9, 16), (17, 30), (31, 10**9)]
    stat = defaultdict(lambda: defaultdict(float))
    for a, b in zip(acc, acc[1:]):
        wall = int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])
        if wall > 2e6:  # between batches
            continue
        nact = int(rows[a]["Grid_Size_Y"])
        # the pass that ends at accumulation b: its search (and re-search in exact mode) precede b
        seg_names = " ".join(r["Kernel_Name"] for r in rows[a:b + 1])
        mode = "exact" if "nn_exact_kernel" in seg_names or "<true>" in seg_names else "fast"
        key = mode + " " + next(f"{lo}-{hi}" for lo, hi in bins if lo <= nact <= hi)
        st = stat[key]
        st["passes"] += 1
        st["iters"] += nact
        st["wall_us"] += wall / 1e3
        for r in rows[a:b]:
            n = r["Kernel_Name"].split("(")[0].replace("void ", "").split("::")[-1][:24]
            st[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for mode in ("exact", "fast"):
        w = sum(s["wall_us"] for k, s in stat.items() if k.startswith(mode))
        it = sum(s["iters"] for k, s in stat.items() if k.startswith(mode))
        if it:
            print(f"{mode}: wall {w / 1e3:.2f} ms over {it:.0f} iterations: {1e3 * it / w:.0f} iterations/s of GPU passes")
    tot_wall = sum(s["wall_us"] for s in stat.values())
    for key, _ in sorted(stat.items(), key=lambda kv: (kv[0].split()[0], int(kv[0].split()[1].split("-")[0]))):
        s = stat[key]
        ks = "  ".join(f"{k}={v / s['passes']:.1f}" for k, v in s.items() if k not in ("passes", "iters", "wall_us"))
        print(f"{key:>13s}: passes {s['passes']:5.0f} iters {s['iters']:6.0f} wall {s['wall_us'] / 1e3:7.2f} ms "
              f"({100 * s['wall_us'] / tot_wall:4.1f}%)  us/pass {s['wall_us'] / s['passes']:6.1f}  "
              f"us/iter {s['wall_us'] / s['iters']:6.1f} | per pass: {ks}")


if __name__ == "__main__":
    main()
