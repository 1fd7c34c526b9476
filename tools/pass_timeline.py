"""Per-pass timeline of the last gicp_batch in a rocprofv3 kernel trace:
for every ICP pass, the duration of each kernel and the gaps between them.

    python tools/pass_timeline.py gpurun_out/kt/run_results.db [--every 10]
    python tools/pass_timeline.py gpurun_out/kt/<host>/<pid>_kernel_trace.csv [--every 10]

A pass starts at an xform_queries_kernel launch.  Prints, per pass, the
wall time from that launch to the next pass's, and the kernel durations
(us), so the fixed per-pass cost (launch latency, one-block kernels) can be
separated from the work that scales with the running starts.
"""
import sqlite3
import sys


def short(n):
    n = n.split("(")[0].replace("void ", "")
    return n.split("::")[-1][:22]


def main():
    every = int(sys.argv[sys.argv.index("--every") + 1]) if "--every" in sys.argv else 10
    if sys.argv[1].endswith(".csv"):  # rocprofv3 --output-format csv kernel trace
        import csv
        rows = sorted((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                      for r in csv.DictReader(open(sys.argv[1])))
        rows.sort(key=lambda r: r[1])
    else:
        db = sqlite3.connect(sys.argv[1])
        rows = db.execute("select name, start, end from kernels order by start").fetchall()
    starts = [i for i, r in enumerate(rows) if "xform_queries_kernel" in r[0]]
    # the last batch: passes after the last large gap (> 2 ms) between passes
    last = 0
    for a, b in zip(starts, starts[1:]):
        if rows[b][1] - rows[a][1] > 2e6:
            last = starts.index(b)
    passes = starts[last:]
    tot = {}
    print(f"{'pass':>4s} {'wall us':>8s}  kernels (us)")
    for p, (a, b) in enumerate(zip(passes, passes[1:] + [len(rows)])):
        seg = rows[a:b]
        wall = (rows[b][1] if b < len(rows) else seg[-1][2]) - seg[0][1]
        for n, s, e in seg:
            tot[short(n)] = tot.get(short(n), 0.0) + (e - s) / 1e3
        if p % every == 0 or b == len(rows):
            ks = "  ".join(f"{short(n)}={(e - s) / 1e3:.1f}" for n, s, e in seg)
            print(f"{p:4d} {wall / 1e3:8.1f}  {ks}")
    span = (rows[-1][2] - rows[passes[0]][1]) / 1e3
    print(f"passes {len(passes)}, span {span:.0f} us; kernel totals (us):",
          {k: round(v) for k, v in sorted(tot.items(), key=lambda x: -x[1])})


if __name__ == "__main__":
    main()
