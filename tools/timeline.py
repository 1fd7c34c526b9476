"""Per-pass kernel timeline of the LAST batch in a rocprofv3 kernel-trace csv:
    python tools/timeline.py <kernel_trace.csv> [--every N]
Prints per pass the kernels' durations and the idle gap before each."""
import csv
import sys


def main():
    f = sys.argv[1]
    every = int(sys.argv[sys.argv.index("--every") + 1]) if "--every" in sys.argv else 1
    rows = list(csv.DictReader(open(f)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 r["Kernel_Name"].split("(")[0].split("::")[-1].replace("void ", "")[:16]) for r in rows)
    ks = [k for k in ks if "rocclr" not in k[2]]
    # the last batch: after the last gap > 200 us
    start = 0
    for i in range(1, len(ks)):
        if ks[i][0] - ks[i - 1][1] > 200_000:
            start = i
    ks = ks[start:]
    heads = [i for i, k in enumerate(ks) if k[2].startswith("nn_search")]
    tot = 0.0
    for p, (a, b) in enumerate(zip(heads, heads[1:] + [len(ks)])):
        seg = ks[a:b]
        wall = (ks[b][0] if b < len(ks) else seg[-1][1]) - seg[0][0]
        tot += wall
        if p % every == 0:
            s = "  ".join(f"{n}={(e - st) / 1e3:.1f}(+{(st - (seg[i - 1][1] if i else st)) / 1e3:.1f})"
                          for i, (st, e, n) in enumerate(seg))
            print(f"{p:3d} wall {wall / 1e3:6.1f}  {s}")
    print(f"passes {len(heads)}  total {tot / 1e3:.1f} us")


if __name__ == "__main__":
    main()
