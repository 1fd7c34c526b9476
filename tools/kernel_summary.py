"""Print a per-kernel summary (calls, total ms, avg us) from a rocprofv3
results database (rocpd SQLite, the default output of `rocprofv3 -d DIR -o NAME`).

    python tools/kernel_summary.py gpurun_out/prof/run_results.db [N]
"""
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
    rows = db.execute("select name, count(*), sum(end-start)/1e6, avg(end-start)/1e3 from kernels "
                      "group by name order by 3 desc").fetchall()
    total = sum(r[2] for r in rows)
    print(f"{'kernel':72s} {'calls':>7s} {'total ms':>10s} {'avg us':>9s} {'%':>6s}")
    for name, calls, ms, avg in rows[:top]:
        print(f"{name[:72]:72s} {calls:7d} {ms:10.2f} {avg:9.1f} {100 * ms / total:6.1f}")
    print(f"{'total':72s} {'':7s} {total:10.2f}")


if __name__ == "__main__":
    main()
