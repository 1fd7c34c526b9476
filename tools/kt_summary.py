"""Per-kernel call count and mean duration from a rocprofv3 --kernel-trace
rocpd database (the default output format): python tools/kt_summary.py DIR"""
import glob
import sqlite3
import sys

for d in sys.argv[1:]:
    for db in glob.glob(f"{d}/**/*.db", recursive=True):
        rows = sqlite3.connect(db).execute(
            "select name, count(*), avg(duration), sum(duration) from kernels group by name "
            "order by sum(duration) desc limit 8").fetchall()
        print(d)
        for name, n, avg, tot in rows:
            print(f"  {n:6d} x {avg / 1e3:9.2f} us  total {tot / 1e6:8.2f} ms  {str(name)[:70]}")
