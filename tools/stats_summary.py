"""Per-kernel summary of rocprofv3 --stats CSVs:  python tools/stats_summary.py DIR... [top]"""
import csv
import glob
import sys


def main():
    dirs = [a for a in sys.argv[1:] if not a.isdigit()]
    top = int(next((a for a in sys.argv[1:] if a.isdigit()), 6))
    for d in dirs:
        f = sorted(glob.glob(f"{d}/**/*_kernel_stats.csv", recursive=True))
        if not f:
            print(d, "no stats")
            continue
        rows = list(csv.DictReader(open(f[-1])))
        print(f"== {d}")
        for x in rows[:top]:
            print(f"  {x['Name'][:58]:58s} {int(x['Calls']):6d} {float(x['TotalDurationNs']) / 1e6:8.2f} ms "
                  f"{float(x['AverageNs']) / 1e3:8.1f} us {float(x['Percentage']):5.1f}%")


if __name__ == "__main__":
    main()
