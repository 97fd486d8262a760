"""Per-kernel summary (the rocprofv3 --stats table) from a rocprofv3 rocpd SQLite output.

Usage: python scripts/rocpd_stats.py RESULTS.db OUT.csv
rocprofv3 7.2 writes its default rocpd database (`-d DIR -o NAME` -> DIR/NAME_results.db); its `top_kernels`
view holds the same columns as the CSV kernel_stats summary (durations in microseconds here).
"""
import csv
import sqlite3
import sys


def main():
    db, out = sys.argv[1], sys.argv[2]
    con = sqlite3.connect(db)
    cur = con.execute("select name, total_calls, total_duration, average, percentage from top_kernels")
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
        for name, calls, tot, avg, pct in cur:
            w.writerow([name, calls, round(tot, 3), round(avg, 3), round(pct, 4)])
            print(f"{calls:6d} {avg:14.3f} us  {pct:6.2f}%  {name[:110]}")


if __name__ == "__main__":
    main()
