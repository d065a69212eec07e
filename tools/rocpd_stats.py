"""Kernel statistics CSV (rocprofv3 --stats layout) from a rocprofv3 results
database (run_results.db), for runs made without --output-format csv.

    python tools/rocpd_stats.py gpurun_out/prof_v5/run_results.db > profiles/x_kernel_stats.csv
"""
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    cur = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels")
    print('"Name","Calls","TotalDurationNs","AverageNs","Percentage"')
    for name, calls, total, avg, pct in cur.fetchall():
        # the view reports microseconds
        print(f'"{name}",{calls},{total * 1000:.0f},{avg * 1000:.3f},{pct:.2f}')


if __name__ == "__main__":
    main(sys.argv[1])
