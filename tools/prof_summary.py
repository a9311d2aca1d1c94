"""Per-kernel summary (calls, total/avg duration, share) of a rocprofv3 --kernel-trace --stats run.

Reads either the ``*_kernel_stats.csv`` rocprofv3 writes with ``--output-format csv`` or the
``*_results.db`` (rocpd SQLite, its ``top_kernels`` view) and writes a CSV for profiles/.

Usage: python tools/prof_summary.py <run_results.db | run_kernel_stats.csv> <out.csv>
"""
import csv
import sqlite3
import sys


def rows_from_db(path):
    c = sqlite3.connect(path)
    # the top_kernels view reports microseconds
    return [(r[0], int(r[1]), float(r[2]) * 1e3, float(r[3]) * 1e3, float(r[4]))
            for r in c.execute("select name, total_calls, total_duration, average, percentage from top_kernels")]


def rows_from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]),
                        float(r["Percentage"])))
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    rows = rows_from_db(src) if src.endswith(".db") else rows_from_csv(src)
    rows.sort(key=lambda r: -r[2])
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
        for r in rows:
            w.writerow([r[0], r[1], f"{r[2]:.0f}", f"{r[3]:.1f}", f"{r[4]:.3f}"])
    for r in rows[:12]:
        print(f"{r[4]:6.2f}%  {r[1]:7d} x {r[3] / 1e3:8.2f} us  {r[0][:110]}")


if __name__ == "__main__":
    main()
