"""Per-kernel duration statistics from a rocprofv3 --kernel-trace database (rocpd SQLite, the
ROCm 7 default output) in the column layout of rocprofv3's kernel_stats.csv.

  python tools/rocprof_stats.py gpurun_out/prof/run_results.db > profiles/rNN_kernel_stats.csv
"""
import csv
import sqlite3
import sys


def main(db_path):
    con = sqlite3.connect(db_path)
    rows = con.execute("select name, duration from kernels").fetchall()
    stats = {}
    for name, dur in rows:
        s = stats.setdefault(name, [0, 0.0, float("inf"), 0.0])
        s[0] += 1
        s[1] += dur
        s[2] = min(s[2], dur)
        s[3] = max(s[3], dur)
    total = sum(s[1] for s in stats.values()) or 1.0
    out = csv.writer(sys.stdout)
    out.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, (n, tot, mn, mx) in sorted(stats.items(), key=lambda kv: -kv[1][1]):
        out.writerow([name, n, int(tot), round(tot / n, 1), round(100.0 * tot / total, 3), int(mn), int(mx)])


if __name__ == "__main__":
    main(sys.argv[1])
