"""Summarise a rocprofv3 kernel trace (rocpd SQLite ``*_results.db`` or ``kernel_stats.csv``) into the
per-kernel stats table committed under profiles/ (Name, Calls, TotalDurationNs, AverageNs, Percentage).

  python tools/prof_summary.py gpurun_out/prof_r1/run_results.db > profiles/r1_....csv
"""
import csv
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                     "from kernels group by name order by sum(end-start) desc").fetchall()
    return rows


def main():
    path = sys.argv[1]
    rows = from_db(path)
    tot = sum(r[2] for r in rows)
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, n, s, a, mn, mx in rows:
        w.writerow([name, n, int(s), round(a, 1), round(100.0 * s / tot, 3), int(mn), int(mx)])


if __name__ == "__main__":
    main()
