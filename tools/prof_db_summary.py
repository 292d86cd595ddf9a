"""Kernel-time summary from a rocprofv3 --kernel-trace SQLite output (run_results.db): per kernel name the
dispatch count, total / average duration, and per-family totals per sampler step.

  python tools/prof_db_summary.py gpurun_out/x/prof/run_results.db [steps] > profiles/...csv
"""
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name_col}, start, end from kernels").fetchall()
    agg = defaultdict(lambda: [0, 0.0])
    for n, s, e in rows:
        agg[n][0] += 1
        agg[n][1] += (e - s)
    tot = sum(v[1] for v in agg.values())
    print("Name,Calls,TotalDurationNs,AverageNs,Percentage,MsPerStep")
    for n, (k, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"\"{n}\",{k},{int(t)},{t / k:.1f},{100 * t / tot:.3f},{t / 1e6 / steps:.3f}")


if __name__ == "__main__":
    main()
