"""Per-UNet-call kernel time by (kernel, grid) from a rocprofv3 --kernel-trace CSV: which dispatch shapes
hold the step (grid x in workgroups, grid y); calls are normalised by the number of level-0 spatial
attention dispatches (10 flash16_kernel<8, false> -- flash_attn_kernel<8, false> before round 3 step 28 -- per UNet
call at 576x1024).

  python tools/trace_by_grid.py gpurun_out/<dir>/run_kernel_trace.csv|run_results.db [--top 45] [--filter gn_]
"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=45)
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    agg = collections.defaultdict(lambda: [0, 0.0])
    if a.csv.endswith(".db"):                       # rocprofv3 -o run (SQLite output)
        import sqlite3
        rows = sqlite3.connect(a.csv).execute(
            "select name, grid_x, workgroup_x, grid_y, grid_z, start, end from kernels").fetchall()
        it = ((n, gx // wx, gy * gz, (e - s) / 1e3) for n, gx, wx, gy, gz, s, e in rows)
    else:
        it = ((r["Kernel_Name"], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), int(r["Grid_Size_Y"]),
               (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in csv.DictReader(open(a.csv)))
    for name, gx, gy, us in it:
        n = re.sub(r"\(.*", "", name).replace("void ", "")
        k = (n, gx, gy)
        agg[k][0] += 1
        agg[k][1] += us
    calls = sum(v[0] for k, v in agg.items() if k[0] in ("flash_attn_kernel<8, false>", "flash16_kernel<8, false>")) / 10
    tot = sum(v[1] for v in agg.values()) / calls
    print(f"UNet calls {calls:.0f}; kernel ms per call {tot / 1e3:.1f}")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        if a.filter in k[0]:
            print(f"{v[1] / calls / 1e3:7.2f} ms {v[0] / calls:5.1f}x {v[1] / v[0]:8.1f} us  {k}")


if __name__ == "__main__":
    main()
