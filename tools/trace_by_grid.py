"""Per-UNet-call kernel time by (kernel, grid) from a rocprofv3 --kernel-trace CSV: which dispatch shapes
hold the step (grid x in workgroups, grid y); calls are normalised by the number of level-0 spatial
attention dispatches (10 flash_attn_kernel<8, false> per UNet call at 576x1024).

  python tools/trace_by_grid.py gpurun_out/<dir>/run_kernel_trace.csv [--top 45] [--filter gn_]
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
    for r in csv.DictReader(open(a.csv)):
        n = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
        k = (n, int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), int(r["Grid_Size_Y"]))
        agg[k][0] += 1
        agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    calls = sum(v[0] for k, v in agg.items() if k[0] == "flash_attn_kernel<8, false>") / 10
    tot = sum(v[1] for v in agg.values()) / calls
    print(f"UNet calls {calls:.0f}; kernel ms per call {tot / 1e3:.1f}")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        if a.filter in k[0]:
            print(f"{v[1] / calls / 1e3:7.2f} ms {v[0] / calls:5.1f}x {v[1] / v[0]:8.1f} us  {k}")


if __name__ == "__main__":
    main()
