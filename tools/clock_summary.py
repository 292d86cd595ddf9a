"""Per-kernel-family effective clock from tools/clock_pass.sh: GRBM_GUI_ACTIVE (summed over the 8 XCDs by
rocprofv3) / 8 / the dispatch's wall time, averaged over dispatches weighted by time.

  python tools/clock_summary.py <dir_a> [<dir_b> ...]
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

FAMILIES = [("gemm8p conv", r"gemm8p_kernel<\d+, 1,"), ("gemm8p dense", r"gemm8p_kernel<\d+, [02],"),
            ("flash16", r"flash16_kernel"), ("ffn_geglu", r"ffn_geglu_kernel"), ("scan_pair", r"scan_pair_kernel"),
            ("gn", r"gn_(apply|stats)_kernel")]


def find(d, name):
    hits = glob.glob(os.path.join(d, "**", name), recursive=True)
    return hits[0] if hits else None


def load(d):
    cc = find(d, "run_counter_collection.csv")
    kt = find(d, "run_kernel_trace.csv")
    times = {}
    if kt:
        with open(kt) as f:
            for r in csv.DictReader(f):
                times[r["Dispatch_Id"]] = (r["Kernel_Name"], float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    fam = defaultdict(lambda: [0.0, 0.0])            # family -> [active cycles / 8, ns]
    with open(cc) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
                continue
            name = r["Kernel_Name"]
            if "Start_Timestamp" in r and r.get("End_Timestamp"):
                ns = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            elif r["Dispatch_Id"] in times:
                ns = times[r["Dispatch_Id"]][1]
            else:
                continue
            if ns < 300e3:                                  # the quotient reads high below ~0.3 ms
                continue
            for label, pat in FAMILIES:
                if re.search(pat, name):
                    fam[label][0] += float(r["Counter_Value"]) / 8.0
                    fam[label][1] += ns
                    break
    return {k: v[0] / v[1] for k, v in fam.items() if v[1] > 0}      # cycles per ns = GHz


def main():
    res = [(d, load(d)) for d in sys.argv[1:]]
    print("family        " + "  ".join(f"{os.path.basename(d.rstrip('/')):>10s}" for d, _ in res) + "   (GHz)")
    for label, _ in FAMILIES:
        print(f"{label:13s} " + "  ".join(f"{r.get(label, float('nan')):10.3f}" for _, r in res))


if __name__ == "__main__":
    main()
