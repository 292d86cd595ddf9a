"""Summarise tools/pmc_kernels.sh output: per probe, the dominant kernel's counters averaged per dispatch
and the derived figures (MFMA busy fraction of SQ_BUSY_CYCLES, VALU / LDS / wait shares of wave
cycles, HBM bytes with the gfx950 FETCH_SIZE x 2 correction, L2 hit rate).

  python tools/pmc_table.py gpurun_out/pmc > profiles/r2_pmc_kernels.md
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return vals


def main():
    root = sys.argv[1]
    print("| probe | kernel | dispatches | MFMA busy / SQ busy | VALU active / wave cyc | LDS active | wait (parked) | "
          "wait (issue) | VALU insts / wave | trans insts / wave | MFMA insts / wave | LDS bank conflict / LDS inst | "
          "HBM read MB | HBM write MB | L2 hit |")
    print("|" + "---|" * 15)
    for d in sorted(glob.glob(os.path.join(root, "*"))):
        if not os.path.isdir(d):
            continue
        vals = load(d)
        if not vals:
            continue
        name = max(vals, key=lambda k: sum(vals[k].get("SQ_WAVE_CYCLES", [0])))
        v = {c: sum(x) / len(x) for c, x in vals[name].items()}
        n = len(vals[name].get("SQ_WAVES", []))
        g = lambda c: v.get(c, float("nan"))  # noqa: E731
        waves = g("SQ_WAVES")
        wc = g("SQ_WAVE_CYCLES")
        row = [os.path.basename(d), name.split("(")[0][:40], n,
               g("SQ_VALU_MFMA_BUSY_CYCLES") / (4 * g("SQ_BUSY_CYCLES")) if g("SQ_BUSY_CYCLES") else float("nan"),
               g("SQ_ACTIVE_INST_VALU") / wc, g("SQ_ACTIVE_INST_LDS") / wc, g("SQ_WAIT_ANY") / wc,
               g("SQ_WAIT_INST_ANY") / wc, g("SQ_INSTS_VALU") / waves, g("SQ_INSTS_VALU_TRANS_F32") / waves,
               g("SQ_INSTS_MFMA") / waves, g("SQ_LDS_BANK_CONFLICT") / max(g("SQ_INSTS_LDS"), 1),
               2 * 1024 * g("FETCH_SIZE") / 1e6, 1024 * g("WRITE_SIZE") / 1e6,
               g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum"))]
        print("| " + " | ".join(f"{x:.3g}" if isinstance(x, float) else str(x) for x in row) + " |")


if __name__ == "__main__":
    main()
