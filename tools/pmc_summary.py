"""Per-kernel HBM traffic from two rocprofv3 --pmc passes (tools/pmc_pass.sh): FETCH_SIZE and WRITE_SIZE
are reported in KiB per dispatch; on gfx950 FETCH_SIZE counts half the bytes of wide streaming reads
(MI355X_MICROARCH.md, HBM section), so read bytes = 2 x FETCH_SIZE x 1024 and write bytes = WRITE_SIZE x 1024.

  python tools/pmc_summary.py gpurun_out/pmc1 > profiles/r1_pmc_traffic.csv
"""
import csv
import os
import sys
from collections import defaultdict


def load(path, counter):
    vals = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return vals


def main():
    d = sys.argv[1]
    fetch = load(os.path.join(d, "FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE")
    write = load(os.path.join(d, "WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE")
    rows = []
    for name, fv in fetch.items():
        wv = write.get(name, [])
        rd = 2.0 * 1024.0 * sum(fv)
        wr = 1024.0 * sum(wv)
        rows.append((name, len(fv), rd, wr))
    rows.sort(key=lambda r: -(r[2] + r[3]))
    if "--json" in sys.argv:
        # per-launch average over every acth_gemm kernel (names containing "gemm"), for
        # bench.py's roofline.traffic
        import json
        out = sys.argv[sys.argv.index("--json") + 1]
        src = sys.argv[sys.argv.index("--source") + 1] if "--source" in sys.argv else d
        import re
        fams = {"acth_gemm": lambda k: "gemm" in k, "flash_attn": lambda k: "flash_attn" in k or "flash16" in k,
                # the implicit-GEMM 3x3 convs (phased kernel, A mode 1): their per-tap image re-reads
                "gemm_conv": lambda k: re.match(r"gemm8p_kernel<\d+, 1,", k) is not None,
                "selective_scan": lambda k: "scan" in k, "groupnorm": lambda k: k.startswith("gn_"),
                "layernorm": lambda k: "layernorm" in k, "geglu_ffn": lambda k: "ffn_geglu" in k,
                "mamba_combine": lambda k: "mamba_combine" in k}
        # the bench configuration the counted run used (bench.py only reports traffic for that same workload)
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from actalker_amd._lib import kernel_source_digest
        res = {"_workload": sys.argv[sys.argv.index("--workload") + 1] if "--workload" in sys.argv else None,
               "_kernel_sources": kernel_source_digest()}
        for fam, match in fams.items():
            g = [r for r in rows if match(r[0].split("(")[0].replace("void ", ""))]
            n = sum(r[1] for r in g)
            if not n:
                continue
            res[fam] = {"hbm_bytes_per_launch": sum(r[2] + r[3] for r in g) / n, "dispatches": n,
                        "read_bytes": sum(r[2] for r in g), "write_bytes": sum(r[3] for r in g), "source": src}
        with open(out, "w") as fh:
            json.dump(res, fh, indent=1)
        return
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Dispatches", "ReadBytesTotal", "WriteBytesTotal", "HbmBytesPerDispatch"])
    for name, n, rd, wr in rows:
        w.writerow([name, n, int(rd), int(wr), int((rd + wr) / max(n, 1))])


if __name__ == "__main__":
    main()
