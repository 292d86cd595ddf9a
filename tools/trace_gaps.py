"""GPU idle time inside bench.py's timed loop, from a rocprofv3 --kernel-trace CSV of a run with
ACTH_TRACE_MARK=1 (a spin kernel on each side of the timed loop): kernel busy time vs the span between the
markers, and the largest idle gaps with the kernels on either side. Diagnostic only.

  python tools/trace_gaps.py gpurun_out/<dir>/run_kernel_trace.csv [--steps K] [--top 25]
"""
import argparse
import collections
import csv
import re


def short(n):
    return re.sub(r"\(.*", "", n).replace("void ", "")[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--stats-csv", default=None,
                    help="also write per-kernel stats of the timed steps (Name, Calls, TotalDurationNs, AverageNs, "
                         "Percentage, MsPerStep) to this file")
    a = ap.parse_args()
    rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                   for r in csv.DictReader(open(a.csv))), key=lambda x: x[0])
    marks = [i for i, r in enumerate(rows) if "sleep" in r[2].lower() or "spin" in r[2].lower()]
    if len(marks) < 2:
        raise SystemExit(f"need two marker kernels, found {len(marks)}")
    i0, i1 = marks[-2], marks[-1]
    ks = rows[i0 + 1:i1]
    span = ks[-1][1] - ks[0][0]
    busy, end, gaps = 0, ks[0][0], []
    for k, (s, e, n) in enumerate(ks):
        if s > end:
            gaps.append((s - end, short(ks[k - 1][2]) if k else "-", short(n)))
        busy += max(0, e - max(s, end))
        end = max(end, e)
    idle = sum(g[0] for g in gaps)
    print(f"timed kernels {len(ks)}  span {span / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms  idle {idle / 1e6:.2f} ms "
          f"({100 * idle / span:.1f} %)  per step: span {span / 1e6 / a.steps:.2f} busy {busy / 1e6 / a.steps:.2f}")
    hist = collections.Counter()
    for g, _, _ in gaps:
        hist["<2us" if g < 2e3 else "2-5us" if g < 5e3 else "5-20us" if g < 2e4 else "20-100us" if g < 1e5
             else ">=100us"] += g
    print("idle by gap size (ms):", {k: round(v / 1e6, 2) for k, v in hist.items()})
    pair = collections.defaultdict(lambda: [0, 0])
    for g, p, n in gaps:
        if g >= 5e3:
            pair[(p, n)][0] += 1
            pair[(p, n)][1] += g
    if a.stats_csv:
        agg = collections.defaultdict(lambda: [0, 0])
        for s, e, n in ks:
            agg[n][0] += 1
            agg[n][1] += e - s
        tot = sum(v[1] for v in agg.values())
        with open(a.stats_csv, "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MsPerStep"])
            for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
                w.writerow([n, c, t, round(t / c, 1), round(100.0 * t / tot, 3), round(t / 1e6 / a.steps, 3)])
    print("largest idle sources (gaps >= 5 us, grouped by kernel pair):")
    for (p, n), (c, g) in sorted(pair.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"  {g / 1e6:7.3f} ms {c:5d}x  {p}  ->  {n}")


if __name__ == "__main__":
    main()
