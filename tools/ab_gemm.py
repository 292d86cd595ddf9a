"""A/B of two acth_gemm main-loop variants selected by tile flag bits, interleaved in one process (rounds x
variants, median and min per shape), with a bitwise comparison of their outputs (same K order: the variants
must agree exactly).

  python tools/ab_gemm.py [--flags-b 0x2000] [--only 0,1,2] [--rounds 5] [--residual]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from actalker_amd import ops  # noqa: E402
from tools.bench_gemm import CONV_HW, SHAPES  # noqa: E402


def operands(mode, M, N, K, act, dev, residual):
    g = torch.Generator(device="cpu").manual_seed(0)
    kw = {}
    if mode == "conv":
        cin = K // 9
        H, W = CONV_HW[M]
        B = M // (H * W)
        a = torch.randn(B * H * W, cin, generator=g).to(dev, torch.bfloat16)
        kw["conv"] = dict(H=H, W=W, Ho=H, Wo=W, stride=1, upsample=False, B=B)
    elif mode == "temporal":
        a = torch.randn(M, K // 3, generator=g).to(dev, torch.bfloat16)
        kw["temporal"] = dict(F=14, S=9216 if M in (774144, 516096) else 2304 if M in (193536, 129024) else 576)
    else:
        a = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * K ** -0.5).to(dev, torch.bfloat16)
    bias = torch.randn(N, generator=g).to(dev)
    if residual and act != 2:
        kw["residual"] = torch.randn(M, N, generator=g).to(dev, torch.bfloat16)
    return a, w, bias, kw


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flags-a", type=lambda s: int(s, 0), default=0x1000)
    ap.add_argument("--flags-b", type=lambda s: int(s, 0), default=0x2000)
    ap.add_argument("--extra", default="", help="comma-separated further flag sets, timed only (diagnostics)")
    ap.add_argument("--only", default="")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--tile", type=int, default=0)
    ap.add_argument("--residual", action="store_true")
    a_ = ap.parse_args()
    dev = torch.device("cuda:0")
    only = {int(i) for i in a_.only.split(",")} if a_.only else None
    print(f"A = flags {a_.flags_a:#x}, B = flags {a_.flags_b:#x}, tile {a_.tile}", flush=True)
    for idx, (mode, M, N, K, act) in enumerate(SHAPES):
        if only is not None and idx not in only:
            continue
        a, w, bias, kw = operands(mode, M, N, K, act, dev, a_.residual)
        outs, times = {}, {"A": [], "B": []}
        for name, fl in (("A", a_.flags_a), ("B", a_.flags_b)):
            outs[name] = ops.gemm(a, w, bias=bias, act=act, tile=a_.tile | fl, **kw)
        torch.cuda.synchronize()
        same = torch.equal(outs["A"], outs["B"])
        for _ in range(a_.rounds):
            for name, fl in (("A", a_.flags_a), ("B", a_.flags_b)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a_.iters):
                    ops.gemm(a, w, bias=bias, act=act, tile=a_.tile | fl, **kw)
                e1.record()
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1) / a_.iters)
        for xf in [int(x, 0) for x in a_.extra.split(",") if x]:
            ts = []
            for _ in range(a_.rounds):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a_.iters):
                    ops.gemm(a, w, bias=bias, act=act, tile=a_.tile | xf, **kw)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / a_.iters)
            print(f"     flags {xf:#x}: {2.0 * M * N * K / statistics.median(ts) / 1e9:7.1f} TF/s", flush=True)
        fl = 2.0 * M * N * K
        ta, tb = statistics.median(times["A"]), statistics.median(times["B"])
        print(f"[{idx:2d}] {mode:8s} {M:7d}x{N:5d}x{K:5d} act {act}: A {fl / ta / 1e9:7.1f} TF/s "
              f"(min {min(times['A']) * 1e3:8.1f} us) | B {fl / tb / 1e9:7.1f} TF/s (min {min(times['B']) * 1e3:8.1f} us)"
              f" | A/B speed {tb / ta:.3f} | bitwise equal {same}", flush=True)
        del a, w, bias, kw, outs


if __name__ == "__main__":
    main()
