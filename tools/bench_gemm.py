"""Micro-benchmark of acth_gemm per tile variant on the UNet's dominant shapes (random data).

  python tools/bench_gemm.py [--tiles 1,2,3] [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from actalker_amd import ops  # noqa: E402

# (mode, M, N, K, act) — bench.py ACTH_GEMM_STATS at 576x1024, 84-frame calls (profiles/r2_step0_gemm_shapes.log),
# ordered by their share of the mode-0 step
SHAPES = [
    ("dense", 774144, 2560, 320, 2), ("dense", 193536, 5120, 640, 2), ("dense", 48384, 10240, 1280, 2),
    ("dense", 774144, 320, 320, 0), ("dense", 774144, 320, 1280, 0), ("conv", 774144, 320, 2880, 0),
    ("dense", 193536, 640, 640, 0), ("dense", 193536, 640, 2560, 0), ("dense", 774144, 960, 320, 0),
    ("dense", 48384, 1280, 5120, 0), ("conv", 48384, 1280, 11520, 0), ("conv", 193536, 640, 5760, 0),
    ("dense", 48384, 1280, 1280, 0), ("temporal", 774144, 320, 960, 0), ("dense", 193536, 1920, 640, 0),
    ("dense", 774144, 640, 320, 0), ("conv", 12096, 1280, 11520, 0),
    # reference points (not UNet shapes): square 4096^3 / 8192^3 (operands L2 / MALL resident),
    # and a 2048-wide K = 4096 panel streaming a 1 GB A from HBM
    ("dense", 4096, 4096, 4096, 0), ("dense", 8192, 8192, 8192, 0), ("dense", 131072, 2048, 4096, 0),
    # the Mamba x_proj at levels 0 / 1 / 2 (N = 2 (R + 32); fp32 out in the UNet)
    ("dense", 776916, 104, 640, 0), ("dense", 196308, 144, 1280, 0), ("dense", 51156, 224, 2560, 0),
    ("conv", 774144, 4, 2880, 0),        # conv_out
]
CONV_HW = {774144: (72, 128), 193536: (36, 64), 48384: (18, 32), 12096: (9, 16),
           516096: (72, 128), 129024: (36, 64), 32256: (18, 32), 8064: (9, 16)}


def run(mode, M, N, K, act, tile, iters, dev, sink=False, residual=False):
    g = torch.Generator(device="cpu").manual_seed(0)
    kw = {}
    if mode == "conv":
        cin = K // 9
        H, W = CONV_HW[M]
        B = M // (H * W)
        a = torch.randn(B * H * W, cin, generator=g).to(dev, torch.bfloat16)
        kw["conv"] = dict(H=H, W=W, Ho=H, Wo=W, stride=1, upsample=False, B=B)
    elif mode == "temporal":
        cin = K // 3
        a = torch.randn(M, cin, generator=g).to(dev, torch.bfloat16)
        kw["temporal"] = dict(F=14, S=9216 if M in (774144, 516096) else 2304 if M in (193536, 129024) else 576)
    else:
        a = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * K ** -0.5).to(dev, torch.bfloat16)
    bias = torch.randn(N, generator=g).to(dev)
    if residual and act != 2:   # residual-stream epilogue (attention / proj_out GEMMs)
        kw["residual"] = torch.randn(M, N, generator=g).to(dev, torch.bfloat16)
    if sink:   # every row block writes the same 256 output rows (L2-resident): no HBM write traffic
        kw["out"] = torch.empty(256, N // 2 if act == 2 else N, device=dev, dtype=torch.bfloat16)
        kw["orow"] = (256, 0, 0)
    try:
        ops.gemm(a, w, bias=bias, act=act, tile=tile, **kw)
    except Exception as e:  # noqa: BLE001
        return None, str(e)[:60]
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        ops.gemm(a, w, bias=bias, act=act, tile=tile, **kw)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    return 2.0 * M * N * K / (ms / 1e3) / 1e12, ms


def run_lib(M, N, K, iters, dev):
    """torch.matmul (hipBLASLt) on the same dense shape, no epilogue: the library reference point."""
    g = torch.Generator(device="cpu").manual_seed(0)
    a = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * K ** -0.5).to(dev, torch.bfloat16)
    torch.matmul(a, w.t())
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        torch.matmul(a, w.t())
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    return 2.0 * M * N * K / (ms / 1e3) / 1e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="0,1,2,3")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--flags", type=int, default=0, help="OR-ed into tile (0x100: skip epilogue)")
    ap.add_argument("--only", default="", help="comma-separated SHAPES indices")
    ap.add_argument("--lib", action="store_true", help="add a torch.matmul (hipBLASLt) column for dense shapes")
    ap.add_argument("--sink", action="store_true", help="write all output row blocks to one 256-row buffer")
    ap.add_argument("--residual", action="store_true", help="add a bf16 residual (M, N) in the epilogue")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    tiles = [int(t) for t in args.tiles.split(",")]
    print("mode      M       N     K    act " + " ".join(f"tile{t:d}(TF/s)" for t in tiles)
          + ("   hipblaslt" if args.lib else ""), flush=True)
    only = {int(i) for i in args.only.split(",")} if args.only else None
    for idx, (mode, M, N, K, act) in enumerate(SHAPES):
        if only is not None and idx not in only:
            continue
        cells = []
        for t in tiles:
            tf, ms = run(mode, M, N, K, act, t | args.flags, args.iters, dev, args.sink, args.residual)
            cells.append(f"{tf:12.1f}" if tf is not None else f"{'n/a':>12s}")
        if args.lib:
            cells.append(f"{run_lib(M, N, K, args.iters, dev):12.1f}" if mode == "dense" else f"{'-':>12s}")
        print(f"{mode:8s} {M:7d} {N:5d} {K:5d} {act:3d} " + " ".join(cells), flush=True)


if __name__ == "__main__":
    main()
