"""One kernel family at one shape, repeated, for rocprofv3 PMC passes (tools/pmc_kernels.sh): the
per-dispatch counters then belong to a single kernel configuration.

  python tools/pmc_probe.py gemm <SHAPES index> [--residual]
  python tools/pmc_probe.py flash <nbatch> <S> <heads>
  python tools/pmc_probe.py scan <nb> <L> <D> <R>
  python tools/pmc_probe.py ffn <M>
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from actalker_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kind")
    ap.add_argument("args", nargs="*", type=int)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--residual", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    if a.kind == "gemm":
        from tools.bench_gemm import SHAPES, run
        mode, M, N, K, act = SHAPES[a.args[0]]
        tf, ms = run(mode, M, N, K, act, 0, a.iters, dev, residual=a.residual)
        print(f"gemm {mode} {M}x{N}x{K} act {act}: {ms:.3f} ms {tf:.1f} TF/s")
    elif a.kind == "flash":
        nb, S, H = a.args
        qkv = torch.randn(nb * S, 3 * H * 64, generator=g).to(dev, torch.bfloat16)
        for _ in range(a.iters):
            ops.flash_attn(qkv, nb, S, H)
        torch.cuda.synchronize()
    elif a.kind in ("scan", "scanq"):          # scanq: bf16 x_proj rows (scan_quad_kernel)
        nb, L, D, R = a.args
        u = torch.randn(nb * L, D, generator=g).to(dev, torch.bfloat16)
        xdbl = (0.3 * torch.randn(nb * L, 2 * (R + 32), generator=g)).to(dev)
        if a.kind == "scanq":
            xdbl = xdbl.to(torch.bfloat16)
        dtw = (0.1 * torch.randn(2, D, R, generator=g)).to(dev)
        dtb = torch.full((2, D), -3.0).to(dev)
        alog = torch.log(torch.arange(1, 17).float()).repeat(2 * D, 1).to(dev)
        Dp = torch.ones(2 * D).to(dev)
        for _ in range(a.iters):
            ops.selective_scan(u, xdbl, dtw, dtb, alog, Dp, nb=nb, L=L, R=R, n_keep=L - 33)
        torch.cuda.synchronize()
    elif a.kind == "ffn":
        from actalker_amd.modules import pack_ffn_w2, pack_geglu
        M, C = a.args[0], 320
        x = torch.randn(M, C, generator=g).to(dev, torch.bfloat16)
        res = torch.randn(M, C, generator=g).to(dev, torch.bfloat16)
        w1, b1 = pack_geglu(torch.randn(8 * C, C, generator=g) * C ** -0.5, 0.1 * torch.randn(8 * C, generator=g))
        w2 = pack_ffn_w2(torch.randn(C, 4 * C, generator=g) * (4 * C) ** -0.5)
        w1, b1, w2 = w1.to(dev), b1.to(dev), w2.to(dev)
        b2 = torch.zeros(C, device=dev)
        for _ in range(a.iters):
            ops.geglu_ffn(x, w1, b1, w2, b2, residual=res)
        torch.cuda.synchronize()
    else:
        raise SystemExit(f"unknown kind {a.kind}")


if __name__ == "__main__":
    main()
