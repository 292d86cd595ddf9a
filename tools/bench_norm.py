"""Micro-benchmark of GroupNorm (+SiLU, stats + apply passes) and LayerNorm at the UNet's level shapes.

  python tools/bench_norm.py        (ACTH_LIB=<other build> for an A/B of two libraries)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from actalker_amd import ops  # noqa: E402

# (rows, C, rows per statistics batch): spatial GN per frame / temporal GN per 14-frame window, 84 frames
SHAPES = [(774144, 320, 9216), (774144, 320, 14 * 9216), (193536, 640, 2304), (193536, 640, 14 * 2304),
          (48384, 1280, 576), (48384, 1280, 14 * 576)]


def main(iters=20):
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    for M, C, rps in SHAPES:
        x = torch.randn(M, C, generator=g).to(dev, torch.bfloat16)
        gamma, beta = torch.ones(C, device=dev), torch.zeros(C, device=dev)
        ops.groupnorm(x, gamma, beta, 1e-6, rps, silu=True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            ops.groupnorm(x, gamma, beta, 1e-6, rps, silu=True)
        e1.record()
        torch.cuda.synchronize()
        us = 1000.0 * e0.elapsed_time(e1) / iters
        gbs = 2 * M * C * 2 / (us * 1e3)          # algorithmic: x read once, y written once
        print(f"groupnorm M={M} C={C} rows/stat={rps}: {us:.1f} us  {gbs:.0f} GB/s (algorithmic)", flush=True)

    for M, C in ((774144, 320), (193536, 640), (48384, 1280)):
        x = torch.randn(M, C, generator=g).to(dev, torch.bfloat16)
        gamma, beta = torch.randn(C, generator=g).to(dev), torch.randn(C, generator=g).to(dev)
        ops.layernorm(x, gamma, beta, 1e-5)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            ops.layernorm(x, gamma, beta, 1e-5)
        e1.record()
        torch.cuda.synchronize()
        us = 1000.0 * e0.elapsed_time(e1) / iters
        print(f"layernorm M={M} C={C}: {us:.1f} us  {2 * M * C * 2 / (us * 1e3):.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
