"""Micro-benchmark of the fused bidirectional selective scan at the UNet's level shapes.

  python tools/bench_scan.py          # single-pass paired-lane kernel vs two-pass chunked kernel
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from actalker_amd import ops  # noqa: E402

# (nb, L, D = 2C, R): audio branch at levels 0 / 1 / 2 (S + 33 tokens)
SHAPES = [(56, 9249, 640, 20), (56, 2337, 1280, 40), (56, 609, 2560, 80)]


def main(iters=3):
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    for nb, L, D, R in SHAPES:
        u = torch.randn(nb * L, D, generator=g).to(dev, torch.bfloat16)
        xdbl = (0.3 * torch.randn(nb * L, 2 * (R + 32), generator=g)).to(dev)
        dtw = (0.1 * torch.randn(2, D, R, generator=g)).to(dev)
        dtb = torch.full((2, D), -3.0).to(dev)
        alog = torch.log(torch.arange(1, 17).float()).repeat(2 * D, 1).to(dev)
        Dp = torch.ones(2 * D).to(dev)
        n_keep = L - 33
        res = {}
        for nc in (1, None):
            args = dict(nb=nb, L=L, R=R, n_keep=n_keep, nchunks=nc)
            y = ops.selective_scan(u, xdbl, dtw, dtb, alog, Dp, **args)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                ops.selective_scan(u, xdbl, dtw, dtb, alog, Dp, **args)
            e1.record()
            torch.cuda.synchronize()
            res[nc] = (e0.elapsed_time(e1) / iters, y)
        err = max(((res[1][1][i].float() - res[None][1][i].float()).norm() / res[None][1][i].float().norm()).item()
                  for i in range(2))
        print(f"scan nb={nb} L={L} D={D} R={R}: pair {res[1][0]:.3f} ms  two-pass {res[None][0]:.3f} ms  "
              f"rel diff {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
