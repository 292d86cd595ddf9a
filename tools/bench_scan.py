"""Micro-benchmark of the fused bidirectional selective scan at the UNet's level shapes.

  python tools/bench_scan.py          # paired-lane single pass vs two-pass chunked kernels
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from actalker_amd import ops  # noqa: E402

# (nb, L, D = 2C, R): audio branch at levels 0 / 1 / 2 (S + 33 tokens); nb as in the bench step
# (grid quantisation over 256 CUs depends on nb: measure at the real nb)
SHAPES = [(84, 9249, 640, 20), (84, 2337, 1280, 40), (84, 609, 2560, 80)]   # the bench step: 6 units x 14 frames


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
        variants = [("pair", 1), ("chunk2", 2), ("chunk4", 4)]
        for name, nc in variants:
            args = dict(nb=nb, L=L, R=R, n_keep=n_keep, nchunks=nc)
            y = ops.selective_scan(u, xdbl, dtw, dtb, alog, Dp, **args)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                ops.selective_scan(u, xdbl, dtw, dtb, alog, Dp, **args)
            e1.record()
            torch.cuda.synchronize()
            res[name] = (e0.elapsed_time(e1) / iters, y)
        ref = res["pair"][1]
        cells = []
        for name, _ in variants:
            err = max(((res[name][1][i].float() - ref[i].float()).norm() / ref[i].float().norm()).item()
                      for i in range(2))
            cells.append(f"{name} {res[name][0]:.3f} ms (d {err:.1e})")
        print(f"scan nb={nb} L={L} D={D} R={R}: " + "  ".join(cells), flush=True)


if __name__ == "__main__":
    main()
