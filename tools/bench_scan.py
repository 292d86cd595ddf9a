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


def main(iters=3, only_quad=False):
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    shapes = SHAPES
    if "--shape" in sys.argv:
        shapes = [tuple(int(v) for v in a.split(",")) for a in sys.argv[sys.argv.index("--shape") + 1:]]
    for nb, L, D, R in shapes:
        u = torch.randn(nb * L, D, generator=g).to(dev, torch.bfloat16)
        xdbl = (0.3 * torch.randn(nb * L, 2 * (R + 32), generator=g)).to(dev)
        dtw = (0.1 * torch.randn(2, D, R, generator=g)).to(dev)
        dtb = torch.full((2, D), -3.0).to(dev)
        alog = torch.log(torch.arange(1, 17).float()).repeat(2 * D, 1).to(dev)
        Dp = torch.ones(2 * D).to(dev)
        n_keep = L - 33 if L > 33 else L
        res = {}
        xbf = xdbl.to(torch.bfloat16)
        variants = [("pair", 1, xdbl), ("pairbf", 1, xbf), ("quad", 1, xbf)]
        if only_quad:
            variants = [("quad", 1, xbf)]
        if "--seg" in sys.argv:
            # the two-pass wavefront-segmented form (scan_kernel<R, PASS>: each chunk from a zero state, the
            # chunk-end states carried across in pass 2; fp32 xdbl rows) beside the single-pass paired-lane kernel
            variants = [("pairbf", 1, xbf), ("seg2", 2, xdbl), ("seg4", 4, xdbl), ("seg8", 8, xdbl)]
        for name, nc, xd in variants:
            ops.SCAN_ALGO = 1 if name == "quad" else 0
            args = dict(nb=nb, L=L, R=R, n_keep=n_keep, nchunks=nc)
            y = ops.selective_scan(u, xd, dtw, dtb, alog, Dp, **args)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                ops.selective_scan(u, xd, dtw, dtb, alog, Dp, **args)
            e1.record()
            torch.cuda.synchronize()
            res[name] = (e0.elapsed_time(e1) / iters, y)
        # mode 2: both branches (audio L, expression L - 31) in one paired launch
        for name, xd in ((("quad2", xbf),) if only_quad else (("pair2", xdbl), ("pairbf2", xbf), ("quad2", xbf))):
            ops.SCAN_ALGO = 1 if name == "quad2" else 0
            La = dict(u=u, xdbl=xd, dt_w=dtw, dt_b=dtb, A_log=alog, Dskip=Dp, nb=nb, L=L, R=R, n_keep=n_keep)
            ops.selective_scan2(La, dict(La))
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                ops.selective_scan2(La, dict(La))
            e1.record()
            torch.cuda.synchronize()
            print(f"  {name} (two branches, one launch) {e0.elapsed_time(e1) / iters:.3f} ms", flush=True)
        ref = res[variants[0][0]][1]
        cells = []
        for name, _, _ in variants:
            err = max(((res[name][1][i].float() - ref[i].float()).norm() / ref[i].float().norm()).item()
                      for i in range(2))
            cells.append(f"{name} {res[name][0]:.3f} ms (d {err:.1e})")
        print(f"scan nb={nb} L={L} D={D} R={R}: " + "  ".join(cells), flush=True)


if __name__ == "__main__":
    main(only_quad="--quad" in sys.argv)
# C5's per-rank load (8 GPUs, mode 2: 5 units x 14 frames = 70 batch elements per UNet call):
#   python tools/bench_scan.py --seg --shape 70,9249,640,20 70,2337,1280,40 70,609,2560,80
