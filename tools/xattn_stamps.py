"""Where a fused cross-attention workgroup's time goes (acth_xattn at the level-0 shape: 84 frames x 9216
tokens, C = 320, 5 heads, masks on): per-workgroup s_memtime stamps (acth_debug_xattn_stamps) at entry,
h rows + head 0 landed, LN2 statistics, after the head loop, after epilogue phase 1, at the end. Prints the
kernel time and mean cycles per phase.

  python tools/xattn_stamps.py [--frames 84] [--temporal]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from actalker_amd import _lib, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=84)
    ap.add_argument("--temporal", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.load()
    C, H, S = 320, 5, 9216
    nctx = a.frames // 14 if a.temporal else a.frames
    rpc = a.frames * S // nctx
    M = a.frames * S
    g = torch.Generator().manual_seed(0)
    bf = lambda t: t.to(dev, torch.bfloat16)   # noqa: E731
    h = bf(torch.randn(M, C, generator=g))
    wq, woT = bf(torch.randn(C, C, generator=g) * C ** -0.5), bf(torch.randn(C, C, generator=g) * C ** -0.5)
    kv, vid, vb = bf(torch.randn(nctx * 32, 2 * C, generator=g)), bf(torch.randn(nctx, C, generator=g)), \
        bf(torch.randn(nctx, C, generator=g))
    n2 = (torch.ones(C, device=dev), torch.zeros(C, device=dev))
    n3 = (torch.ones(C, device=dev), torch.zeros(C, device=dev), 1e-5)
    ma = None if a.temporal else torch.rand(S, generator=g).to(dev)
    kp, vp, gb, base, vbw = ops.ip_fold(wq, woT, None, vid, kv=kv, vb=vb, heads=H, norm2=n2)

    def run():
        return ops.xattn(h, 1e-5, n3, base, heads=H, rows_per_ctx=rpc, S=rpc if a.temporal else S, kp=kp, vp=vp,
                         gb=gb, vbw=vbw, mask_a=ma, mask_b=ma, sa=1.25, sb=1.25)

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    _lib.check(lib.acth_debug_xattn_stamps(None, 0, 1), "stamps on")
    run()
    torch.cuda.synchronize()
    _lib.check(lib.acth_debug_xattn_stamps(None, 0, 0), "stamps off")
    n = min(M // 64, 8192)
    buf = (ctypes.c_ulonglong * (6 * n))()
    _lib.check(lib.acth_debug_xattn_stamps(buf, n, 0), "stamps")
    st = np.frombuffer(buf, dtype=np.uint64).reshape(n, 6).astype(np.float64)
    ok = (st[:, 5] > st[:, 0]) & (st[:, 0] > 0)
    st = st[ok]
    d = np.diff(st, axis=1)
    tot = st[:, 5] - st[:, 0]
    gbytes = 3 * M * C * 2 / 1e9
    print(f"M={M} ({'temporal' if a.temporal else 'spatial'}): {ms:.3f} ms ({gbytes / ms:.2f} TB/s on 3 passes); "
          f"{len(st)} WGs stamped; cycles/WG mean {tot.mean():.0f} (median {np.median(tot):.0f})")
    for i, nm in enumerate(["prologue (h rows, head 0)", "LN2 stats", "head loop", "epilogue 1", "epilogue 2-4"]):
        print(f"  {nm:26s} {d[:, i].mean():9.0f}  (p10 {np.percentile(d[:, i], 10):.0f} "
              f"p90 {np.percentile(d[:, i], 90):.0f})")
    s0 = np.sort(st[:, 0])
    print(f"  kernel span (stamped WGs) {st[:, 5].max() - st[:, 0].min():.0f} cycles; start spread of the first "
          f"256 WGs {s0[255] - s0[0]:.0f}")


if __name__ == "__main__":
    main()
