"""Where a fused-FFN workgroup's time goes: per-workgroup s_memtime stamps (acth_debug_ffn_stamps) at
entry, after the prologue (x rows in VGPRs, W1 chunk 0 in LDS), after chunk 0, after chunks 10 and 30,
after the chunk loop, after the epilogue. Prints mean cycles per phase and per chunk.

  python tools/ffn_stamps.py [--M 774144] [--modes plain,ln,ln_add,ln_mix]

Modes: plain = residual; ln = the prologue LayerNorm with residual = x (norm3 -> ff); ln_add = also the
frame-embedding row add (norm_in + pos_emb -> ff_in); ln_mix = ln with the AlphaBlender mix (temporal ff).
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from actalker_amd import _lib, ops  # noqa: E402
from actalker_amd.modules import pack_ffn_w2, pack_geglu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=774144)
    ap.add_argument("--modes", default="plain,ln,ln_add,ln_mix")
    a = ap.parse_args()
    for mode in a.modes.split(","):
        one(a.M, mode)


def one(M, mode):
    dev = torch.device("cuda:0")
    lib = _lib.load()
    C = 320
    g = torch.Generator().manual_seed(0)
    x = torch.randn(M, C, generator=g).to(dev, torch.bfloat16)
    res = torch.randn(M, C, generator=g).to(dev, torch.bfloat16)
    w1, b1 = pack_geglu(torch.randn(8 * C, C, generator=g) * C ** -0.5, 0.1 * torch.randn(8 * C, generator=g))
    w2 = pack_ffn_w2(torch.randn(C, 4 * C, generator=g) * (4 * C) ** -0.5)
    w1, b1, w2 = w1.to(dev), b1.to(dev), w2.to(dev)
    b2 = torch.zeros(C, device=dev)
    out = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
    ln = (1.0 + 0.1 * torch.randn(C, generator=g)).to(dev), (0.1 * torch.randn(C, generator=g)).to(dev), 1e-5
    S = 9216
    emb = torch.randn((M + S - 1) // S, C, generator=g).to(dev, torch.bfloat16)

    def run():
        if mode == "plain":
            ops.geglu_ffn(x, w1, b1, w2, b2, residual=res, out=out)
        else:
            ops.geglu_ffn(x, w1, b1, w2, b2, residual=x, out=out, ln=ln, add=emb if mode == "ln_add" else None,
                          add_div=S, mix=res if mode == "ln_mix" else None, mix_alpha=0.3)

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
    _lib.check(lib.acth_debug_ffn_stamps(None, 0, 1), "stamps on")
    run()
    torch.cuda.synchronize()
    _lib.check(lib.acth_debug_ffn_stamps(None, 0, 0), "stamps off")
    n = min((M + 127) // 128, 8192)
    buf = (ctypes.c_ulonglong * (8 * n))()
    _lib.check(lib.acth_debug_ffn_stamps(buf, n, 0), "stamps")
    st = np.frombuffer(buf, dtype=np.uint64).reshape(n, 8)[:, :7].astype(np.float64)
    ok = (st[:, 6] > st[:, 0]) & (st[:, 0] > 0)
    st = st[ok]
    d = np.diff(st, axis=1)
    tot = st[:, 6] - st[:, 0]
    names = ["prologue", "chunk0", "chunks1-10", "chunks11-30", "chunks31-40", "epilogue"]
    per = [1, 1, 10, 20, 10, 1]
    print(f"[{mode}] M={M}: {ms:.3f} ms; {len(st)} WGs stamped; mean cycles/WG total {tot.mean():.0f} "
          f"(median {np.median(tot):.0f}, p90 {np.percentile(tot, 90):.0f})")
    for i, nm in enumerate(names):
        print(f"  {nm:12s} {d[:, i].mean():9.0f}  per chunk {d[:, i].mean() / per[i]:8.0f}  "
              f"(p10 {np.percentile(d[:, i], 10):.0f} p90 {np.percentile(d[:, i], 90):.0f})")
    # wave of workgroups: start-time spread of the first 256
    s0 = np.sort(st[:256, 0])
    print(f"  first 256 WGs start spread {s0[-1] - s0[0]:.0f} cycles; kernel span (stamped WGs) "
          f"{st[:, 6].max() - st[:, 0].min():.0f}")


if __name__ == "__main__":
    main()
