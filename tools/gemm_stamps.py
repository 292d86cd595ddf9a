"""Where a phased-GEMM workgroup's time goes: per-workgroup s_memtime stamps (tile bit 0x400) at entry,
after the prologue's K tile 0 has landed, after the main loop and after the epilogue, for the
bench_gemm shapes. Prints per-phase mean cycles per workgroup and the kernel's wall time.

  python tools/gemm_stamps.py [--only 0,3] [--residual]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from actalker_amd import _lib, ops  # noqa: E402
from tools.bench_gemm import SHAPES, run  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="0,3,4,5")
    ap.add_argument("--residual", action="store_true")
    ap.add_argument("--tile", type=int, default=0)
    ap.add_argument("--sink", action="store_true", help="every row block writes the same 256 output rows")
    ap.add_argument("--timeline", action="store_true", help="histogram of the epilogue fraction of resident WGs")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.load()
    for idx in [int(i) for i in a.only.split(",")]:
        mode, M, N, K, act = SHAPES[idx]
        tf, ms = run(mode, M, N, K, act, a.tile, 5, dev, sink=a.sink, residual=a.residual)
        flags = 0x400 | (0x800 if a.timeline else 0)
        tf2, ms2 = run(mode, M, N, K, act, a.tile | flags, 1, dev, sink=a.sink, residual=a.residual)
        mt = (M + 255) // 256
        nt = -(-N // 320) if (a.tile or 5) == 5 and act != 2 else -(-N // 256)
        n = min(mt * nt, 16384)
        buf = (ctypes.c_ulonglong * (4 * n))()
        _lib.check(lib.acth_debug_gemm_stamps(buf, n), "stamps")
        st = np.frombuffer(buf, dtype=np.uint64).reshape(n, 4).astype(np.float64)
        ok = (st[:, 3] > st[:, 0]) & (st[:, 0] > 0)
        xcd = (np.arange(n) % 8)[ok]
        st = st[ok]
        if a.timeline:
            # phase concurrency (stamps from the chip-wide 100 MHz s_memrealtime): at 400 instants over the
            # kernel, the fraction of resident workgroups that are in their epilogue
            s0 = st
            t0, t1 = s0[:, 0].min(), s0[:, 3].max()
            ts = np.linspace(t0, t1, 400)
            nres = ((s0[None, :, 0] <= ts[:, None]) & (ts[:, None] < s0[None, :, 3])).sum(1)
            epi = ((s0[None, :, 2] <= ts[:, None]) & (ts[:, None] < s0[None, :, 3])).sum(1)
            fr = epi / np.maximum(nres, 1)
            hist = np.histogram(fr[nres > 0], bins=5, range=(0, 1))[0]
            print(f"  epilogue-fraction histogram (0-0.2 .. 0.8-1): {hist.tolist()}, mean resident {nres.mean():.1f}, "
                  f"epilogue fraction std {fr[nres > 0].std():.3f}", flush=True)
            st = st * 20.0            # 100 MHz ticks -> ~2 GHz cycles for the per-phase means below
        d = np.diff(st, axis=1)
        tot = st[:, 3] - st[:, 0]
        print(f"{mode} {M}x{N}x{K} act {act}{' +res' if a.residual else ''}{' sink' if a.sink else ''}: {ms:.3f} ms ({tf:.0f} TF/s), "
              f"stamped {ms2:.3f} ms; {len(st)} WGs; cycles/WG mean: prologue {d[:, 0].mean():.0f}, "
              f"main {d[:, 1].mean():.0f}, epilogue {d[:, 2].mean():.0f}, total {tot.mean():.0f} "
              f"(median {np.median(tot):.0f}, p90 {np.percentile(tot, 90):.0f})", flush=True)


if __name__ == "__main__":
    main()
