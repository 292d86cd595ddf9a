"""Per-wave segment cycle sums of the phased GEMM's ring main loop (diagnostic build, G8_RING_STAMPS=1, loaded
through ACTH_LIB): per bench_gemm SHAPES index, the mean cycles per 32-deep sub-tile each wave half spends in its
read + DMA-issue segment, the barrier after it, the MFMA segment and the barrier after that (waves 0-3 lead,
4-7 trail by one barrier). Shares only: the stamps' lgkmcnt(0) fences change the timing.

  ACTH_LIB=diag/libactalker_hip_stamps.so python tools/ring_stamps.py --only 18,5
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from actalker_amd import _lib  # noqa: E402
from tools.bench_gemm import SHAPES, run  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="18")
    ap.add_argument("--tile", type=int, default=0)
    ap.add_argument("--flags", type=lambda s: int(s, 0), default=0, help="extra tile flag bits (diagnostics)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.load()
    for idx in [int(i) for i in a.only.split(",")]:
        mode, M, N, K, act = SHAPES[idx]
        run(mode, M, N, K, act, a.tile | a.flags, 3, dev)
        run(mode, M, N, K, act, a.tile | a.flags | 0x400, 1, dev)
        buf = (ctypes.c_ulonglong * (4096 * 4))()
        _lib.check(lib.acth_debug_gemm_stamps(buf, 4096), "stamps")
        st = np.frombuffer(buf, dtype=np.uint64).reshape(512, 8, 4).astype(np.float64)
        ok = st.sum(axis=(1, 2)) > 0
        st = st[ok] / ((K + 31) // 32)
        e, l_ = st[:, :4].mean(axis=(0, 1)), st[:, 4:].mean(axis=(0, 1))
        names = ("read+DMA", "barrier1", "MFMA", "barrier2")
        print(f"[{idx}] {mode} {M}x{N}x{K} flags {a.flags:#x}: {ok.sum()} WGs; cycles per 32-deep sub-tile", flush=True)
        print("   early waves: " + ", ".join(f"{n} {v:.0f}" for n, v in zip(names, e)) + f"; total {e.sum():.0f}")
        print("   late waves:  " + ", ".join(f"{n} {v:.0f}" for n, v in zip(names, l_)) + f"; total {l_.sum():.0f}")
        per_wave = st.sum(axis=2)
        print(f"   per-wave totals: min {per_wave.min():.0f} max {per_wave.max():.0f}")


if __name__ == "__main__":
    main()
