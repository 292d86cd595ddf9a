"""Reference point for the GEMM main loop: acth_gemm (auto tile) against torch.matmul (hipBLASLt on ROCm) on the
UNet's dense shapes, plain products (no epilogue operands), bf16, same data. Diagnostic only.

  python tools/bench_blas.py [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from actalker_amd import ops  # noqa: E402

SHAPES = [(774144, 320, 320), (774144, 960, 320), (193536, 640, 640), (193536, 1920, 640), (48384, 1280, 1280),
          (48384, 3840, 1280), (193536, 5120, 640), (48384, 10240, 1280), (774144, 2560, 320), (4096, 4096, 4096),
          (8192, 8192, 8192)]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for M, N, K in SHAPES:
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        t_ours = timeit(lambda: ops.gemm(x, w), a.iters)
        t_blas = timeit(lambda: torch.matmul(x, w.t(), out=out), a.iters)
        fl = 2.0 * M * N * K
        print(f"{M:7d} x {N:5d} x {K:5d}: acth_gemm {t_ours * 1e3:8.1f} us {fl / t_ours / 1e9:7.1f} TF/s | "
              f"hipBLASLt {t_blas * 1e3:8.1f} us {fl / t_blas / 1e9:7.1f} TF/s", flush=True)
        del x, w, out


if __name__ == "__main__":
    main()
