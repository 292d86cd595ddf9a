"""Micro-benchmark of the attention kernels at the UNet's level shapes (random data).

  python tools/bench_attn.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from actalker_amd import ops  # noqa: E402

SHAPES = [(84, 9216, 5), (84, 2304, 10), (84, 576, 20), (84, 144, 20)]   # (frames, tokens, heads): the bench step


def main(iters=5, flash_only=False):
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    for nb, S, H in (SHAPES[:2] if flash_only else SHAPES):
        qkv = torch.randn(nb * S, 3 * H * 64, generator=g).to(dev, torch.bfloat16)
        ops.flash_attn(qkv, nb, S, H)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            ops.flash_attn(qkv, nb, S, H)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / iters
        flops = 4.0 * nb * H * S * S * 64
        print(f"flash_attn nb={nb} S={S} H={H}: {ms:.3f} ms  {flops / ms / 1e9:.1f} TFLOP/s", flush=True)
    if flash_only:
        return
    # temporal attention over the 14 frames of a window (B = 4 CFG branches), HBM-bound
    for S, H in ((9216, 5), (2304, 10), (576, 20)):
        B, F = 4, 14
        qkv = torch.randn(B * F * S, 3 * H * 64, generator=g).to(dev, torch.bfloat16)
        ops.temporal_attn(qkv, B, F, S, H)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            ops.temporal_attn(qkv, B, F, S, H)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / iters
        nbytes = B * F * S * H * 64 * 2 * 4            # q, k, v read + o written
        print(f"temporal_attn S={S} H={H}: {ms:.3f} ms  {nbytes / ms / 1e9:.2f} TB/s", flush=True)


if __name__ == "__main__":
    main(flash_only="--flash" in sys.argv)
