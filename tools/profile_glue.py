"""Where the torch glue of a sampler step comes from: one bench-configuration step (mode 0, 576x1024, N = 14)
under torch.profiler, the aten ops that launch copy / fill / cat / index kernels grouped by their Python call
site. Diagnostic only (not part of the product or the bench).

    python tools/profile_glue.py [--mode 0] [--top 40]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    from actalker_amd import pipeline as pl
    dev = torch.device("cuda", 0)
    unet = bench.build_unet(dev).to(dev)
    gate, _ = bench.MODES[args.mode]
    N, fpb, H, W = 14, 14, 576, 1024
    inp = bench.synthetic_inputs(N, fpb, H, W, args.mode)
    be = pl.HipBackend(unet, H // 8, W // 8, inp["masks"], gate, inp["added"], N + fpb, fpb, inp["image_latents"],
                       inp["image_embeddings"], inp["audio_prompts"], inp["vasa_prompts"], inp["pose_fea"])
    cfg = pl.LoopConfig(num_frames=N, frames_per_batch=fpb, overlap=0, shift_offset=7)
    with torch.no_grad():
        pl.denoise(be, inp["latents"], cfg, steps=2)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        with torch.no_grad():
            pl.denoise(be, inp["latents"], cfg, steps=2)
        torch.cuda.synchronize()
    names = ("aten::copy_", "aten::fill_", "aten::zero_", "aten::cat", "aten::index_select", "aten::index",
             "aten::clone", "aten::contiguous", "aten::to", "aten::_to_copy", "aten::repeat_interleave",
             "aten::eq", "aten::all", "aten::mul", "aten::add", "aten::zeros", "aten::full", "aten::item",
             "aten::_local_scalar_dense", "aten::nonzero", "aten::repeat", "aten::arange", "aten::sigmoid")
    ka = prof.key_averages(group_by_stack_n=6)
    rows = [e for e in ka if e.key in names]
    rows.sort(key=lambda e: -e.count)
    print(f"{'op':28s} {'count/2 steps':>14s}  stack")
    for e in rows[:args.top]:
        stack = " <- ".join(s.replace(ROOT + "/", "") for s in (e.stack or [])[:6] if "/torch/" not in s)
        print(f"{e.key:28s} {e.count:14d}  {stack}")


if __name__ == "__main__":
    main()
