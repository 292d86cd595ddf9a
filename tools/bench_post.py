"""Timing of the stages around the denoising loop at the BASELINE shape (576x1024, N = 14 -> T = 28
latent frames): PoseGuider over the N pose frames, the adapter MLPs, the VAE ref-image encode and
the temporal decode of all T frames in decode_chunk_size chunks (inference.yaml:70 uses 10; 14 =
one window). Random-init weights (no checkpoints offline). Prints one JSON line.

  python tools/bench_post.py [--chunk 10] [--iters 3]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters):
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
    ap.add_argument("--chunk", type=int, default=10)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--frames", type=int, default=14)
    a = ap.parse_args()
    from actalker_amd.adapters import AudioProjModel, IDProjModel, PoseGuider, VasaProjModel
    from actalker_amd.synthetic import init_synthetic_
    from actalker_amd.vae import AutoencoderKLTemporalDecoder, decode_latents
    dev = torch.device("cuda:0")
    N, fpb, H, W = a.frames, 14, 576, 1024
    T = N + fpb
    g = torch.Generator().manual_seed(1)
    vae = init_synthetic_(AutoencoderKLTemporalDecoder(), 61).to(dev)
    pg = init_synthetic_(PoseGuider(320, block_out_channels=(16, 32, 96, 256)), 62).to(dev)
    ap_ = init_synthetic_(AudioProjModel(10, 5, 384, 1024, 1024, 32), 63).to(dev)
    idp = init_synthetic_(IDProjModel(512, 1024, 1024), 64).to(dev)
    vp = init_synthetic_(VasaProjModel(512, 1018), 65).to(dev)
    lat = torch.randn(1, T, 4, H // 8, W // 8, generator=g).to(dev)
    ref = (torch.rand(1, 3, H, W, generator=g) * 2 - 1).to(dev)
    pose = torch.rand(1, 3, N, H, W, generator=g).to(dev)
    audio = torch.randn(1, N, 10, 5, 384, generator=g).to(dev)
    with torch.no_grad():
        out = {
            "decode_ms": timed(lambda: decode_latents(vae, lat, T, a.chunk), a.iters),
            "encode_ms": timed(lambda: vae.encode(ref).latent_dist.mean, a.iters),
            "pose_guider_ms": timed(lambda: pg(pose), a.iters),
            "audio_proj_ms": timed(lambda: ap_(audio), a.iters),
            "id_vasa_proj_ms": timed(lambda: (idp(torch.randn(1, 1, 512, device=dev)),
                                              vp(torch.randn(N, 512, device=dev))), a.iters),
        }
    out.update(frames=N, latent_frames=T, decode_chunk_size=a.chunk, resolution=f"{H}x{W}",
               decode_ms_per_frame=out["decode_ms"] / T)
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in out.items()}))


if __name__ == "__main__":
    main()
