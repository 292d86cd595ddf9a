"""BASELINE C1 workload (BASELINE.json configs[0]): mode 0 (audio only, gate [1, 0]), 14 frames, 25 steps, at
the geometry the reference's preprocessing makes of assets/ref.jpg -- a 576x576 crop
(src/dataset/test_preprocess.py:278-282), latent 72x72, so the UNet levels are 72x72 / 36x36 / 18x18 / 9x9.

Shared by tools/gen_golden_c1.py (the fp32 oracle loop on the CPU, hours; writes
tests/golden/c1_loop25_mode0.safetensors) and the GPU tests (the HIP loop on exactly this workload, and one
reference-run UNet call at this geometry, tests/golden_unet_ref.py case ``c1_mode0``).

The loop settings are config/inference.yaml's: frames_per_batch 14 (BASELINE), overlap 0, shift_offset 7,
guidance (min = max) appearance 2.0 / audio 7.5 / vasa 3, fps 12.5, motion buckets 12 / 20. Inputs are synthetic
(seeded; no assets are decoded here: librosa / cv2 / the Whisper and ArcFace weights are absent), stacked as the
pipeline stacks them (pipeline:162-205: ID [0, e, e, e], image latents [0, l, l, l], audio [u, u, a, a],
VASA [u, u, u, v], the last fpb frames of audio / VASA the uncond pad :176-181), with a face box, mouth (lower
half) and expression (upper half) mask at 576x576. Weights: the full-size synthetic UNet of tests/golden_full.py.
"""
import torch

N, FPB, H, W = 14, 14, 72, 72
H_PX, W_PX = 8 * H, 8 * W
SHIFT, OVERLAP = 7, 0
GATE = [1, 0]
GUIDANCE = (2.0, 7.5, 3.0)
ADDED = [12.5, 12.0, 20.0]
INPUT_SEED = 2025


def loop_inputs(seed: int = INPUT_SEED):
    """(latents_all, image_latents, image_embeddings, audio_prompts, vasa_prompts, pose_fea, added_time_ids,
    (face, mouth, exp) masks) in the oracle loop's shapes (oracle.reference_cpu.denoise_loop)."""
    g = torch.Generator().manual_seed(seed)
    T = N + FPB
    ref_lat = 0.18215 * torch.randn(1, 1, 4, H, W, generator=g)
    latents = ref_lat + 700.0 * torch.randn(1, T, 4, H, W, generator=g)      # add_noise at sigma_max (:586-598)
    il = torch.randn(1, T, 4, H, W, generator=g)
    imgl = torch.cat([torch.zeros_like(il), il, il, il])
    e = torch.randn(1, 1, 1, 1024, generator=g).expand(1, T, 1, 1024)        # one ID embedding for all frames
    ide = torch.cat([torch.zeros_like(e), e, e, e])
    a_u = torch.randn(1, N, 32, 1024, generator=g)
    a_c = torch.randn(1, N, 32, 1024, generator=g)
    pad_a = a_u[:, :1].expand(1, FPB, 32, 1024)
    a_u, a_c = torch.cat([a_u, pad_a], 1), torch.cat([a_c, pad_a], 1)
    aud = torch.cat([a_u, a_u, a_c, a_c])
    v_u = torch.randn(1, N, 1, 1024, generator=g)
    v_c = torch.randn(1, N, 1, 1024, generator=g)
    pad_v = v_u[:, :1].expand(1, FPB, 1, 1024)
    v_u, v_c = torch.cat([v_u, pad_v], 1), torch.cat([v_c, pad_v], 1)
    vas = torch.cat([v_u, v_u, v_u, v_c])
    pose = 0.1 * torch.randn(1, N, 320, H, W, generator=g)                   # N pose frames: indexed mod N
    added = torch.tensor([ADDED] * 4)
    face = torch.zeros(1, 1, H_PX, W_PX)
    face[..., H_PX // 4: 3 * H_PX // 4, 5 * W_PX // 16: 11 * W_PX // 16] = 1.0
    mouth = torch.zeros(1, 1, H_PX, W_PX)
    mouth[..., H_PX // 2:, :] = 1.0
    return (latents, imgl, ide.contiguous(), aud.contiguous(), vas.contiguous(), pose, added,
            (face, mouth, 1.0 - mouth))


def inputs_checksum():
    from tests import golden_full as gf
    latents, imgl, ide, aud, vas, pose, added, masks = loop_inputs()
    return gf.checksum(latents, imgl, ide, aud, vas, pose, added, *masks)
