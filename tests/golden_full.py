"""Inputs of the full-geometry UNet parity cases (BASELINE C2-C4 shapes: 576x1024 -> latent 72x128,
block widths 320/640/1280/1280, 5/10/20/20 heads, Mamba scans of length 9249 / 2337 / 609), shared by
tools/gen_golden_full.py (oracle fixtures, generated on the CPU) and tests/test_full_geometry_gpu.py.

Everything is regenerated from seeds (the weights by actalker_amd.synthetic, the inputs here), so only
the oracle outputs and input checksums are committed (tests/golden/unet_full_<case>.safetensors)."""
import math

import torch

H_PX, W_PX = 576, 1024
WEIGHT_SEED = 72589
B, F = 1, 2
# timestep of a mid-schedule step (Karras step 12 of 25: sigma ~ 1.66, t = 0.25 ln sigma)
SIGMA = 1.6555
CASES = ("mode0", "mode1", "mode2", "half")


def build_full_unet(seed=WEIGHT_SEED):
    from actalker_amd.synthetic import init_synthetic_
    from actalker_amd.unet_spatio_temporal_condition_mambaID_v10_two_ip import (UNetSpatioTemporalConditionModel,
                                                                               add_ip_adapters)
    with torch.device("meta"):
        unet = UNetSpatioTemporalConditionModel(num_frames=25)
    unet = unet.to_empty(device="cpu")
    add_ip_adapters(unet, [32, 32], [1.25, 1.25])
    init_synthetic_(unet, seed)
    return unet


def case_inputs(case: str, seed: int = 11, h_px: int = H_PX, w_px: int = W_PX):
    """(sample, t, ehs, added, pose, masks) for one case; masks follow the pipeline's gates
    (pipeline:702-711): mode0 [face, 0] with zero VASA tokens, mode1 [0, face] with zero audio
    tokens, mode2 [ones, ones], half = [mouth (lower half), expression (upper half)] under gate [1, 1],
    face0 = mode 0 with a centre face box instead of an all-ones face. h_px x w_px: the pixel geometry
    (576x1024 = BASELINE C2-C5; 576x576 = C1)."""
    H_PX, W_PX = h_px, w_px
    g = torch.Generator().manual_seed(seed)
    h, w = H_PX // 8, W_PX // 8
    sample = torch.randn(B, F, 8, h, w, generator=g)
    t = torch.tensor(0.25 * math.log(SIGMA))
    ide = torch.randn(B * F, 1, 1024, generator=g)
    aud = torch.randn(B * F, 32, 1024, generator=g)
    vas = torch.randn(B * F, 1, 1024, generator=g)
    pose = 0.1 * torch.randn(B, F, 320, h, w, generator=g)
    added = torch.tensor([[12.5, 12.0, 20.0]] * B)
    one, zero = torch.ones(1, 1, H_PX, W_PX), torch.zeros(1, 1, H_PX, W_PX)
    lower = zero.clone()
    lower[..., H_PX // 2:, :] = 1.0
    if case == "mode0":
        masks, vas = [one, zero], torch.zeros_like(vas)
    elif case == "face0":
        face = zero.clone()
        face[..., H_PX // 4: 3 * H_PX // 4, 5 * W_PX // 16: 11 * W_PX // 16] = 1.0
        masks, vas = [face, zero], torch.zeros_like(vas)
    elif case == "mode1":
        masks, aud = [zero, one], torch.zeros_like(aud)
    elif case == "mode2":
        masks = [one, one]
    elif case == "half":
        masks = [lower, 1 - lower]
    else:
        raise ValueError(case)
    return sample, t, (ide, [aud, vas]), added, pose, masks


def checksum(*ts):
    """Order-sensitive fp64 fingerprint of tensors (guards that the box regenerates the same weights
    and inputs): per tensor its sum, sum of squares and a position-weighted sum over a stride-97
    subsample, each tensor's terms weighted by its position in the list."""
    acc = torch.zeros(3, dtype=torch.float64)
    for j, x in enumerate(ts):
        x = x.detach().flatten()
        sub = x[::97].double()
        i = torch.arange(sub.numel(), dtype=torch.float64)
        part = torch.stack([x.double().sum(), x.double().pow(2).sum(), (sub * torch.cos(i * 0.001)).sum()])
        acc += part * (1.0 + 1e-3 * j)
    return acc
