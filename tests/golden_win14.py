"""The headline window shape pinned by a reference run (VERDICT r4 "what's weak" 1 / next item 2): one 14-frame
window at 576x1024 (latent 72x128), the three CFG branches the benched mode-0 step evaluates for it -- uncond,
drop audio+vasa, drop vasa (= cond under gate [1, 0]; pipeline:162-200) -- in ONE UNet call, exactly as
``pipeline.HipBackend.run_units`` builds it (window input scaling, CFG prefix sharing between branches 1 and 2,
batched per-call context projections, automatic units-per-call).

Shared by tools/gen_golden_unet_ref.py (case ``win14_mode0``: the REFERENCE UNet package run by path on the CPU,
B = 3 x F = 14, inputs stacked as the reference pipeline stacks them at pipeline:712-729) and
tests/test_full_geometry_gpu.py (the HIP backend's call on the same tensors, each unit held to its golden batch
element).
"""
import math

import torch

H_PX, W_PX = 576, 1024
H, W = H_PX // 8, W_PX // 8
F = 14
NB = 3                   # CFG branches of the window: 0 uncond, 1 drop audio+vasa, 2 drop vasa (cond audio)
GATE = [1, 0]            # mode 0 (audio-only): VASA prompts gated to zero (pipeline:724)
SIGMA = 1.6555           # Karras step 12 of 25
SEED = 17


def loop_tensors(seed: int = SEED):
    """The pipeline-internal tensors after CFG stacking (pipeline:128-205, 636-638) for one window of F frames:
    (lat (1, F, 4, h, w) noisy latents, imgl (NB, F, 4, h, w), ide (NB, F, 1, 1024), aud (NB, F, 32, 1024),
    vas (NB, F, 1, 1024), pose (1, F, 320, h, w), added (NB, 3), masks (face, mouth, exp))."""
    g = torch.Generator().manual_seed(seed)
    lat = SIGMA * torch.randn(1, F, 4, H, W, generator=g) + 0.18215 * torch.randn(1, 1, 4, H, W, generator=g)
    il = torch.randn(1, 1, 4, H, W, generator=g).expand(1, F, 4, H, W)
    imgl = torch.cat([torch.zeros_like(il), il, il]).contiguous()
    e = torch.randn(1, 1, 1, 1024, generator=g).expand(1, F, 1, 1024)
    ide = torch.cat([torch.zeros_like(e), e, e]).contiguous()
    a_u, a_c = torch.randn(1, F, 32, 1024, generator=g), torch.randn(1, F, 32, 1024, generator=g)
    aud = torch.cat([a_u, a_u, a_c]).contiguous()
    v_u = torch.randn(1, F, 1, 1024, generator=g)
    vas = torch.cat([v_u, v_u, v_u]).contiguous()
    pose = 0.1 * torch.randn(1, F, 320, H, W, generator=g)
    added = torch.tensor([[12.5, 12.0, 20.0]] * NB)
    face = torch.zeros(1, 1, H_PX, W_PX)
    face[..., H_PX // 4: 3 * H_PX // 4, 5 * W_PX // 16: 11 * W_PX // 16] = 1.0
    mouth = torch.zeros(1, 1, H_PX, W_PX)
    mouth[..., H_PX // 2:, :] = 1.0
    return lat, imgl, ide, aud, vas, pose, added, (face, mouth, 1.0 - mouth)


def reference_inputs(seed: int = SEED):
    """The reference pipeline's UNet call on these tensors (pipeline:712-729): scale_model_input (x / sqrt(sigma^2
    + 1)), image latents concatenated on channels, prompts flattened and gated, pose repeated per branch, the
    gate's masks [face, 0] (pipeline:702-711). Returns (sample, t, ehs, added, pose, masks)."""
    lat, imgl, ide, aud, vas, pose, added, (face, mouth, exp) = loop_tensors(seed)
    x = (lat / math.sqrt(SIGMA * SIGMA + 1.0)).repeat(NB, 1, 1, 1, 1)
    sample = torch.cat([x, imgl], dim=2)
    t = torch.tensor(0.25 * math.log(SIGMA))
    ehs = (ide.flatten(0, 1), [aud.flatten(0, 1) * GATE[0], vas.flatten(0, 1) * GATE[1]])
    masks = [face, torch.zeros_like(face)]
    return sample, t, ehs, added, pose.repeat(NB, 1, 1, 1, 1), masks
