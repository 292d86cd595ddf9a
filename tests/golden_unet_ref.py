"""Cases of the REFERENCE-RUN UNet forward goldens, shared by
tools/gen_golden_unet_ref.py (runs the reference's own UNet package on the CPU) and the tests.

The fixtures pin the reference's orchestration -- unet_spatio_temporal_condition_mambaID_v10_two_ip.py
:362-517, unet_3d_blocks.py:2047-2592, TransformerSTmodel.py:4001-4155 (and the plain mid transformer
:200-421), attention.py:223-343 / 418-473, attention_processor.py:1528-1605 / 2747-2934, mamba_layer.py
:1394-1553 / 1902-1986 -- executed unchanged; only the diffusers 0.29.2 leaves (oracle/diffusers_leaves.py)
and mamba-ssm's selective_scan_ref are restatements.

* ``tiny_f25_half`` / ``tiny_f25_mode2``: the same tiny UNet at the reference's shipped window, F = 25 frames
  (config/inference.yaml:4 -> Inference.py:573), B = 2; the temporal attention then spans two 16-frame MFMA
  blocks (acth_temporal_attn's F <= 32 instantiation).
* ``tiny_*``: the full UNet topology (4 down / mid / 4 up blocks, 15 v10 transformers with Mamba, IP
  adapters) at widths 64/128/128/128, heads 1/2/2/2, B = 2 CFG branches x F = 3 frames, latent 16x32
  (128x256 px masks). Mask cases follow the pipeline's gates (pipeline:702-711): mode0 [face, 0] with
  zero VASA tokens, mode1 [0, face] with zero audio tokens, mode2 [ones, ones], half [mouth (lower
  half), expression (upper half)], box [centre box, upper half] (a partial mask whose token rows are
  not whole image rows).
* ``full_half`` / ``full_mode0`` / ``full_mode2``: the real 1.775 B-parameter UNet (widths 320/640/1280/1280,
  heads 5/10/20/20) at 576x1024, B = 1 x F = 2, the inputs and weights of tests/golden_full.py's ``half`` /
  ``mode0`` / ``mode2`` cases, so the same fixtures also pin the oracle's full-geometry outputs.
* ``win14_mode0``: the same UNet at the headline window shape, 576x1024, B = 3 CFG branches x F = 14 frames, mode 0
  (tests/golden_win14.py: the inputs stacked as the reference pipeline stacks one window's uncond / drop audio+vasa /
  drop vasa branches).
* ``win14_mode2``: the same window in mode 2 (gate [1, 1], masks [mouth, exp]), B = 4 CFG branches x F = 14 -- the
  C4 / C5 workload's UNet call. Generated as four batch-1 reference forwards (batch elements are independent in the
  UNet; one B = 4 fp32 call at this size would not fit the build host's memory), concatenated.
* ``win14_mode1``: the same window in mode 1 (expression-only, gate [0, 1], masks [0, face]): the reference run for
  the distinct branches 0, 1, 3 (branch 2's gated inputs are bitwise branch 1's), batch-1 forwards.
* ``win25_mode0``: the mode-0 window at the reference's shipped length, F = 25 (config/inference.yaml:4), 576x1024,
  B = 3 CFG branches, batch-1 forwards.
* ``c1win14_mode0``: the mode-0 window call at BASELINE C1's geometry, 576x576, F = 14, B = 3, batch-1 forwards.
* ``c1_face0``: the same UNet at BASELINE C1's geometry, 576x576 (latent 72x72; levels 72x72 / 36x36 / 18x18 /
  9x9), B = 1 x F = 2, mode 0 (gate [1, 0], zero VASA tokens) with a centre face box as the audio mask.

Weights are actalker_amd.synthetic values by parameter name (reference names: the key sets are equal,
tests/test_checkpoint_cpu.py), regenerated from the seed on every host; the fixtures hold outputs and
checksums only.
"""
import math

import torch

TINY_CFG = dict(block_out_channels=(64, 128, 128, 128), num_attention_heads=(1, 2, 2, 2), cross_attention_dim=1024,
                layers_per_block=2, num_frames=3)
TINY_SEED = 5
TINY_B, TINY_F, TINY_H, TINY_W = 2, 3, 16, 32
TINY_CASES = ("tiny_mode0", "tiny_mode1", "tiny_mode2", "tiny_half", "tiny_box", "tiny_f25_half", "tiny_f25_mode2")
# the reference's shipped window: config/inference.yaml:4 n_sample_frames = 25 -> Inference.py:573 frames_per_batch,
# so every temporal block (attention.py:431-433, the temporal ResBlocks' (3,1,1) convs and GroupNorm) spans 25 frames
F25 = 25
FULL_CASES = ("full_half", "full_mode0", "full_mode2", "c1_face0", "win14_mode0", "win14_mode1", "win14_mode2",
              "win25_mode0", "c1win14_mode0")
# reference forward run one batch element at a time
PER_ELEMENT = ("win14_mode1", "win14_mode2", "win25_mode0", "c1win14_mode0")
# batch elements a per-element case runs (default: all); win14_mode1's element 2 is bitwise element 1's input
ELEMENTS = {"win14_mode1": (0, 1, 3)}
CASES = TINY_CASES + FULL_CASES
SIGMA = 1.6555  # Karras step 12 of 25; t = 0.25 ln sigma


def tiny_inputs(case: str, seed: int = 23):
    g = torch.Generator().manual_seed(seed)
    B, F, h, w = TINY_B, TINY_F, TINY_H, TINY_W
    if case.startswith("tiny_f25_"):
        F = F25
        case = "tiny_" + case[len("tiny_f25_"):]
    sample = torch.randn(B, F, 8, h, w, generator=g)
    t = torch.tensor(0.25 * math.log(SIGMA))
    ide = torch.randn(B * F, 1, 1024, generator=g)
    aud = torch.randn(B * F, 32, 1024, generator=g)
    vas = torch.randn(B * F, 1, 1024, generator=g)
    pose = 0.1 * torch.randn(B, F, TINY_CFG["block_out_channels"][0], h, w, generator=g)
    added = torch.tensor([[12.5, 12.0, 20.0]] * B)
    Hp, Wp = 8 * h, 8 * w
    one, zero = torch.ones(1, 1, Hp, Wp), torch.zeros(1, 1, Hp, Wp)
    face = zero.clone()
    face[..., Hp // 4: 3 * Hp // 4, 5 * Wp // 16: 11 * Wp // 16] = 1.0
    lower = zero.clone()
    lower[..., Hp // 2:, :] = 1.0
    kind = case.split("_", 1)[1]
    if kind == "mode0":
        masks, vas = [face, zero], torch.zeros_like(vas)
    elif kind == "mode1":
        masks, aud = [zero, face], torch.zeros_like(aud)
    elif kind == "mode2":
        masks = [one, one]
    elif kind == "half":
        masks = [lower, 1.0 - lower]
    elif kind == "box":
        masks = [face, 1.0 - lower]
    else:
        raise ValueError(case)
    return sample, t, (ide, [aud, vas]), added, pose, masks


def case_inputs(case: str):
    if case in TINY_CASES:
        return tiny_inputs(case)
    from tests import golden_full as gf
    if case in ("full_half", "full_mode0", "full_mode2"):
        return gf.case_inputs(case.split("_", 1)[1])
    if case == "c1_face0":
        return gf.case_inputs("face0", h_px=576, w_px=576)
    if case.startswith("win14_mode") or case.startswith("win25_mode"):
        from tests import golden_win14 as gw
        return gw.reference_inputs(mode=int(case[-1]), frames=int(case[3:5]))
    if case == "c1win14_mode0":
        from tests import golden_win14 as gw
        return gw.reference_inputs(mode=0, frames=14, w_px=576)
    raise ValueError(case)


def build_hip_unet(case: str):
    """The product UNet with the case's synthetic weights (CPU; caller moves it)."""
    if case in FULL_CASES:
        from tests import golden_full as gf
        return gf.build_full_unet()
    from actalker_amd.synthetic import init_synthetic_
    from actalker_amd.unet_spatio_temporal_condition_mambaID_v10_two_ip import (UNetSpatioTemporalConditionModel,
                                                                               add_ip_adapters)
    torch.manual_seed(0)
    unet = UNetSpatioTemporalConditionModel(**TINY_CFG)
    add_ip_adapters(unet, [32, 32], [1.25, 1.25])
    init_synthetic_(unet, TINY_SEED)
    return unet


def oracle_cfg(case: str):
    if case in FULL_CASES:
        return None
    return dict(block_out_channels=TINY_CFG["block_out_channels"], num_attention_heads=TINY_CFG["num_attention_heads"])
