"""Deterministic synthetic weights / inputs for the golden SS2D_cond_v10 cases.

Shared by tools/gen_golden.py (which runs the reference module) and the tests (which run the
oracle and the HIP path on the same weights). Weights are a pure function of (seed, names, shapes):
one CPU torch.Generator walks the parameter names in sorted order.
"""
from __future__ import annotations

import math
from typing import Dict, Tuple

import torch

CASES = {
    # toy width, all three pipeline modes plus a partial (half-face) mask pair
    "toy_mode2": dict(seed=11, d_model=32, d_cond=64, BF=3, S=24, mask_hw=(8, 12), masks="ones_ones"),
    "toy_mode0": dict(seed=12, d_model=32, d_cond=64, BF=3, S=24, mask_hw=(8, 12), masks="ones_zeros"),
    "toy_half": dict(seed=13, d_model=32, d_cond=64, BF=2, S=24, mask_hw=(8, 12), masks="lower_upper"),
    # real level-0 width (C=320, d_cond=1024), mid-block token count geometry (9x16)
    "c320_mode2": dict(seed=21, d_model=320, d_cond=1024, BF=2, S=144, mask_hw=(72, 128), masks="ones_ones"),
    "c320_mode1": dict(seed=22, d_model=320, d_cond=1024, BF=2, S=144, mask_hw=(72, 128), masks="zeros_ones"),
    "c320_half": dict(seed=23, d_model=320, d_cond=1024, BF=2, S=144, mask_hw=(72, 128), masks="lower_upper"),
    "c320_mode0": dict(seed=24, d_model=320, d_cond=1024, BF=2, S=144, mask_hw=(72, 128), masks="ones_zeros"),
}

# Level shapes of the BASELINE geometry: the real 576x1024 masks downsampled to the
# level's token grid (72x128 / 36x64 / 18x32, mamba_layer.py:1962-1981) and the real sequence lengths
# (L = S + 33 audio / S + 2 expression). Inputs are regenerated from the seed; the fixtures
# (tests/golden/ss2d_level_<case>.safetensors) hold the reference output at every ``sub``-th token row,
# the input checksum and the selected-token counts.
LEVEL_CASES = {
    "l0_mode2": dict(seed=31, d_model=320, d_cond=1024, BF=1, S=9216, mask_hw=(576, 1024), masks="ones_ones", sub=7),
    "l0_mode0": dict(seed=32, d_model=320, d_cond=1024, BF=1, S=9216, mask_hw=(576, 1024), masks="ones_zeros", sub=7),
    "l0_box": dict(seed=33, d_model=320, d_cond=1024, BF=2, S=9216, mask_hw=(576, 1024), masks="box_upper", sub=7),
    "l1_half": dict(seed=34, d_model=640, d_cond=1024, BF=2, S=2304, mask_hw=(576, 1024), masks="lower_upper", sub=3),
    "l1_box": dict(seed=35, d_model=640, d_cond=1024, BF=1, S=2304, mask_hw=(576, 1024), masks="lower_box", sub=3),
    "l2_mode2": dict(seed=36, d_model=1280, d_cond=1024, BF=2, S=576, mask_hw=(576, 1024), masks="ones_ones", sub=1),
    "l2_mode1": dict(seed=37, d_model=1280, d_cond=1024, BF=2, S=576, mask_hw=(576, 1024), masks="zeros_ones", sub=1),
    "l2_box": dict(seed=38, d_model=1280, d_cond=1024, BF=1, S=576, mask_hw=(576, 1024), masks="box_lower", sub=1),
}


def golden_weights(seed: int, shapes: Dict[str, Tuple[int, ...]]) -> Dict[str, torch.Tensor]:
    g = torch.Generator().manual_seed(seed)
    out = {}
    for k in sorted(shapes):
        shp = shapes[k]
        leaf = k.rsplit(".", 1)[-1]
        if leaf == "A_logs":
            t = torch.log(torch.arange(1, shp[-1] + 1, dtype=torch.float32)).expand(shp).clone()
            t += 0.1 * torch.randn(shp, generator=g)
        elif leaf == "Ds":
            t = 1.0 + 0.1 * torch.randn(shp, generator=g)
        elif leaf == "dt_projs_bias":
            dt = torch.exp(torch.rand(shp, generator=g) * (math.log(0.1) - math.log(0.001)) + math.log(0.001))
            t = dt + torch.log(-torch.expm1(-dt))
        elif leaf == "dt_projs_weight":
            r = shp[-1]
            t = (torch.rand(shp, generator=g) * 2 - 1) * r ** -0.5
        elif len(shp) == 1 and "norm" in k and leaf == "weight":
            t = 1.0 + 0.1 * torch.randn(shp, generator=g)
        elif len(shp) == 1:
            t = 0.1 * torch.randn(shp, generator=g)
        else:
            t = torch.randn(shp, generator=g) / math.sqrt(shp[-1])
        out[k] = t.float().contiguous()
    return out


def _mask(kind: str, hw):
    H, W = hw
    m = torch.zeros(1, 1, H, W)
    if kind == "ones":
        m[:] = 1.0
    elif kind == "lower":
        m[..., H // 2:, :] = 1.0
    elif kind == "upper":
        m[..., : H // 2, :] = 1.0
    elif kind == "box":                      # a face box whose edges fall between latent rows / columns
        m[..., int(0.26 * H): int(0.74 * H), int(0.33 * W): int(0.69 * W)] = 1.0
    return m


def make_masks(case):
    a, e = case["masks"].split("_")
    return [_mask(a, case["mask_hw"]), _mask(e, case["mask_hw"])]


def make_inputs(case):
    g = torch.Generator().manual_seed(case["seed"] + 1000)
    BF, S, C, Dc = case["BF"], case["S"], case["d_model"], case["d_cond"]
    x = torch.randn(BF, S, C, generator=g)
    id_emb = torch.randn(BF, 1, Dc, generator=g)
    conds = torch.randn(BF, 33, Dc, generator=g)
    return x, id_emb, conds, make_masks(case)
