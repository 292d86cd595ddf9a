"""VASA expression / head-pose encoders (actalker_amd.vasa) against the REFERENCE modules of
src/dataset/vasa_feature_v2.py (goldens: tools/gen_golden_vasa.py).

CPU: parameter names and shapes equal the reference's (strict checkpoint loads, Inference.py:154/160).
GPU: outputs on the same seeded weights and images. Tolerance (bf16 activations through 50 / 18 conv
layers, GroupNorm re-normalising each): relative L2 <= 3e-2 on the expression features and pose logits,
|rotation| error <= 1 degree."""
import json
import os

import pytest
import torch
from safetensors.torch import load_file

from tests import golden_vasa as gv

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _models():
    from actalker_amd.vasa import HeadExpression, HeadPose_train
    return HeadExpression(512), HeadPose_train()


def test_vasa_state_dict_layout_matches_reference():
    with open(os.path.join(GOLD, "vasa_keys.json")) as fh:
        want = json.load(fh)
    exp_m, pose_m = _models()
    assert {k: list(v.shape) for k, v in exp_m.state_dict().items()} == want["HeadExpression"]
    assert {k: list(v.shape) for k, v in pose_m.state_dict().items()} == want["HeadPose_train"]


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / b.norm()).item()


@pytest.mark.gpu
def test_vasa_encoders_match_reference(dev):
    g = load_file(os.path.join(GOLD, "vasa_encoders.safetensors"))
    exp_m, pose_m = _models()
    exp_m.load_state_dict(gv.seeded_weights({k: tuple(v.shape) for k, v in exp_m.state_dict().items()}, 1), strict=True)
    pose_m.load_state_dict(gv.seeded_weights({k: tuple(v.shape) for k, v in pose_m.state_dict().items()}, 2),
                           strict=True)
    exp_m, pose_m = exp_m.to(dev), pose_m.to(dev)
    face, pose_img = gv.images()
    feat = exp_m(face.to(dev))
    logits = pose_m.head_pose_net(pose_img.to(dev) * 2 - 1.0)
    pose = pose_m(pose_img.to(dev) * 2 - 1.0)
    assert feat.shape == g["expression"].shape
    assert _rel(feat, g["expression"]) < 3e-2
    assert _rel(logits, g["pose_logits"]) < 3e-2
    assert (pose["rotation"].cpu() - g["rotation"]).abs().max().item() < 1.0
    assert (pose["translation"].cpu() - g["translation"]).abs().max().item() < 2e-2


@pytest.mark.gpu
def test_vasa_prompts_assembly(dev):
    """Inference.py:486-500 composition: vasa_linear(expression ++ 0) ++ [rotation, 0 translation]."""
    from actalker_amd.adapters import VasaProjModel
    from actalker_amd.vasa import vasa_prompts
    exp_m, pose_m = _models()
    exp_m.load_state_dict(gv.seeded_weights({k: tuple(v.shape) for k, v in exp_m.state_dict().items()}, 1), strict=True)
    pose_m.load_state_dict(gv.seeded_weights({k: tuple(v.shape) for k, v in pose_m.state_dict().items()}, 2),
                           strict=True)
    torch.manual_seed(0)
    lin = VasaProjModel(input_dim=512, output_dim=1018)          # Inference.py:78 (1018 + 6 pose = 1024)
    exp_m, pose_m, lin = exp_m.to(dev), pose_m.to(dev), lin.to(dev)
    face, pose_img = gv.images()
    p, u = vasa_prompts(exp_m, pose_m, lin, face.to(dev), pose_img.to(dev))
    assert p.shape == (gv.N_IMG, 1024) and u.shape == (gv.N_IMG, 1024)
    g = load_file(os.path.join(GOLD, "vasa_encoders.safetensors"))
    assert (p[:, -6:-3].cpu() - g["rotation"]).abs().max().item() < 1.0
    assert float(p[:, -3:].abs().max()) == 0.0 and float(u[:, -6:].abs().max()) == 0.0
