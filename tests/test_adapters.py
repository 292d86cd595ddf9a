"""Conditioning adapters: AudioProjModel, IDProjModel, VasaProjModel,
PoseGuider (Inference.py:72-78).

Pinning: tests/golden/adapters_*.safetensors hold outputs of the REFERENCE modules
(src/models/audio_adapter/{audio_proj,pose_guider}.py, run by tools/gen_golden_adapters.py) on
seeded inputs with ``actalker_amd.synthetic`` weights. The CPU oracle restatement must match them
to fp32 rounding; the HIP path (bf16 activations, fp32 accumulation) must match them within the
tolerances below (relative L2).
"""
import json
import os

import pytest
import torch
from safetensors.torch import load_file

from actalker_amd.synthetic import synthetic_state_dict
from oracle import reference_cpu as ref
from tests.adapter_cases import ADAPTER_CASES, adapter_input

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TOL_GPU = {"audio_proj": 2e-2, "id_proj": 2e-2, "vasa_proj": 2e-2, "pose_guider": 3e-2, "pose_guider_odd": 3e-2}


def _product_module(case):
    from actalker_amd import adapters
    return getattr(adapters, case["cls"])(**case["kwargs"])


def _weights(case):
    m = _product_module(case)
    return synthetic_state_dict(case["seed"], {k: tuple(v.shape) for k, v in m.state_dict().items()}), m


def _oracle(case, sd, x):
    cls = case["cls"]
    if cls == "AudioProjModel":
        return ref.audio_proj_model(sd, "", x, case["kwargs"]["context_tokens"])
    if cls == "IDProjModel":
        return ref.id_proj_model(sd, "", x)
    if cls == "VasaProjModel":
        return ref.vasa_proj_model(sd, "", x)
    return ref.pose_guider(sd, "", x, n_blocks=2 * (len(case["kwargs"]["block_out_channels"]) - 1))


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


def test_golden_index_matches_cases():
    idx = json.load(open(os.path.join(GOLD, "adapters_index.json")))
    assert set(idx) == set(ADAPTER_CASES)
    for k, case in ADAPTER_CASES.items():
        assert idx[k]["seed"] == case["seed"] and idx[k]["in_shape"] == case["in_shape"]


@pytest.mark.parametrize("name", sorted(ADAPTER_CASES))
def test_oracle_matches_reference_golden(name):
    case = ADAPTER_CASES[name]
    g = load_file(os.path.join(GOLD, f"adapters_{name}.safetensors"))
    x = adapter_input(case)
    assert torch.equal(x, g["x"])
    sd, _ = _weights(case)
    y = _oracle(case, sd, x)
    assert y.shape == g["y"].shape
    assert _rel(y, g["y"]) < 1e-5


def test_product_state_dict_names_match_reference():
    # the golden generator loaded the same synthetic state dict into the reference module with
    # strict=True, so equal key sets prove the drop-in names
    for name, case in ADAPTER_CASES.items():
        sd, m = _weights(case)
        m.load_state_dict(sd, strict=True)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(ADAPTER_CASES))
def test_adapter_gpu_matches_reference_golden(dev, name):
    case = ADAPTER_CASES[name]
    g = load_file(os.path.join(GOLD, f"adapters_{name}.safetensors"))
    sd, m = _weights(case)
    m.load_state_dict(sd, strict=True)
    m = m.to(dev)
    y = m(g["x"].to(dev))
    torch.cuda.synchronize()
    assert y.shape == g["y"].shape
    assert torch.isfinite(y.float()).all()
    err = _rel(y.cpu(), g["y"])
    assert err < TOL_GPU[name], f"{name}: rel-L2 {err:.3e}"


@pytest.mark.gpu
def test_pose_guider_full_resolution_vs_oracle(dev):
    """Full 576x1024 pose frames (the PoseGuider's real input size) through every layer."""
    case = dict(ADAPTER_CASES["pose_guider"], in_shape=[1, 3, 2, 576, 1024])
    sd, m = _weights(case)
    m.load_state_dict(sd, strict=True)
    x = torch.rand(1, 3, 2, 576, 1024, generator=torch.Generator().manual_seed(7))
    y = m.to(dev)(x.to(dev))
    torch.cuda.synchronize()
    want = _oracle(case, sd, x)
    assert y.shape == (1, 320, 2, 72, 128)
    assert _rel(y.cpu(), want) < 3e-2


@pytest.mark.gpu
def test_conv_direct_kernel_vs_torch(dev):
    """acth_conv_direct against torch fp32 convs: Cin 3/16/96, stride 1/2, Cout 3/16/96, temporal taps."""
    from actalker_amd import ops
    torch.manual_seed(0)
    for cin, cout, stride, H, W in ((3, 16, 1, 33, 47), (16, 32, 2, 40, 64), (96, 96, 1, 18, 32), (128, 3, 1, 16, 24),
                                    (96, 256, 2, 19, 31)):
        B = 2
        x = torch.randn(B, cin, H, W)
        w = torch.randn(cout, cin, 3, 3) / (9 * cin) ** 0.5
        b = 0.1 * torch.randn(cout)
        want = torch.nn.functional.silu(torch.nn.functional.conv2d(x, w, b, stride=stride, padding=1))
        xt = ops.nchw_to_tokens(x.to(dev))
        y = ops.conv_direct(xt, ops.pack_conv_direct(w).to(dev), b.to(dev), B=B, H=H, W=W, stride=stride,
                            act=ops.ACT_SILU)
        got = ops.tokens_to_nchw(y, B, want.shape[2], want.shape[3]).cpu()
        assert _rel(got, want) < 1e-2, (cin, cout, stride)
    # temporal (3,1,1) taps over F frames, fp32 output
    B, Fr, C, S = 2, 5, 3, 77
    x = torch.randn(B, C, Fr, S)
    w = torch.randn(C, C, 3, 1, 1) / 3.0
    b = 0.1 * torch.randn(C)
    want = torch.nn.functional.conv3d(x[..., None], w, b, padding=(1, 0, 0))[..., 0]        # (B, C, F, S)
    xt = x.permute(0, 2, 3, 1).reshape(-1, C).contiguous().to(dev).to(torch.bfloat16)
    y = ops.conv_direct(xt, ops.pack_conv_direct(w).to(dev), b.to(dev), B=B, temporal=dict(F=Fr, S=S), out_f32=True)
    got = y.cpu().view(B, Fr, S, C).permute(0, 3, 1, 2)
    assert _rel(got, want) < 1e-2


@pytest.mark.gpu
def test_vasa_proj_1018_wide(dev):
    """VasaProjModel(512, vasa_expression_dim=1018) as Inference.py:78 builds it (width % 8 != 0)."""
    from actalker_amd.adapters import VasaProjModel
    m = VasaProjModel(512, 1018)
    sd = synthetic_state_dict(36, {k: tuple(v.shape) for k, v in m.state_dict().items()})
    m.load_state_dict(sd)
    x = torch.randn(5, 512, generator=torch.Generator().manual_seed(8))
    y = m.to(dev)(x.to(dev))
    assert y.shape == (5, 1018)
    assert _rel(y.cpu(), ref.vasa_proj_model(sd, "", x)) < 2e-2


@pytest.mark.gpu
def test_softmax_rows_vs_torch(dev):
    from actalker_amd import ops
    torch.manual_seed(1)
    for rows, cols, scale in ((7, 9216, 0.044), (3, 100, 1.0), (5, 1, 0.5)):
        x = 20 * torch.randn(rows, cols)
        y = ops.softmax_rows(x.to(dev), scale).float().cpu()
        want = torch.softmax(scale * x, -1)
        assert (y - want).abs().max().item() < 4e-3
        assert torch.allclose(y.sum(-1), torch.ones(rows), atol=2e-2)
