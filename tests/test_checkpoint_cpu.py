"""Checkpoint / config surface (Inference.py:41-148, 200-201, 428-433): path resolution, strict loads of
the five ACTalker .pth files, adapter-state merge renumbering, fp32 SSM parameters, diffusers-folder
VAE loading. CPU only (no kernels run)."""
import json
import os

import pytest
import torch

from actalker_amd import checkpoint as ck
from actalker_amd.synthetic import synthetic_state_dict

YAML = """
output_dir: {out}
exp_name: exp
resume_from_checkpoint: {resume}
pose_guider_checkpoint_path: {ckdir}/pose_guider-7.pth
unet_checkpoint_path: {ckdir}/unet-7.pth
audio_linear_checkpoint_path: {ckdir}/audio_linear-7.pth
adapter_module_checkpoint_path: {ckdir}/adapter_module-7.pth
id_proj_checkpoint_path: {ckdir}/id_proj_model-7.pth
vasa_linear_checkpoint_path: {ckdir}/vasa_linear-7.pth
unet_cls: 'src.models.base.unet_spatio_temporal_condition_mambaID_v10_two_ip.UNetSpatioTemporalConditionModel'
weight_dtype: 'fp16'
vasa_expression_dim: 1018
ip_audio_scale: 1.25
data:
  n_sample_frames: 25
"""


def _cfg(tmp_path, resume="False"):
    p = tmp_path / "inference.yaml"
    p.write_text(YAML.format(out=tmp_path / "out", resume=resume, ckdir=tmp_path / "ck"))
    return ck.load_config(str(p))


def test_config_attribute_access(tmp_path):
    cfg = _cfg(tmp_path)
    assert cfg.data.n_sample_frames == 25 and cfg.weight_dtype == "fp16"
    assert ck.weight_dtype_of(cfg) == torch.float16
    assert ck.resolve_unet_cls(cfg.unet_cls).__module__.startswith("actalker_amd.")


def test_resolve_paths_config_step_and_latest(tmp_path):
    assert ck.resolve_checkpoint_paths(_cfg(tmp_path))["unet"].endswith("ck/unet-7.pth")
    cfg = _cfg(tmp_path, resume="136000")
    assert ck.resolve_checkpoint_paths(cfg)["id_proj"].endswith("out/exp/id_proj_model-136000.pth")
    for s in (500, 12000, 3000):
        os.makedirs(tmp_path / "out" / "exp" / f"checkpoint-{s}")
    paths = ck.resolve_checkpoint_paths(_cfg(tmp_path, resume="True"))
    assert paths["adapter_module"].endswith("out/exp/adapter_module-12000.pth")


def _tiny_set():
    from actalker_amd.adapters import AudioProjModel, IDProjModel, PoseGuider, VasaProjModel
    from actalker_amd.unet_spatio_temporal_condition_mambaID_v10_two_ip import (UNetSpatioTemporalConditionModel,
                                                                               add_ip_adapters)
    unet = UNetSpatioTemporalConditionModel(block_out_channels=(64, 128, 128, 128), num_attention_heads=(1, 2, 2, 2),
                                            layers_per_block=2, num_frames=3)
    adapters = add_ip_adapters(unet, [32, 32], [1.25, 1.25])
    return (unet, adapters, PoseGuider(64, block_out_channels=(16, 32, 96, 256)),
            AudioProjModel(seq_len=2, blocks=5, channels=16, intermediate_dim=64, output_dim=1024, context_tokens=4),
            IDProjModel(512, 1024, 1024), VasaProjModel(512, 1018))


def test_load_checkpoints_strict_round_trip(tmp_path):
    mods = _tiny_set()
    names = ["unet", "adapter_module", "pose_guider", "audio_linear", "id_proj", "vasa_linear"]
    os.makedirs(tmp_path / "ck")
    paths, want = {}, {}
    for i, (n, m) in enumerate(zip(names, mods)):
        sd = synthetic_state_dict(100 + i, {k: tuple(v.shape) for k, v in m.state_dict().items()})
        paths[n] = str(tmp_path / "ck" / f"{n}.pth")
        torch.save(sd, paths[n])
        want[n] = sd
    fresh = _tiny_set()
    ck.load_checkpoints(paths, *fresh)
    for n, m in zip(names, fresh):
        if n == "adapter_module":
            continue          # unet-*.pth (loaded after the adapter file, as in the reference) holds the
            #                   processors' to_k_ip / to_v_ip too and overwrites them
        got = m.state_dict()
        for k, v in want[n].items():
            assert torch.equal(got[k].float(), v), (n, k)
    # a missing key fails the strict load
    bad = dict(want["id_proj"])
    bad.pop("proj3.bias")
    torch.save(bad, paths["id_proj"])
    with pytest.raises(RuntimeError):
        ck.load_checkpoints(paths, *_tiny_set())


def test_adapter_merge_renumbers_collisions():
    from actalker_amd.unet_spatio_temporal_condition_mambaID_v10_two_ip import load_adapter_states
    _, adapters, *_ = _tiny_set()
    k0 = "0.to_k_ip.0.weight"
    w = adapters.state_dict()[k0]
    a, b = torch.full_like(w, 1.0), torch.full_like(w, 2.0)
    info = load_adapter_states(adapters, [{k0: a}, {k0: b}])
    sd = adapters.state_dict()
    assert torch.equal(sd["0.to_k_ip.0.weight"], a) and torch.equal(sd["0.to_k_ip.1.weight"], b)
    assert not info.unexpected_keys


def test_dtype_policy_keeps_ssm_fp32():
    unet, *_ = _tiny_set()
    ck.apply_dtype_policy(unet, torch.float16)
    for name, p in unet.named_parameters():
        want = torch.float32 if any(s in name for s in ck.SSM_FP32_KEYS) else torch.float16
        assert p.dtype == want, name
    assert any(any(s in n for s in ck.SSM_FP32_KEYS) for n, _ in unet.named_parameters())


def test_vae_from_pretrained_folder(tmp_path):
    from safetensors.torch import save_file
    from actalker_amd.vae import AutoencoderKLTemporalDecoder
    cfg = {"_class_name": "AutoencoderKLTemporalDecoder", "block_out_channels": [64, 64, 128, 128],
           "latent_channels": 4, "scaling_factor": 0.18215, "force_upcast": True, "layers_per_block": 2}
    m = AutoencoderKLTemporalDecoder(block_out_channels=(64, 64, 128, 128))
    sd = synthetic_state_dict(3, {k: tuple(v.shape) for k, v in m.state_dict().items()})
    os.makedirs(tmp_path / "vae")
    (tmp_path / "vae" / "config.json").write_text(json.dumps(cfg))
    save_file({k: v.half() for k, v in sd.items()}, str(tmp_path / "vae" / "diffusion_pytorch_model.fp16.safetensors"))
    v = AutoencoderKLTemporalDecoder.from_pretrained(str(tmp_path), subfolder="vae", variant="fp16")
    assert v.config.block_out_channels == (64, 64, 128, 128)
    assert torch.equal(v.state_dict()["quant_conv.weight"], sd["quant_conv.weight"].half().float())


def test_unet_state_dict_layout_matches_reference():
    """Every key and shape of the reference UNet (default SVD-XT config, after the reference
    add_ip_adapters(unet, [32, 32], [1.25, 1.25]); tools/gen_golden_keys.py imports the reference
    package by path) equals this build's, so a real ACTalker checkpoint loads with strict=True
    (Inference.py:124-127); the config fields match too (v10:73-99)."""
    import json
    from actalker_amd.unet_spatio_temporal_condition_mambaID_v10_two_ip import (UNetSpatioTemporalConditionModel,
                                                                               add_ip_adapters)
    with open(os.path.join(os.path.dirname(__file__), "golden", "unet_reference_keys.json")) as fh:
        ref_layout = json.load(fh)
    with torch.device("meta"):
        unet = UNetSpatioTemporalConditionModel()
    add_ip_adapters(unet, [32, 32], [1.25, 1.25])
    ours = {k: list(v.shape) for k, v in unet.state_dict().items()}
    want = ref_layout["keys"]
    assert sorted(set(want) - set(ours)) == [] and sorted(set(ours) - set(want)) == []
    assert {k: v for k, v in ours.items() if want[k] != v} == {}
    for k, v in ref_layout["config"].items():
        got = getattr(unet.config, k)
        assert (list(got) if isinstance(got, tuple) else got) == v, k
