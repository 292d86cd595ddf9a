"""Reference UNet state_dict layout: key names and shapes of the REFERENCE
``UNetSpatioTemporalConditionModel`` (unet_spatio_temporal_condition_mambaID_v10_two_ip.py:73-251,
default SVD-XT config) after the reference ``add_ip_adapters(unet, [32, 32], [1.25, 1.25])``
(unet_spatio_temporal_condition.py:519-566, the one Inference.py:22/70 calls), i.e. the key set
``unet.load_state_dict(..., strict=True)`` (Inference.py:124-127) checks a checkpoint against.

Runs in the build container only (needs /root/reference). The reference package
(src/models/base: UNet, unet_3d_blocks, TransformerSTmodel, attention, attention_processor,
mamba_layer) is imported by path and runs unchanged on the meta device. diffusers 0.29.2 is absent:
its config / model mixins are stubbed minimally, and the building blocks the reference takes from it
(SpatioTemporalResBlock, ResnetBlock2D, Downsample2D, Upsample2D, TimestepEmbedding, Timesteps,
FeedForward) are the oracle's CPU stand-ins (oracle/diffusers_leaves.py, diffusers 0.29.2 names and
signatures) -- so the key names those blocks contribute internally are the restatement's, while everything the reference
files define (block nesting, attribute names, Mamba / IP-adapter parameters, the attention modules
of attention_processor.py) is the reference's own. Other diffusers / timm / pyzorder / mamba_ssm
names are import-only stubs.

Writes tests/golden/unet_reference_keys.json: {"keys": {name: shape}, "config": {...}}.
"""
from __future__ import annotations

import importlib
import inspect
import json
import logging as _logging
import os
import sys
import types
from dataclasses import dataclass

import torch
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle.reference_cpu import mask_downsample, selective_scan_ref  # noqa: E402

REFDIR = "/root/reference/src/models/base"


def _mod(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


class _Stub:
    def __init__(self, *a, **k):
        raise RuntimeError(f"{type(self).__name__} is an import-only stub")


def _stub(name):
    return type(name, (_Stub,), {})


def install_stubs():
    from oracle import diffusers_leaves as am
    _mod("timm")
    _mod("timm.models")
    _mod("timm.models.resnet", Bottleneck=object)
    _mod("timm.models.layers", DropPath=object, to_2tuple=lambda x: (x, x), trunc_normal_=lambda *a, **k: None)
    _mod("pyzorder", ZOrderIndexer=object)
    _mod("mamba_ssm")
    _mod("mamba_ssm.ops")
    _mod("mamba_ssm.ops.selective_scan_interface", selective_scan_fn=selective_scan_ref,
         selective_scan_ref=selective_scan_ref)

    def register_to_config(init):
        sig = inspect.signature(init)

        def wrapped(self, *args, **kwargs):
            bound = sig.bind(self, *args, **kwargs)
            bound.apply_defaults()
            cfg = {k: v for k, v in bound.arguments.items() if k != "self"}
            init(self, *args, **kwargs)
            self.__dict__["_cfg"] = cfg
        return wrapped

    class ConfigMixin:
        @property
        def config(self):
            return types.SimpleNamespace(**self.__dict__["_cfg"])

    class ModelMixin(nn.Module):
        @property
        def device(self):
            return next(self.parameters()).device

        @property
        def dtype(self):
            return next(self.parameters()).dtype

    @dataclass
    class BaseOutput:
        pass

    class IPAdapterMaskProcessor:
        downsample = staticmethod(mask_downsample)

    logging_ns = types.SimpleNamespace(get_logger=_logging.getLogger)
    _mod("diffusers", __version__="0.29.2")
    _mod("diffusers.configuration_utils", ConfigMixin=ConfigMixin, register_to_config=register_to_config)
    _mod("diffusers.loaders", UNet2DConditionLoadersMixin=type("UNet2DConditionLoadersMixin", (), {}))
    _mod("diffusers.utils", BaseOutput=BaseOutput, logging=logging_ns, deprecate=lambda *a, **k: None,
         is_torch_version=lambda *a, **k: True)
    _mod("diffusers.utils.torch_utils", apply_freeu=lambda *a, **k: None, maybe_allow_in_graph=lambda c: c)
    _mod("diffusers.utils.import_utils", is_torch_npu_available=lambda: False, is_xformers_available=lambda: False)
    _mod("diffusers.image_processor", IPAdapterMaskProcessor=IPAdapterMaskProcessor)
    _mod("diffusers.models")
    _mod("diffusers.models.lora", LoRALinearLayer=type("LoRALinearLayer", (nn.Module,), {}))
    _mod("diffusers.models.modeling_utils", ModelMixin=ModelMixin)
    _mod("diffusers.models.embeddings", TimestepEmbedding=am.TimestepEmbedding, Timesteps=am.Timesteps,
         SinusoidalPositionalEmbedding=_stub("SinusoidalPositionalEmbedding"))
    _mod("diffusers.models.resnet", Downsample2D=am.Downsample2D, ResnetBlock2D=am.ResnetBlock2D,
         SpatioTemporalResBlock=am.SpatioTemporalResBlock, TemporalConvLayer=_stub("TemporalConvLayer"),
         Upsample2D=am.Upsample2D)
    _mod("diffusers.models.transformers")
    _mod("diffusers.models.transformers.dual_transformer_2d", DualTransformer2DModel=_stub("DualTransformer2DModel"))
    _mod("diffusers.models.transformers.transformer_2d", Transformer2DModel=_stub("Transformer2DModel"))
    _mod("diffusers.models.transformers.transformer_temporal", TransformerTemporalModel=_stub("TransformerTemporalModel"),
         TransformerTemporalModelOutput=_stub("TransformerTemporalModelOutput"))
    # diffusers.models.attention: Attention is filled in from the reference attention_processor below
    _mod("diffusers.models.attention", FeedForward=am.FeedForward, AdaLayerNorm=_stub("AdaLayerNorm"),
         AdaLayerNormZero=_stub("AdaLayerNormZero"), AdaLayerNormContinuous=_stub("AdaLayerNormContinuous"),
         GatedSelfAttentionDense=_stub("GatedSelfAttentionDense"), _chunked_feed_forward=lambda *a, **k: None,
         BasicTransformerBlock=_stub("BasicTransformerBlock"),
         TemporalBasicTransformerBlock=_stub("TemporalBasicTransformerBlock"))


def load_reference_unet():
    sys.dont_write_bytecode = True
    install_stubs()
    pkg = types.ModuleType("refbase")
    pkg.__path__ = [REFDIR]
    sys.modules["refbase"] = pkg
    ap = importlib.import_module("refbase.attention_processor")
    sys.modules["diffusers.models.attention"].Attention = ap.Attention
    v10 = importlib.import_module("refbase.unet_spatio_temporal_condition_mambaID_v10_two_ip")
    plain = importlib.import_module("refbase.unet_spatio_temporal_condition")
    return v10.UNetSpatioTemporalConditionModel, plain.add_ip_adapters


def main():
    cls, add_ip = load_reference_unet()
    with torch.device("meta"):
        unet = cls()
    add_ip(unet, [32, 32], [1.25, 1.25])
    keys = {k: list(v.shape) for k, v in unet.state_dict().items()}
    cfg = {k: (list(v) if isinstance(v, tuple) else v) for k, v in unet.__dict__["_cfg"].items() if k != "attn_cls"}
    out = os.path.join(ROOT, "tests", "golden", "unet_reference_keys.json")
    with open(out, "w") as fh:
        json.dump({"keys": keys, "config": cfg}, fh, indent=0, sort_keys=True)
    n = sum(int(torch.tensor(s).prod()) if s else 1 for s in keys.values())
    print(f"{len(keys)} keys, {n / 1e9:.3f} B parameters -> {out}")


if __name__ == "__main__":
    main()
