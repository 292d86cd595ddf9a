"""Golden outputs of the REFERENCE attention processors.

Runs in the build container only (needs /root/reference). Loads
/root/reference/src/models/base/attention_processor.py by path; the diffusers names it imports are
absent from this image and are supplied as import-only stubs (deprecate, logging, is_*_available,
maybe_allow_in_graph, LoRALinearLayer: none of them on the path exercised here) plus the restated
IPAdapterMaskProcessor.downsample (diffusers 0.29.2; oracle.reference_cpu.mask_downsample, the same
restatement tools/gen_golden.py supplies to mamba_layer.py). The reference ``Attention`` module and
its ``AttnProcessor2_0`` / ``IPAdapterAttnProcessor2_0`` run unchanged, including the in-place
``ip_hidden_states`` mutation (:2842-2843): each IP case is evaluated twice on the same list and the
second (4-D, mutated) call must reproduce the first.

Writes tests/golden/attn_<case>.safetensors (output row subsample, see tests/golden_attn.py).
    python tools/gen_golden_attn.py [case ...]
"""
from __future__ import annotations

import importlib.util
import logging as _logging
import os
import sys
import types

import torch
from safetensors.torch import save_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle.reference_cpu import mask_downsample  # noqa: E402
from tests import golden_attn as ga  # noqa: E402

REF = "/root/reference/src/models/base/attention_processor.py"


def _stub_modules():
    mods = {n: types.ModuleType(n) for n in ("diffusers", "diffusers.image_processor", "diffusers.utils",
                                             "diffusers.utils.import_utils", "diffusers.utils.torch_utils",
                                             "diffusers.models", "diffusers.models.lora")}

    class IPAdapterMaskProcessor:
        downsample = staticmethod(mask_downsample)

    class LoRALinearLayer(torch.nn.Module):
        pass

    mods["diffusers.image_processor"].IPAdapterMaskProcessor = IPAdapterMaskProcessor
    mods["diffusers.utils"].deprecate = lambda *a, **k: None
    mods["diffusers.utils"].logging = types.SimpleNamespace(get_logger=_logging.getLogger)
    mods["diffusers.utils.import_utils"].is_torch_npu_available = lambda: False
    mods["diffusers.utils.import_utils"].is_xformers_available = lambda: False
    mods["diffusers.utils.torch_utils"].maybe_allow_in_graph = lambda cls: cls
    mods["diffusers.models.lora"].LoRALinearLayer = LoRALinearLayer
    sys.modules.update(mods)


def load_reference():
    _stub_modules()
    spec = importlib.util.spec_from_file_location("ref_attention_processor", REF)
    mod = importlib.util.module_from_spec(spec)
    sys.dont_write_bytecode = True
    spec.loader.exec_module(mod)
    return mod


def run_case(ap, name, case):
    C, heads = case["C"], case["heads"]
    cross = None if case["kind"].startswith("self") else 1024
    attn = ap.Attention(query_dim=C, cross_attention_dim=cross, heads=heads, dim_head=64, bias=False,
                        out_bias=True)
    if cross is not None:
        attn.set_processor(ap.IPAdapterAttnProcessor2_0(hidden_size=C, cross_attention_dim=1024,
                                                        num_tokens=[32, 32], scale=[1.25, 1.25]))
    else:
        attn.set_processor(ap.AttnProcessor2_0())
    attn.load_state_dict(ga.weights(name, case), strict=True)
    attn.eval()
    x, ide, aud, vas = ga.inputs(name, case)
    with torch.no_grad():
        if case["kind"].startswith("self"):
            return attn(x)
        if case["kind"] == "ip":
            ips = [aud, vas]
            kw = dict(ip_adapter_masks=ga.masks(case["mask"]))
            y = attn(x, encoder_hidden_states=(ide, ips), **kw)
            assert ips[0].dim() == 4 and ips[1].dim() == 4            # the in-place mutation happened
            y2 = attn(x, encoder_hidden_states=(ide, ips), **kw)       # a later block sees the 4-D list
            assert torch.equal(y, y2)
            return y
        # temporal: contexts time-pooled per window, repeated over the window's S rows
        S = case["S"]
        rep = lambda t: t.repeat_interleave(S, dim=0)                 # noqa: E731
        ips = [rep(aud), rep(vas)]
        y = attn(x, encoder_hidden_states=(rep(ide), ips))
        y2 = attn(x, encoder_hidden_states=(rep(ide), [t.unsqueeze(1) for t in ips]))
        assert torch.allclose(y, y2, rtol=1e-5, atol=1e-6)
        return y


def main(names):
    ap = load_reference()
    for name in names:
        case = ga.CASES[name]
        y = run_case(ap, name, case)
        sub = ga.subsample(y, case)
        save_file({"y": sub}, os.path.join(ROOT, "tests", "golden", f"attn_{name}.safetensors"))
        print(name, tuple(y.shape), "->", tuple(sub.shape), f"rms {y.pow(2).mean().sqrt():.4f}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:] or list(ga.CASES))
