"""Generate golden vectors for the conditioning adapters from the REFERENCE modules themselves.

Runs in the build container only (needs /root/reference). It loads
/root/reference/src/models/audio_adapter/{audio_proj,pose_guider}.py by path. Their only missing
dependency is diffusers' ``ModelMixin`` base class (import-only: the modules use nothing from it
but ``nn.Module`` behaviour), stubbed here as ``torch.nn.Module``.

Configurations are the ones Inference.py:72-78 builds: PoseGuider(320, (16, 32, 96, 256)),
AudioProjModel(seq_len=10, blocks=5, channels=384, intermediate_dim=1024, output_dim=1024,
context_tokens=32), IDProjModel(512, 1024, 1024), VasaProjModel(512, 1024). Weights are
``actalker_amd.synthetic.synthetic_state_dict(seed, shapes)`` (pure function of seed, name and
shape), so the tests regenerate them instead of storing them; PoseGuider's zero-initialised
conv_out (pose_guider.py:56-63) is overwritten like every other parameter so the fixture checks it.

Writes tests/golden/adapters_<case>.safetensors (inputs ``x`` and reference output ``y``) and
tests/golden/adapters_index.json.  Usage:  python tools/gen_golden_adapters.py
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys
import types

import torch
from safetensors.torch import save_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from actalker_amd.synthetic import synthetic_state_dict  # noqa: E402
from tests.adapter_cases import ADAPTER_CASES, adapter_input  # noqa: E402

REF_DIR = "/root/reference/src/models/audio_adapter"
OUT = os.path.join(ROOT, "tests", "golden")


def _stub_diffusers():
    dif = types.ModuleType("diffusers")
    models = types.ModuleType("diffusers.models")
    mu = types.ModuleType("diffusers.models.modeling_utils")
    dif.ModelMixin = torch.nn.Module
    mu.ModelMixin = torch.nn.Module
    sys.modules.update({"diffusers": dif, "diffusers.models": models, "diffusers.models.modeling_utils": mu})


def _load(name):
    spec = importlib.util.spec_from_file_location("ref_" + name, os.path.join(REF_DIR, name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    sys.dont_write_bytecode = True
    _stub_diffusers()
    ap = _load("audio_proj")
    pg = _load("pose_guider")
    os.makedirs(OUT, exist_ok=True)
    index = {}
    for name, case in ADAPTER_CASES.items():
        cls = {"AudioProjModel": ap.AudioProjModel, "IDProjModel": ap.IDProjModel,
               "VasaProjModel": ap.VasaProjModel, "PoseGuider": pg.PoseGuider}[case["cls"]]
        m = cls(**case["kwargs"])
        sd = synthetic_state_dict(case["seed"], {k: tuple(v.shape) for k, v in m.state_dict().items()})
        m.load_state_dict(sd, strict=True)
        m.eval()
        x = adapter_input(case)
        with torch.no_grad():
            y = m(x)
        fn = f"adapters_{name}.safetensors"
        save_file({"x": x.contiguous(), "y": y.contiguous()}, os.path.join(OUT, fn))
        index[name] = dict(case, file=fn, y_shape=list(y.shape), y_abs_mean=float(y.abs().mean()))
        print(name, tuple(x.shape), "->", tuple(y.shape), float(y.abs().mean()))
    with open(os.path.join(OUT, "adapters_index.json"), "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
