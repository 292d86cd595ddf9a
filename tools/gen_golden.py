"""Generate golden vectors for SS2D_cond_v10 from the REFERENCE module itself.

Runs in the build container only (needs /root/reference). It loads
/root/reference/src/models/base/mamba_layer.py by path and supplies the pieces that are absent
from this image:
  * import-only modules it never uses on this path: timm.models.resnet.Bottleneck,
    timm.models.layers.{DropPath,to_2tuple,trunc_normal_}, pyzorder.ZOrderIndexer (stubs);
  * diffusers.image_processor.IPAdapterMaskProcessor.downsample (diffusers 0.29.2, restated);
  * mamba_ssm's selective_scan_fn (1.2.0, restated ``selective_scan_ref``; mamba_layer.py:21-34
    binds the module-global name).
Weights are a deterministic function of a seed (``golden_weights``), so tests regenerate them
instead of storing them. Fixtures written: tests/golden/ss2d_cond_v10_<case>.safetensors holding
inputs (x, id_emb, conds, masks) and the reference output ``y``; plus a JSON index.

Usage:  python tools/gen_golden.py            (toy / c320 cases, full tensors)
        python tools/gen_golden.py levels [case ...]   (LEVEL_CASES: 576x1024 masks, real S; ~1-2 min)
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys
import time
import types

import torch
from safetensors.torch import save_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle.reference_cpu import mask_downsample, selective_scan_ref  # noqa: E402
from tests.golden_weights import golden_weights, CASES, LEVEL_CASES, make_inputs  # noqa: E402
from tests.golden_full import checksum  # noqa: E402

REF = "/root/reference/src/models/base/mamba_layer.py"
OUT = os.path.join(ROOT, "tests", "golden")


def _stub_modules():
    timm = types.ModuleType("timm")
    tm = types.ModuleType("timm.models")
    tr = types.ModuleType("timm.models.resnet")
    tl = types.ModuleType("timm.models.layers")
    tr.Bottleneck = object
    tl.DropPath = object
    tl.to_2tuple = lambda x: (x, x)
    tl.trunc_normal_ = lambda *a, **k: None
    sys.modules.update({"timm": timm, "timm.models": tm, "timm.models.resnet": tr, "timm.models.layers": tl})
    pz = types.ModuleType("pyzorder")
    pz.ZOrderIndexer = object
    sys.modules["pyzorder"] = pz
    dif = types.ModuleType("diffusers")
    ip = types.ModuleType("diffusers.image_processor")

    class IPAdapterMaskProcessor:
        downsample = staticmethod(mask_downsample)

    ip.IPAdapterMaskProcessor = IPAdapterMaskProcessor
    sys.modules.update({"diffusers": dif, "diffusers.image_processor": ip})
    ms = types.ModuleType("mamba_ssm")
    mo = types.ModuleType("mamba_ssm.ops")
    mi = types.ModuleType("mamba_ssm.ops.selective_scan_interface")
    mi.selective_scan_fn = selective_scan_ref
    mi.selective_scan_ref = selective_scan_ref
    sys.modules.update({"mamba_ssm": ms, "mamba_ssm.ops": mo, "mamba_ssm.ops.selective_scan_interface": mi})


def load_reference_mamba():
    _stub_modules()
    spec = importlib.util.spec_from_file_location("ref_mamba_layer", REF)
    mod = importlib.util.module_from_spec(spec)
    sys.dont_write_bytecode = True
    spec.loader.exec_module(mod)
    return mod


def level_main(ref, names):
    """Level-shape cases: reference output at every ``sub``-th token row plus checksums (inputs regenerate)."""
    for name in names:
        case = LEVEL_CASES[name]
        m = ref.SS2D_cond_v10(d_model=case["d_model"], d_cond=case["d_cond"], cond_size=32, dropout=0.1,
                              d_state=16, size=8, scan_type="sweep", num_direction=2)
        sd = golden_weights(case["seed"], {k: tuple(v.shape) for k, v in m.state_dict().items()})
        m.load_state_dict(sd, strict=True)
        m.eval()
        x, id_emb, conds, masks = make_inputs(case)
        n_sel = [int(mask_downsample(mk[:, 0], 1, case["S"], 1).view(-1).int().nonzero().numel()) for mk in masks]
        t0 = time.time()
        with torch.no_grad():
            y = m(x, id_emb, conds, masks)
        ysub = y[:, ::case["sub"]].contiguous()
        save_file({"y_sub": ysub, "inputs_checksum": checksum(x, id_emb, conds, *masks),
                   "n_selected": torch.tensor(n_sel, dtype=torch.int64)},
                  os.path.join(OUT, f"ss2d_level_{name}.safetensors"))
        print(name, tuple(y.shape), "selected", n_sel, f"{time.time() - t0:.1f}s", float(y.abs().mean()), flush=True)


def main():
    ref = load_reference_mamba()
    os.makedirs(OUT, exist_ok=True)
    if len(sys.argv) > 1 and sys.argv[1] == "levels":
        level_main(ref, sys.argv[2:] or list(LEVEL_CASES))
        return
    index = {}
    for name, case in CASES.items():
        m = ref.SS2D_cond_v10(d_model=case["d_model"], d_cond=case["d_cond"], cond_size=32, dropout=0.1,
                              d_state=16, size=8, scan_type="sweep", num_direction=2)
        sd = golden_weights(case["seed"], {k: tuple(v.shape) for k, v in m.state_dict().items()})
        m.load_state_dict(sd, strict=True)
        m.eval()
        x, id_emb, conds, masks = make_inputs(case)
        with torch.no_grad():
            y = m(x, id_emb, conds, masks)
        tensors = dict(x=x, id_emb=id_emb, conds=conds, mask_a=masks[0], mask_e=masks[1], y=y.contiguous())
        fn = f"ss2d_cond_v10_{name}.safetensors"
        save_file({k: v.contiguous() for k, v in tensors.items()}, os.path.join(OUT, fn))
        index[name] = dict(case, file=fn, y_abs_mean=float(y.abs().mean()))
        print(name, tuple(y.shape), float(y.abs().mean()))
    with open(os.path.join(OUT, "index.json"), "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
