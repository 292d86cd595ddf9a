"""Reference-run UNet forward goldens: the REFERENCE's own UNet package
(unet_spatio_temporal_condition_mambaID_v10_two_ip.py, unet_3d_blocks.py, TransformerSTmodel.py,
attention.py, attention_processor.py, mamba_layer.py) imported by path exactly as tools/gen_golden_keys.py
does, the reference ``add_ip_adapters`` (unet_spatio_temporal_condition.py:519-566) installed, seeded
synthetic weights loaded with ``strict=True``, and ``UNetSpatioTemporalConditionModel.forward``
(v10:362-517) run in fp32 on the CPU for the cases of tests/golden_unet_ref.py.

diffusers 0.29.2 is absent: its leaves are the oracle's CPU stand-ins (oracle/diffusers_leaves.py), the
mask downsample and mamba-ssm's selective_scan_ref are the oracle's restatements. No actalker_amd module
takes part in the forward (the product package only supplies the seeded weight values).

Runs in the build container only (needs /root/reference). Writes tests/golden/unet_ref_<case>.safetensors
= {out, weights_checksum, inputs_checksum}.

    python tools/gen_golden_unet_ref.py [case ...]     (tiny cases ~10 s each; full_half ~2-4 min)
"""
import os
import sys
import time

import torch
from safetensors.torch import save_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from actalker_amd.synthetic import synthetic_state_dict  # noqa: E402
from tests import golden_full as gf  # noqa: E402
from tests import golden_unet_ref as gu  # noqa: E402
from tools.gen_golden_keys import load_reference_unet  # noqa: E402


def build_reference_unet(cls, add_ip, case):
    if case in gu.FULL_CASES:
        with torch.device("meta"):
            unet = cls()
        unet = unet.to_empty(device="cpu")
        seed = gf.WEIGHT_SEED
    else:
        unet = cls(**gu.TINY_CFG)
        seed = gu.TINY_SEED
    add_ip(unet, [32, 32], [1.25, 1.25])
    shapes = {k: tuple(v.shape) for k, v in unet.state_dict().items()}
    sd = synthetic_state_dict(seed, shapes)
    unet.load_state_dict(sd, strict=True)
    return unet.eval(), sd


def main(cases):
    cls, add_ip = load_reference_unet()
    torch.set_grad_enabled(False)
    built = {}
    for case in cases:
        kind = "full" if case in gu.FULL_CASES else "tiny"
        if kind not in built:
            built.clear()
            built[kind] = build_reference_unet(cls, add_ip, case)
        unet, sd = built[kind]
        wsum = gf.checksum(*[sd[k] for k in sorted(sd)])
        sample, t, ehs, added, pose, masks = gu.case_inputs(case)
        isum = gf.checksum(sample, ehs[0], *ehs[1], pose, *masks)
        # the reference mutates the ip_hidden_states list in place (attention_processor.py:2842-2843): hand it
        # its own list
        t0 = time.time()
        if case in gu.PER_ELEMENT:
            # one batch element per reference forward (the UNet treats batch elements independently: GroupNorm,
            # attention and the scans are per element), concatenated along the batch
            B, F = sample.shape[:2]
            outs = []
            for b in gu.ELEMENTS.get(case, range(B)):
                fs = slice(b * F, (b + 1) * F)
                ref_ehs = (ehs[0][fs].clone(), [e[fs].clone() for e in ehs[1]])
                outs.append(unet(sample[b:b + 1], t, ref_ehs, added[b:b + 1], spatial_condition=pose[b:b + 1],
                                 cross_attention_kwargs={"ip_adapter_masks": [m.clone() for m in masks]},
                                 return_dict=False)[0])
                print(f"{case}: element {b} done at {time.time() - t0:.0f}s", flush=True)
            out = torch.cat(outs)          # the elements run, in order (gu.ELEMENTS)
        else:
            ref_ehs = (ehs[0].clone(), [e.clone() for e in ehs[1]])
            out = unet(sample, t, ref_ehs, added, spatial_condition=pose,
                       cross_attention_kwargs={"ip_adapter_masks": [m.clone() for m in masks]}, return_dict=False)[0]
        dt = time.time() - t0
        print(f"{case}: reference forward {dt:.1f}s, out {tuple(out.shape)} rms {out.pow(2).mean().sqrt():.4f}",
              flush=True)
        save_file({"out": out.contiguous().float(), "weights_checksum": wsum, "inputs_checksum": isum},
                  os.path.join(ROOT, "tests", "golden", f"unet_ref_{case}.safetensors"))


if __name__ == "__main__":
    main(sys.argv[1:] or list(gu.CASES))
