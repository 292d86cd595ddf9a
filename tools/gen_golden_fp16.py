"""The fp16 budget: the full-geometry oracle (576x1024, real widths, B = 1 x F = 2;
tests/golden_full.py) re-run under oracle.precision.rounded(fp16) -- the reference's shipped
weight_dtype fp16 path (config/inference.yaml:66) modelled as fp16 weights / op inputs / op outputs with
fp32 accumulation -- and under rounded(bf16), the precision the HIP build computes in. Writes
tests/golden/unet_full_<case>_rounded.safetensors = {fp16, bf16} outputs; the deviations from the fp32
oracle (tests/golden/unet_full_<case>.safetensors) are printed and stored in profiles/r3_fp16_budget.json.

    python tools/gen_golden_fp16.py [case ...]       (~1.5 min per case and precision on 8 cores)
"""
import json
import os
import sys
import time

import torch
from safetensors.torch import load_file, save_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import precision  # noqa: E402
from oracle import reference_cpu as ref  # noqa: E402
from tests import golden_full as gf  # noqa: E402


def main(cases):
    unet = gf.build_full_unet()
    sd32 = {k: v.detach().float() for k, v in unet.state_dict().items()}
    del unet
    path = os.path.join(ROOT, "profiles", "r3_fp16_budget.json")
    report = json.load(open(path)) if os.path.exists(path) else {}
    for case in cases:
        want = load_file(os.path.join(ROOT, "tests", "golden", f"unet_full_{case}.safetensors"))["out"]
        sample, t, ehs, added, pose, masks = gf.case_inputs(case)
        outs, rep = {}, {}
        for name, dt in (("fp16", torch.float16), ("bf16", torch.bfloat16)):
            sd = precision.round_state_dict(sd32, dt)
            t0 = time.time()
            with torch.no_grad(), precision.rounded(dt):
                o = ref.unet_forward(sd, sample.to(dt).float(), t, (ehs[0].to(dt).float(), [e.to(dt).float() for e in ehs[1]]),
                                     added, pose.to(dt).float(), {"ip_adapter_masks": masks})
            d = o - want
            rep[name] = dict(rel_l2=round((d.norm() / want.norm()).item(), 6), max_abs=round(d.abs().max().item(), 5))
            outs[name] = o.contiguous()
            print(f"{case} {name}-rounded oracle vs fp32 oracle: {rep[name]} ({time.time() - t0:.0f}s)", flush=True)
        save_file(outs, os.path.join(ROOT, "tests", "golden", f"unet_full_{case}_rounded.safetensors"))
        report[case] = rep
    with open(path, "w") as fh:
        json.dump(report, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:] or ["mode0", "half"])
