"""The rounding floor at BASELINE C1's geometry: the C1 window call's inputs
(tests/golden_unet_ref.py ``c1win14_mode0``: 576x576, mode 0, F = 14, B = 3 CFG branches, batch-1 forwards)
re-run through the fp32 oracle under oracle.precision.rounded(bf16) and rounded(fp16) -- every op's inputs,
outputs and weights rounded at its boundary, fp32 accumulation -- and compared per unit with the REFERENCE run
of the same call (tests/golden/unet_ref_c1win14_mode0.safetensors). Writes
tests/golden/unet_c1win14_mode0_floor.safetensors = {bf16, fp16: per-unit rel-L2 of the rounded oracle vs the
reference run; weights_checksum, inputs_checksum}, so tests/test_full_geometry_gpu.py can hold the C1 units to
1.5x the floor measured at C1 rather than the 576x1024 one. Test infrastructure (imports oracle/).

    python tools/gen_golden_c1_floor.py        (~5-10 min per precision on 8 cores)
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
from tests import golden_unet_ref as gu  # noqa: E402

CASE = "c1win14_mode0"


def main():
    torch.set_grad_enabled(False)
    g = load_file(os.path.join(ROOT, "tests", "golden", f"unet_ref_{CASE}.safetensors"))
    unet = gf.build_full_unet()
    sd32 = {k: v.detach().float() for k, v in unet.state_dict().items()}
    del unet
    wsum = gf.checksum(*[sd32[k] for k in sorted(sd32)])
    torch.testing.assert_close(wsum, g["weights_checksum"], rtol=1e-6, atol=1e-6)
    sample, t, ehs, added, pose, masks = gu.case_inputs(CASE)
    isum = gf.checksum(sample, ehs[0], *ehs[1], pose, *masks)
    torch.testing.assert_close(isum, g["inputs_checksum"], rtol=1e-6, atol=1e-6)
    B, F = sample.shape[:2]
    want = g["out"]
    assert want.shape[0] == B
    out = {"weights_checksum": wsum, "inputs_checksum": isum}
    report = {}
    for name, dt in (("bf16", torch.bfloat16), ("fp16", torch.float16)):
        sd = precision.round_state_dict(sd32, dt)
        fl = []
        t0 = time.time()
        for b in range(B):
            fs = slice(b * F, (b + 1) * F)
            e = (ehs[0][fs].clone().to(dt).float(), [x[fs].clone().to(dt).float() for x in ehs[1]])
            with precision.rounded(dt):
                o = ref.unet_forward(sd, sample[b:b + 1].to(dt).float(), t, e, added[b:b + 1],
                                     pose[b:b + 1].to(dt).float(), {"ip_adapter_masks": [m.clone() for m in masks]})
            d = o[0] - want[b]
            fl.append((d.norm() / want[b].norm()).item())
            print(f"{CASE} {name}-rounded oracle, unit {b}: rel-L2 {fl[-1]:.4e} vs the reference run "
                  f"({time.time() - t0:.0f}s)", flush=True)
        out[name] = torch.tensor(fl, dtype=torch.float64)
        report[name] = [round(x, 6) for x in fl]
    save_file(out, os.path.join(ROOT, "tests", "golden", f"unet_{CASE}_floor.safetensors"))
    print(json.dumps(report))


if __name__ == "__main__":
    main()
