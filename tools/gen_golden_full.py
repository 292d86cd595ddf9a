"""Oracle fixtures for the full-geometry UNet parity tests (tests/test_full_geometry_gpu.py).

Runs oracle.reference_cpu.unet_forward (fp32 CPU restatement) on the real SVD-XT + ACTalker v10 UNet
(1.775 B parameters, seeded synthetic weights) at 576x1024, B=1 CFG branch x F=2 frames, for the four
mask cases of tests/golden_full.py, and writes tests/golden/unet_full_<case>.safetensors holding the
oracle output plus checksums of the weights and inputs it was computed from.

    python tools/gen_golden_full.py [case ...]      (~1-2 min per case on 8 cores)
"""
import os
import sys
import time

import torch
from safetensors.torch import save_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import reference_cpu as ref  # noqa: E402
from tests import golden_full as gf  # noqa: E402


def main(cases):
    unet = gf.build_full_unet()
    sd = {k: v.detach().float() for k, v in unet.state_dict().items()}
    wsum = gf.checksum(*[sd[k] for k in sorted(sd)])
    for case in cases:
        sample, t, ehs, added, pose, masks = gf.case_inputs(case)
        t0 = time.time()
        with torch.no_grad():
            out = ref.unet_forward(sd, sample, t, ehs, added, pose, {"ip_adapter_masks": masks})
        print(f"{case}: oracle {time.time() - t0:.1f}s, |out| rms {out.pow(2).mean().sqrt():.4f}", flush=True)
        save_file({"out": out.contiguous(), "weights_checksum": wsum,
                   "inputs_checksum": gf.checksum(sample, ehs[0], *ehs[1], pose, *masks)},
                  os.path.join(ROOT, "tests", "golden", f"unet_full_{case}.safetensors"))


if __name__ == "__main__":
    main(sys.argv[1:] or list(gf.CASES))
