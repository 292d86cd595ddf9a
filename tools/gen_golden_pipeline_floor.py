"""bf16 rounding floor of the reference-run sampler cases (tests/golden_pipeline.py): the oracle's version of each
case (tests/golden_pipeline.oracle_pipeline_loop) run in fp32 and with every op rounded to bf16 at its boundary
(oracle/precision.py). The bf16-rounded loop's deviation from the fp32 loop after the 25 steps is the budget the
HIP bf16 pipeline is held to against the reference run (tests/test_full_geometry_gpu.py). Writes
tests/golden/pipeline_floor_<case>.safetensors {latents, latents_bf16}.

    python tools/gen_golden_pipeline_floor.py [case ...]
"""
import os
import sys
import time

import torch
from safetensors.torch import save_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests import golden_pipeline as gp  # noqa: E402


def main(cases):
    for case in cases:
        out = {}
        for name, dt in (("latents", None), ("latents_bf16", torch.bfloat16)):
            t0 = time.time()
            out[name] = gp.oracle_pipeline_loop(case, dt).contiguous()
            print(f"{case} {name}: {time.time() - t0:.0f}s", flush=True)
        d = out["latents_bf16"] - out["latents"]
        print(f"{case}: bf16-rounded vs fp32 oracle loop rel-L2 {(d.norm() / out['latents'].norm()).item():.4e}",
              flush=True)
        save_file(out, os.path.join(ROOT, "tests", "golden", f"pipeline_floor_{case}.safetensors"))


if __name__ == "__main__":
    main(sys.argv[1:] or list(gp.CASES))
