"""bf16 / fp16 rounding floors of the reference-run sampler cases (tests/golden_pipeline.py): the oracle's version of each
case (tests/golden_pipeline.oracle_pipeline_loop) run in fp32 and with every op rounded to bf16 at its boundary
(oracle/precision.py). The bf16-rounded loop's deviation from the fp32 loop after the 25 steps is the budget the
HIP bf16 pipeline is held to against the reference run (tests/test_full_geometry_gpu.py). Writes
tests/golden/pipeline_floor_<case>.safetensors {latents, latents_bf16, latents_fp16}; the fp16 floor holds the HIP
fp16 pipeline (the reference's shipped weight_dtype).

    python tools/gen_golden_pipeline_floor.py [case ...]
"""
import os
import sys
import time

import torch
from safetensors.torch import load_file, save_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests import golden_pipeline as gp  # noqa: E402


def main(cases, names):
    for case in cases:
        path = os.path.join(ROOT, "tests", "golden", f"pipeline_floor_{case}.safetensors")
        out = load_file(path) if os.path.exists(path) else {}
        for name, dt in (("latents", None), ("latents_bf16", torch.bfloat16), ("latents_fp16", torch.float16)):
            if name not in names and name in out:
                continue
            t0 = time.time()
            out[name] = gp.oracle_pipeline_loop(case, dt).contiguous()
            print(f"{case} {name}: {time.time() - t0:.0f}s", flush=True)
        for name in ("latents_bf16", "latents_fp16"):
            d = out[name] - out["latents"]
            print(f"{case}: {name} vs fp32 oracle loop rel-L2 {(d.norm() / out['latents'].norm()).item():.4e}",
                  flush=True)
        save_file(out, path)


if __name__ == "__main__":
    # ``--only latents_fp16``: recompute just that entry (the others are kept from the existing file)
    args = sys.argv[1:]
    names = {"latents", "latents_bf16", "latents_fp16"}
    if "--only" in args:
        i = args.index("--only")
        names = {args[i + 1]}
        args = args[:i] + args[i + 2:]
    main(args or [c for c in gp.CASES if c not in gp.GEOMETRY], names)
