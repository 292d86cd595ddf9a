"""Oracle fixtures for the 25-step sampler-loop parity tests: oracle.reference_cpu.denoise_loop (the
pipeline:670-756 restatement) around the fp32 oracle UNet (tiny full-topology config of
__graft_entry__._tiny_unet), for modes 0 / 1 / 2 with the pipeline's CFG stacking
(tests/golden_loop.py). Writes tests/golden/loop25_<mode>.safetensors (final latents).

    python tools/gen_golden_loop.py [mode ...]
"""
import os
import sys
import time

import torch
from safetensors.torch import save_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import __graft_entry__ as ge  # noqa: E402
from tests import golden_loop as gl  # noqa: E402


def main(modes):
    unet, cfg = ge._tiny_unet(seed=gl.UNET_SEED)
    sd = {k: v.detach().float().clone() for k, v in unet.state_dict().items()}
    for m in modes:
        t0 = time.time()
        with torch.no_grad():
            out = gl.oracle_loop(sd, cfg, gl.GATES[m])
        print(f"{m}: {time.time() - t0:.1f}s rms {out.pow(2).mean().sqrt():.4f}", flush=True)
        save_file({"latents": out.contiguous()}, os.path.join(ROOT, "tests", "golden", f"loop25_{m}.safetensors"))


if __name__ == "__main__":
    main(sys.argv[1:] or list(gl.GATES))
