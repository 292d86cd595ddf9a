"""Oracle fixtures for the REAL-WIDTH 25-step sampler-loop parity test: the same loop and inputs as
tools/gen_golden_loop.py (N = 4 frames, fpb 2, 16x32 latent, windowed 4-way CFG, partial masks) around the
full-width UNet (320 / 640 / 1280 / 1280, 5 / 10 / 20 / 20 heads, synthetic weights of tests/golden_full.py's
seed), as the fp32 oracle and as the bf16-rounded oracle (every op's inputs and outputs rounded at its
boundary, oracle/precision.py) -- the latter's deviation after 25 steps is the stated budget the HIP bf16 loop
is held to. Writes tests/golden/loop25_full_<mode>.safetensors {latents, latents_bf16}.

    python tools/gen_golden_loop_full.py [mode ...]        (~20-40 min per mode on 8 CPU threads)
"""
import os
import sys
import time

import torch
from safetensors.torch import save_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import precision  # noqa: E402
from tests import golden_full as gf  # noqa: E402
from tests import golden_loop as gl  # noqa: E402


def main(modes):
    unet = gf.build_full_unet()
    sd32 = {k: v.detach().float().clone() for k, v in unet.state_dict().items()}
    wsum = gf.checksum(*[unet.state_dict()[k] for k in sorted(unet.state_dict())])
    del unet
    sdb = precision.round_state_dict(sd32, torch.bfloat16)
    for m in modes:
        out = {"weights_checksum": wsum}
        for name, sd, dt in (("latents", sd32, None), ("latents_bf16", sdb, torch.bfloat16)):
            t0 = time.time()
            with torch.no_grad():
                out[name] = gl.oracle_loop(sd, gl.FULL_CFG, gl.GATES[m], pose_ch=320, dtype=dt).contiguous()
            print(f"{m} {name}: {time.time() - t0:.0f}s rms {out[name].pow(2).mean().sqrt():.4f}", flush=True)
        d = out["latents_bf16"] - out["latents"]
        print(f"{m}: bf16-rounded loop vs fp32 loop rel-L2 {(d.norm() / out['latents'].norm()).item():.4e}", flush=True)
        save_file(out, os.path.join(ROOT, "tests", "golden", f"loop25_full_{m}.safetensors"))


if __name__ == "__main__":
    main(sys.argv[1:] or ["mode0"])
