"""The per-element reference goldens (tests/golden_unet_ref.py PER_ELEMENT) rest on the UNet treating batch elements
independently: run the reference UNet by path on element 0 of win14_mode0 alone and compare it with the committed
B = 3 forward's element 0. Build container only (needs /root/reference).

    OMP_NUM_THREADS=8 python tools/check_reference_batch_independence.py
"""
import os, sys, time, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from safetensors.torch import load_file
from tests import golden_unet_ref as gu
from tools.gen_golden_keys import load_reference_unet
from tools.gen_golden_unet_ref import build_reference_unet
torch.set_grad_enabled(False)
cls, add_ip = load_reference_unet()
unet, sd = build_reference_unet(cls, add_ip, "win14_mode0")
sample, t, ehs, added, pose, masks = gu.case_inputs("win14_mode0")
F = sample.shape[1]
b = 0
fs = slice(b * F, (b + 1) * F)
t0 = time.time()
o = unet(sample[b:b+1], t, (ehs[0][fs].clone(), [e[fs].clone() for e in ehs[1]]), added[b:b+1], spatial_condition=pose[b:b+1],
         cross_attention_kwargs={"ip_adapter_masks": [m.clone() for m in masks]}, return_dict=False)[0]
g = load_file(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "unet_ref_win14_mode0.safetensors"))["out"]
d = ((o[0] - g[0]).norm() / g[0].norm()).item()
print(f"batch-1 reference forward of element 0 vs the B = 3 forward's element 0: rel-L2 {d:.3e}, max |diff| {(o[0]-g[0]).abs().max().item():.3e} ({time.time()-t0:.0f} s)")
