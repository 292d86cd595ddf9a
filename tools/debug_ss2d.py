"""GPU debug: SS2D_cond_v10 c320_mode2 branch-by-branch vs the oracle."""
import os, sys, math
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import reference_cpu as ref
from tests.golden_weights import CASES, golden_weights, make_inputs
from actalker_amd.modules import Ctx, SS2D_cond_v10
from actalker_amd import ops

dev = torch.device("cuda")
def rel(a, b):
    a = a.float().cpu(); b = b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()

for name in ["c320_mode2", "toy_mode2", "c320_half"]:
    case = CASES[name]
    x, id_emb, conds, masks = make_inputs(case)
    m = SS2D_cond_v10(d_model=case["d_model"], d_cond=case["d_cond"], d_state=16, scan_type="sweep", num_direction=2)
    sd = golden_weights(case["seed"], {k: tuple(v.shape) for k, v in m.state_dict().items()})
    m.load_state_dict(sd)
    m = m.to(dev)
    BF, S, C = x.shape
    # oracle audio branch pieces
    sdp = {"m." + k: v for k, v in sd.items()}
    xz1 = ref.linear(sdp, "m.in_proj1", x)
    ide = torch.nn.functional.silu(ref.linear(sdp, "m.id_proj", id_emb))
    ac = torch.nn.functional.silu(ref.linear(sdp, "m.audio_proj", conds[:, :-1]))
    inp = torch.cat([xz1, ide, ac], 1)            # (BF, L, din) identity selection
    L = inp.shape[1]
    yo = ref.ss2d_unit(sdp, "m.audio_unit", inp.permute(0, 2, 1))[:, :, :S].permute(0, 2, 1)
    # product
    u = inp.reshape(BF * L, -1).to(dev, torch.bfloat16)
    for nc in (1, 2):
        y0, y1 = m.audio_unit.scan(u, BF, L, S) if nc is None else (None, None)
        p = m.audio_unit.packed()
        xdbl = ops.gemm(u, p["xproj"], out_f32=True)
        y0, y1 = ops.selective_scan(u, xdbl, p["dt_w"], p["dt_b"], p["A_log"], p["D"], nb=BF, L=L,
                                    R=m.audio_unit.dt_rank, n_keep=S, nchunks=nc)
        yy = (y0.float() + y1.float()).view(BF, S, -1)
        print(name, "L", L, "nc", nc, "audio scan rel", rel(yy, yo), "per-batch", [round(rel(yy[b], yo[b]), 4) for b in range(BF)])
        # xdbl check
        xd_ref = inp.reshape(BF * L, -1).to(torch.bfloat16).float() @ p["xproj"].float().cpu().t()
        print("   xdbl rel", rel(xdbl, xd_ref))
