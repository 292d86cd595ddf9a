"""HIP attention (actalker_amd.modules.Attention.run_self / run_cross) against golden outputs of the
REFERENCE processors (tools/gen_golden_attn.py: attention_processor.py AttnProcessor2_0 :1528-1605 and
IPAdapterAttnProcessor2_0 :2747-2934 run unchanged, diffusers imports stubbed).

The reference weights load into the HIP module with strict=True (same parameter names), the masks
are the real 576x1024 masks (ones / zeros / half), temporal cases use the reference's (B*S, F, C)
layout with time-pooled contexts, which the HIP path takes un-repeated (its K/V are computed once per
window). Tolerance: relative L2 <= 2e-2 on the stored row subsample (bf16 activations)."""
import os

import pytest
import torch
from safetensors.torch import load_file

from tests import golden_attn as ga

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _module(name, case, dev):
    from actalker_amd.modules import Attention, IPAdapterAttnProcessor2_0
    C, heads = case["C"], case["heads"]
    cross = None if case["kind"].startswith("self") else 1024
    m = Attention(C, cross, heads, 64, bias=False, out_bias=True)
    if cross is not None:
        m.set_processor(IPAdapterAttnProcessor2_0(hidden_size=C, cross_attention_dim=1024, num_tokens=[32, 32],
                                                  scale=[1.25, 1.25]))
    m.load_state_dict(ga.weights(name, case), strict=True)
    return m.to(dev)


@pytest.mark.parametrize("name", sorted(ga.CASES))
def test_attention_matches_reference_processor(dev, name):
    from actalker_amd.modules import Ctx
    case = ga.CASES[name]
    m = _module(name, case, dev)
    x, ide, aud, vas = ga.inputs(name, case)
    C, B, S, Fr = case["C"], case["B"], case["S"], case["F"]
    bf = lambda t: t.to(dev, torch.bfloat16).contiguous()        # noqa: E731
    if case["kind"] in ("self", "ip"):
        ctx = Ctx(B, 1, dev)                                       # B frames of one image each
        n = bf(x.reshape(B * S, C))
    else:
        ctx = Ctx(B, Fr, dev)                                      # B windows of F frames
        # reference rows (b*S + s, f) -> token-major rows ((b*F + f)*S + s)
        n = bf(x.view(B, S, Fr, C).permute(0, 2, 1, 3).reshape(B * Fr * S, C))
    zero = torch.zeros_like(n)
    if case["kind"] == "self":
        y = m.run_self(ctx, n, zero, S, temporal=False)
    elif case["kind"] == "self_t":
        y = m.run_self(ctx, n, zero, S, temporal=True)
    elif case["kind"] == "ip":
        ctx.id_tok, ctx.audio_tok, ctx.vasa_tok = bf(ide.reshape(B, 1024)), bf(aud.reshape(B * 32, 1024)), \
            bf(vas.reshape(B, 1024))
        ctx.masks = ga.masks(case["mask"])
        y = m.run_cross(ctx, n, zero, S, temporal=False)
    else:
        ctx.id_mean, ctx.audio_mean, ctx.vasa_mean = bf(ide.reshape(B, 1024)), bf(aud.reshape(B * 32, 1024)), \
            bf(vas.reshape(B, 1024))
        y = m.run_cross(ctx, n, zero, S, temporal=True)
    y = y.float().cpu()
    if case["kind"] in ("self_t", "ip_t"):
        y = y.view(B, Fr, S, C).permute(0, 2, 1, 3).reshape(B * S, Fr, C)
    else:
        y = y.view(B, S, C)
    got = ga.subsample(y, case)
    want = load_file(os.path.join(GOLD, f"attn_{name}.safetensors"))["y"]
    assert got.shape == want.shape
    err = ((got - want).norm() / want.norm()).item()
    assert err < 2e-2, err
