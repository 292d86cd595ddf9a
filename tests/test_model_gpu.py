"""GPU parity of the drop-in modules against the reference's golden vectors and the CPU oracle.

Tolerances (bf16 activations, fp32 accumulation, stated per test):
  * SS2D_cond_v10 vs the reference module's own outputs: rel-L2 <= 2e-2
  * UNet forward vs oracle (tiny width, real topology, 3 frames): rel-L2 <= 5e-2
  * 3 sampler steps of the loop vs the oracle loop: rel-L2 <= 5e-2 on the final latents
"""
import os

import pytest
import torch
from safetensors.torch import load_file

import __graft_entry__ as ge
from oracle import reference_cpu as ref
from tests.golden_weights import CASES, golden_weights, make_inputs

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def rel(a, b):
    a = a.float().cpu()
    b = b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("name", sorted(CASES))
def test_ss2d_cond_v10_matches_reference_golden(dev, name):
    from actalker_amd.modules import Ctx, SS2D_cond_v10
    case = CASES[name]
    g = load_file(os.path.join(GOLD, f"ss2d_cond_v10_{name}.safetensors"))
    x, id_emb, conds, masks = make_inputs(case)
    m = SS2D_cond_v10(d_model=case["d_model"], d_cond=case["d_cond"], cond_size=32, dropout=0.1, d_state=16,
                      size=8, scan_type="sweep", num_direction=2)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    m.load_state_dict(golden_weights(case["seed"], shapes), strict=True)
    m = m.to(dev)
    BF, S, C = x.shape
    ctx = Ctx(BF, 1, dev)
    ctx.id_tok = id_emb.reshape(BF, -1).to(dev, torch.bfloat16)
    ctx.audio_tok = conds[:, :32].reshape(BF * 32, -1).to(dev, torch.bfloat16)
    ctx.vasa_tok = conds[:, 32].reshape(BF, -1).to(dev, torch.bfloat16)
    ctx.masks = masks
    y = m.run(ctx, x.reshape(BF * S, C).to(dev, torch.bfloat16), S)
    err = rel(y.view(BF, S, C), g["y"])
    assert err < 2e-2, err


@pytest.mark.parametrize("name", ["l0_mode2", "l0_mode0", "l0_box", "l1_half", "l1_box", "l2_mode2", "l2_mode1",
                                  "l2_box"])
def test_ss2d_cond_v10_level_shapes_match_reference(dev, name):
    """SS2D_cond_v10 at the BASELINE level shapes -- S = 9216 / 2304 / 576 (scans of L = S + 33 / S + 2), the
    real 576x1024 masks truncated to the level grids (mamba_layer.py:1962-1981) -- against the reference
    module's own outputs (tools/gen_golden.py levels), every ``sub``-th token row. Tolerance rel-L2 <= 2e-2."""
    from actalker_amd.modules import Ctx, SS2D_cond_v10
    from tests import golden_full as gf
    from tests.golden_weights import LEVEL_CASES
    case = LEVEL_CASES[name]
    g = load_file(os.path.join(GOLD, f"ss2d_level_{name}.safetensors"))
    x, id_emb, conds, masks = make_inputs(case)
    torch.testing.assert_close(gf.checksum(x, id_emb, conds, *masks), g["inputs_checksum"], rtol=1e-6, atol=1e-6)
    m = SS2D_cond_v10(d_model=case["d_model"], d_cond=case["d_cond"], cond_size=32, dropout=0.1, d_state=16,
                      size=8, scan_type="sweep", num_direction=2)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    m.load_state_dict(golden_weights(case["seed"], shapes), strict=True)
    m = m.to(dev)
    BF, S, C = x.shape
    ctx = Ctx(BF, 1, dev)
    ctx.id_tok = id_emb.reshape(BF, -1).to(dev, torch.bfloat16)
    ctx.audio_tok = conds[:, :32].reshape(BF * 32, -1).to(dev, torch.bfloat16)
    ctx.vasa_tok = conds[:, 32].reshape(BF, -1).to(dev, torch.bfloat16)
    ctx.masks = masks
    y = m.run(ctx, x.reshape(BF * S, C).to(dev, torch.bfloat16), S)
    err = rel(y.view(BF, S, C)[:, ::case["sub"]], g["y_sub"])
    assert err < 2e-2, err


def _oracle_cfg(cfg):
    return dict(block_out_channels=cfg["block_out_channels"], num_attention_heads=cfg["num_attention_heads"])


@pytest.fixture(scope="module")
def tiny(dev):
    unet, cfg = ge._tiny_unet(seed=9)
    sd = {k: v.detach().clone() for k, v in unet.state_dict().items()}
    return unet.to(dev), sd, cfg


@pytest.mark.parametrize("masks_kind", ["mode2", "mode0", "mode1", "half"])
def test_unet_forward_matches_oracle(dev, tiny, masks_kind):
    unet, sd, cfg = tiny
    sample, t, ehs, added, pose, _ = ge._tiny_inputs(B=2, F=3, H=16, W=32, seed=4)
    H8, W8 = 128, 256
    one, zero = torch.ones(1, 1, H8, W8), torch.zeros(1, 1, H8, W8)
    lower = zero.clone()
    lower[..., H8 // 2:, :] = 1.0
    masks = {"mode2": [one, one], "mode0": [one, zero], "mode1": [zero, one], "half": [lower, 1 - lower]}[masks_kind]
    if masks_kind == "mode0":
        ehs = (ehs[0], [ehs[1][0], torch.zeros_like(ehs[1][1])])
    if masks_kind == "mode1":
        ehs = (ehs[0], [torch.zeros_like(ehs[1][0]), ehs[1][1]])
    cak = {"ip_adapter_masks": masks}
    out = unet(sample.to(dev), t.to(dev), (ehs[0].to(dev), [e.to(dev) for e in ehs[1]]), added.to(dev),
               spatial_condition=pose.to(dev), cross_attention_kwargs=cak, return_dict=False)[0]
    want = ref.unet_forward(sd, sample, t, ehs, added, pose, cak, ip_scale=(1.25, 1.25), cfg=_oracle_cfg(cfg))
    err = rel(out, want)
    assert err < 5e-2, err


class _RefAttnProcessor2_0(torch.nn.Module):
    """Stand-in with the reference's attribute surface (attention_processor.py:1518-1527): no params."""


class _RefIPAdapterAttnProcessor2_0(torch.nn.Module):
    """Stand-in with the reference IPAdapterAttnProcessor2_0's attribute surface (attention_processor.py:
    2717-2745): plain torch Linear lists ``to_k_ip`` / ``to_v_ip``, ``scale`` and ``num_tokens`` lists."""

    def __init__(self, hidden_size, cross_attention_dim, num_tokens, scale):
        super().__init__()
        self.hidden_size, self.cross_attention_dim = hidden_size, cross_attention_dim
        self.num_tokens, self.scale = num_tokens, scale
        self.to_k_ip = torch.nn.ModuleList([torch.nn.Linear(cross_attention_dim, hidden_size, bias=False)
                                            for _ in num_tokens])
        self.to_v_ip = torch.nn.ModuleList([torch.nn.Linear(cross_attention_dim, hidden_size, bias=False)
                                            for _ in num_tokens])


def test_reference_processor_objects_drive_the_unet(dev):
    """The reference's unmodified add_ip_adapters / load_adapter_states (unet_spatio_temporal_condition.py:
    519-591) hand the UNet the reference's own processor objects through set_attn_processor and then load
    weights into them: the HIP UNet runs them as its own (same output bitwise, same state_dict keys) and
    picks up weights loaded into them afterwards (packs keyed on the tensors' version counters)."""
    unet, cfg = ge._tiny_unet(seed=11)
    unet = unet.to(dev)
    sample, t, ehs, added, pose, masks = ge._tiny_inputs(B=1, F=3, H=16, W=32, seed=6)
    args = (sample.to(dev), t.to(dev), (ehs[0].to(dev), [e.to(dev) for e in ehs[1]]), added.to(dev))
    kw = dict(spatial_condition=pose.to(dev), cross_attention_kwargs={"ip_adapter_masks": masks}, return_dict=False)
    ours = unet(*args, **kw)[0]
    keys = sorted(unet.state_dict().keys())
    procs = {}
    for name, p in unet.attn_processors.items():
        if hasattr(p, "to_k_ip"):
            q = _RefIPAdapterAttnProcessor2_0(p.hidden_size, p.cross_attention_dim, [32, 32], [1.25, 1.25]).to(dev)
            q.load_state_dict({k: v.detach().clone() for k, v in p.state_dict().items()})
            procs[name] = q
        else:
            procs[name] = _RefAttnProcessor2_0()
    unet.set_attn_processor(procs)
    assert sorted(unet.state_dict().keys()) == keys
    got = unet(*args, **kw)[0]
    assert torch.equal(got, ours)
    # load_adapter_states-style in-place load into the foreign modules
    adapters = torch.nn.ModuleList([m for m in unet.attn_processors.values()
                                    if isinstance(m, _RefIPAdapterAttnProcessor2_0)])
    sd = {k: (0.5 * v) if ".to_v_ip.0." in k else v for k, v in adapters.state_dict().items()}
    adapters.load_state_dict(sd)
    changed = unet(*args, **kw)[0]
    assert not torch.equal(changed, ours)
    # the same weights through the build's own processors give the same output
    own = {}
    for name, p in unet.attn_processors.items():
        if hasattr(p, "to_k_ip"):
            from actalker_amd.modules import IPAdapterAttnProcessor2_0
            q = IPAdapterAttnProcessor2_0(p.hidden_size, p.cross_attention_dim, [32, 32], [1.25, 1.25]).to(dev)
            q.load_state_dict({k: v.detach().clone() for k, v in p.state_dict().items()})
            own[name] = q
        else:
            from actalker_amd.modules import AttnProcessor2_0
            own[name] = AttnProcessor2_0()
    unet.set_attn_processor(own)
    assert torch.equal(unet(*args, **kw)[0], changed)


def test_cfg_prefix_sharing_matches_full_batch(dev, tiny):
    """forward_tokens(prefix_src=...): batch elements whose prefix inputs are equal (latent + image rows,
    pose, timestep, added time ids) run conv_in .. the first attn1 once; outputs match the unshared call
    (rows are computed per element; only GEMM tile choices for the smaller M may differ)."""
    from actalker_amd import ops
    unet, sd, cfg = tiny
    sample, t, ehs, added, pose, masks = ge._tiny_inputs(B=3, F=3, H=16, W=32, seed=8)
    sample[2] = sample[1]                              # elements 1, 2: same prefix inputs,
    added[2] = added[1]                                # different audio / VASA / ID prompts
    pose[2] = pose[1]
    B, F, H, W = 3, 3, 16, 32
    x = ops.nchw_to_tokens(sample.to(dev))
    sc = ops.nchw_to_tokens(pose.to(dev))
    e = (ehs[0].to(dev), [a.to(dev) for a in ehs[1]])
    cak = {"ip_adapter_masks": masks}
    with torch.no_grad():
        full = unet.forward_tokens(x, B, F, H, W, t.to(dev), e, added.to(dev), sc, cak)
        shared = unet.forward_tokens(x, B, F, H, W, t.to(dev), e, added.to(dev), sc, cak, prefix_src=[0, 1, 1])
        shared_none = unet.forward_tokens(x, B, F, H, W, t.to(dev), e, added.to(dev), sc, cak, prefix_src=[0, 1, 2])
    assert torch.equal(shared_none, full)
    assert rel(shared, full) < 1e-3
    with pytest.raises(ValueError):
        unet.forward_tokens(x, B, F, H, W, t.to(dev), e, added.to(dev), sc, cak, prefix_src=[0, 2, 2])


def test_batched_ctx_projections_match_per_module(dev, tiny):
    """UNet._batched_ctx_projections: every ResBlock's time_emb_proj(temb) and every attn2's to_v(ID token)
    computed as three concatenated-weight GEMMs per call == the per-module GEMMs (only the GEMM tile
    choice for the wider N may differ), with the prefix-sharing context too."""
    from actalker_amd import ops
    unet, sd, cfg = tiny
    sample, t, ehs, added, pose, masks = ge._tiny_inputs(B=3, F=3, H=16, W=32, seed=9)
    B, F, H, W = 3, 3, 16, 32
    x = ops.nchw_to_tokens(sample.to(dev))
    sc = ops.nchw_to_tokens(pose.to(dev))
    e = (ehs[0].to(dev), [a.to(dev) for a in ehs[1]])
    cak = {"ip_adapter_masks": masks}
    try:
        with torch.no_grad():
            unet.acth_batch_ctx_projections = True
            batched = unet.forward_tokens(x, B, F, H, W, t.to(dev), e, added.to(dev), sc, cak)
            unet.acth_batch_ctx_projections = False
            single = unet.forward_tokens(x, B, F, H, W, t.to(dev), e, added.to(dev), sc, cak)
    finally:
        unet.acth_batch_ctx_projections = True
    assert torch.isfinite(batched.float()).all()
    assert rel(batched, single) < 1e-3


def test_ctx_token_cache_reuses_and_invalidates(dev, tiny):
    """The per-call token side of the UNet context (ID / audio / VASA rows, frame means, their batched projections)
    is reused for the same prompt tensors and packed weights, and recomputed -- to the same values -- after an
    in-place write to a prompt tensor or a weight update."""
    from actalker_amd import ops
    unet, sd, cfg = tiny
    sample, t, ehs, added, pose, masks = ge._tiny_inputs(B=3, F=3, H=16, W=32, seed=13)
    B, F = 3, 3
    e = (ehs[0].to(dev), [a.to(dev) for a in ehs[1]])
    cak = {"ip_adapter_masks": masks}
    unet.__dict__.pop("_acth_tok_cache", None)
    attn = unet._ctx_mods()[1][0]                    # first spatial attn2 (its to_v(ID token) is batched)
    w = attn.to_v.weight
    w_old = w.detach().clone()
    try:
        with torch.no_grad(), ops.compute_dtype(unet.compute_dtype()):
            c1 = unet._prep_ctx(B, F, t.to(dev), e, added.to(dev), cak)
            c2 = unet._prep_ctx(B, F, t.to(dev), e, added.to(dev), cak)
            assert c2.vid is c1.vid and c2.id_tok is c1.id_tok and c2.ipkv is c1.ipkv      # hit
            assert c2.tproj is not c1.tproj                                                 # temb: every call
            e[1][0].mul_(1.0)                        # same values, new version: recomputed
            c3 = unet._prep_ctx(B, F, t.to(dev), e, added.to(dev), cak)
            assert c3.vid is not c1.vid
            for k in c1.ipkv:
                assert torch.equal(c3.ipkv[k], c1.ipkv[k])
            w.mul_(2.0)                              # a weight update: new packed weights, new projections
            c4 = unet._prep_ctx(B, F, t.to(dev), e, added.to(dev), cak)
            assert c4.vid is not c3.vid
            assert not torch.equal(c4.vid[id(attn)], c3.vid[id(attn)])
    finally:
        with torch.no_grad():
            w.copy_(w_old)
    assert len(unet.__dict__["_acth_tok_cache"]) <= unet._ACTH_TOK_CACHE


def test_paired_mamba_scan_matches_per_branch(dev, tiny):
    """SS2D_cond_v10 with both branches' scans in one acth_selective_scan2 launch == one launch per branch,
    bit for bit (the tiny inputs' masks select part of each frame, so both branches scan)."""
    from actalker_amd import modules, ops
    unet, sd, cfg = tiny
    sample, t, ehs, added, pose, masks = ge._tiny_inputs(B=3, F=3, H=16, W=32, seed=11)
    B, F, H, W = 3, 3, 16, 32
    x = ops.nchw_to_tokens(sample.to(dev))
    sc = ops.nchw_to_tokens(pose.to(dev))
    e = (ehs[0].to(dev), [a.to(dev) for a in ehs[1]])
    cak = {"ip_adapter_masks": masks}
    mods = [m for m in unet.modules() if isinstance(m, modules.SS2D_cond_v10)]
    assert mods
    try:
        with torch.no_grad():
            paired = unet.forward_tokens(x, B, F, H, W, t.to(dev), e, added.to(dev), sc, cak)
            for m in mods:
                m.acth_pair_scan = False
            single = unet.forward_tokens(x, B, F, H, W, t.to(dev), e, added.to(dev), sc, cak)
    finally:
        for m in mods:
            m.acth_pair_scan = True
    assert torch.isfinite(paired.float()).all()
    assert torch.equal(paired, single)


def test_pipeline_prefix_sharing_matches_unshared_loop(dev, tiny):
    """The sampler loop with LoopConfig.share_cfg_prefix on and off, CFG inputs shaped as the reference
    builds them (pipeline:162-205: branch 0 zero image latents / ID, branches 1-3 equal image latents;
    mode 2, so all four branches run and 1-3 share the prefix)."""
    from actalker_amd import pipeline as pl
    unet, sd, cfg = tiny
    N, fpb, H, W = 4, 2, 16, 32
    T = N + fpb
    g = torch.Generator().manual_seed(23)
    latents = 0.18215 * torch.randn(1, 1, 4, H, W, generator=g) + 700.0 * torch.randn(1, T, 4, H, W, generator=g)
    img1 = torch.randn(1, T, 4, H, W, generator=g)
    imgl = torch.cat([torch.zeros_like(img1), img1, img1, img1])
    ide1 = torch.randn(1, T, 1, 1024, generator=g)
    ide = torch.cat([torch.zeros_like(ide1), ide1, ide1, ide1])
    aud = torch.randn(4, T, 32, 1024, generator=g)
    vas = torch.randn(4, T, 1, 1024, generator=g)
    pose = 0.1 * torch.randn(1, T, 64, H, W, generator=g)
    added = torch.tensor([[12.5, 12.0, 20.0]] * 4)
    lower = torch.zeros(1, 1, 8 * H, 8 * W)
    lower[..., 4 * H:, :] = 1.0
    masks = (torch.ones(1, 1, 8 * H, 8 * W), lower, 1 - lower)
    outs = []
    for share in (True, False):
        backend = pl.HipBackend(unet, H, W, masks, [1, 1], added, T, fpb, imgl, ide, aud, vas, pose)
        assert backend.prefix_classes() == [0, 1, 1, 1]
        lc = pl.LoopConfig(num_frames=N, frames_per_batch=fpb, overlap=0, shift_offset=1, share_cfg_prefix=share)
        with torch.no_grad():
            outs.append(pl.denoise(backend, latents, lc, steps=2))
    assert rel(outs[0], outs[1]) < 2e-3


def test_unet_gate_hint_is_exact(dev, tiny):
    """The pipeline's gate hint only skips work whose result is exactly zero."""
    unet, sd, cfg = tiny
    sample, t, ehs, added, pose, masks = ge._tiny_inputs(B=1, F=3, H=16, W=32, seed=5)
    ehs = (ehs[0], [ehs[1][0], torch.zeros_like(ehs[1][1])])
    masks = [masks[0], torch.zeros_like(masks[1])]
    args = (sample.to(dev), t.to(dev), (ehs[0].to(dev), [e.to(dev) for e in ehs[1]]), added.to(dev))
    a = unet(*args, spatial_condition=pose.to(dev), cross_attention_kwargs={"ip_adapter_masks": masks},
             return_dict=False)[0]
    b = unet(*args, spatial_condition=pose.to(dev),
             cross_attention_kwargs={"ip_adapter_masks": masks, "acth_gate": [1, 0]}, return_dict=False)[0]
    assert rel(a, b) < 1e-3


def test_pipeline_loop_matches_oracle(dev, tiny):
    """3 sampler steps of the windowed 4-way-CFG loop (N=4 frames, window 2, shift 1) vs the oracle."""
    from actalker_amd import pipeline as pl
    unet, sd, cfg = tiny
    N, fpb, H, W = 4, 2, 16, 32
    T = N + fpb
    g = torch.Generator().manual_seed(21)
    latents = 0.18215 * torch.randn(1, 1, 4, H, W, generator=g) + 700.0 * torch.randn(1, T, 4, H, W, generator=g)
    imgl = torch.randn(4, T, 4, H, W, generator=g)
    imgl[0] = 0
    ide = torch.randn(4, T, 1, 1024, generator=g)
    aud = torch.randn(4, T, 32, 1024, generator=g)
    vas = torch.randn(4, T, 1, 1024, generator=g)
    pose = 0.1 * torch.randn(1, T, 64, H, W, generator=g)
    added = torch.tensor([[12.5, 12.0, 20.0]] * 4)
    lower = torch.zeros(1, 1, 8 * H, 8 * W)
    lower[..., 4 * H:, :] = 1.0
    masks = (torch.ones(1, 1, 8 * H, 8 * W), lower, 1 - lower)     # face, mouth, expression
    gate = [1, 1]
    lc = pl.LoopConfig(num_frames=N, frames_per_batch=fpb, overlap=0, shift_offset=1, num_inference_steps=25)
    backend = pl.HipBackend(unet, H, W, masks, gate, added, T, fpb, imgl, ide, aud, vas, pose)
    with torch.no_grad():
        got = pl.denoise(backend, latents, lc, steps=3)

    def unet_fn(sample, t, ehs, added_ids, sc, cak):
        return ref.unet_forward(sd, sample, t, ehs, added_ids, sc, cak, ip_scale=(1.25, 1.25),
                                cfg=_oracle_cfg(cfg))

    want = _oracle_loop(unet_fn, latents, imgl, ide, aud, vas, pose, added, masks, gate, N, fpb, steps=3)
    err = rel(got, want)
    assert err < 5e-2, err


@pytest.mark.parametrize("gate,twins", [([1, 0], {3: 2}), ([0, 1], {2: 1})])
def test_pipeline_loop_twin_branches(dev, tiny, gate, twins):
    """Modes 0 / 1 with the pipeline's CFG stacking (ID [0,e,e,e], audio [u,u,a,a], VASA [u,u,u,v],
    pipeline:162-200, prompts gated at :724): the backend finds the twin branch, the loop evaluates
    3 branches per window and still matches the 4-branch oracle loop (and the 4-branch HIP loop)."""
    from actalker_amd import pipeline as pl
    unet, sd, cfg = tiny
    N, fpb, H, W = 4, 2, 16, 32
    T = N + fpb
    g = torch.Generator().manual_seed(23)
    latents = 0.18215 * torch.randn(1, 1, 4, H, W, generator=g) + 700.0 * torch.randn(1, T, 4, H, W, generator=g)
    il = torch.randn(1, T, 4, H, W, generator=g)
    imgl = torch.cat([torch.zeros_like(il), il, il, il])
    e = torch.randn(1, T, 1, 1024, generator=g)
    ide = torch.cat([torch.zeros_like(e), e, e, e])
    a_u, a_c = torch.randn(1, T, 32, 1024, generator=g), torch.randn(1, T, 32, 1024, generator=g)
    aud = torch.cat([a_u, a_u, a_c, a_c])
    v_u, v_c = torch.randn(1, T, 1, 1024, generator=g), torch.randn(1, T, 1, 1024, generator=g)
    vas = torch.cat([v_u, v_u, v_u, v_c])
    pose = 0.1 * torch.randn(1, T, 64, H, W, generator=g)
    added = torch.tensor([[12.5, 12.0, 20.0]] * 4)
    ones = torch.ones(1, 1, 8 * H, 8 * W)
    masks = (ones, ones, ones)
    backend = pl.HipBackend(unet, H, W, masks, gate, added, T, fpb, imgl, ide, aud, vas, pose)
    assert backend.branch_twins() == twins
    seen = []
    run0 = backend.run_units

    def counting(lat, units, *a, **k):
        seen.extend(units)
        return run0(lat, units, *a, **k)

    backend.run_units = counting
    lc = pl.LoopConfig(num_frames=N, frames_per_batch=fpb, overlap=0, shift_offset=1, num_inference_steps=25)
    with torch.no_grad():
        got = pl.denoise(backend, latents, lc, steps=3)
        assert len(seen) == 3 * 3 * 3 and not any(c in twins for _w, c in seen)
        lc4 = pl.LoopConfig(num_frames=N, frames_per_batch=fpb, overlap=0, shift_offset=1, num_inference_steps=25,
                            dedup_branches=False)
        all4 = pl.denoise(backend, latents, lc4, steps=3)
    assert rel(got, all4) < 1e-2

    def unet_fn(sample, t, ehs, added_ids, sc, cak):
        return ref.unet_forward(sd, sample, t, ehs, added_ids, sc, cak, ip_scale=(1.25, 1.25),
                                cfg=_oracle_cfg(cfg))

    want = _oracle_loop(unet_fn, latents, imgl, ide, aud, vas, pose, added, masks, gate, N, fpb, steps=3)
    err = rel(got, want)
    assert err < 5e-2, err


def test_pipeline_loop_padding_window_twins(dev, tiny):
    """Mode 2 with the pipeline's padding (pipeline:170-184): past frame N every branch's audio / VASA prompt is the
    uncond pad (the first uncond frame repeated), and branches 1-3 share the ID embedding and image latents, so in a
    window made only of padding frames branches 2 and 3 receive branch 1's inputs. The loop evaluates 10 instead of
    12 (window, branch) units on the steps with such a window (shift 0 at N = 4, fpb 2: window [4, 5]) and matches
    the loop that evaluates all four branches everywhere on the real HIP UNet."""
    from actalker_amd import pipeline as pl
    unet, sd, cfg = tiny
    N, fpb, H, W = 4, 2, 16, 32
    T = N + fpb
    g = torch.Generator().manual_seed(29)
    latents = 0.18215 * torch.randn(1, 1, 4, H, W, generator=g) + 700.0 * torch.randn(1, T, 4, H, W, generator=g)
    il = torch.randn(1, T, 4, H, W, generator=g)
    imgl = torch.cat([torch.zeros_like(il), il, il, il])
    e = torch.randn(1, T, 1, 1024, generator=g)
    ide = torch.cat([torch.zeros_like(e), e, e, e])
    a_u, a_c = torch.randn(1, T, 32, 1024, generator=g), torch.randn(1, T, 32, 1024, generator=g)
    v_u, v_c = torch.randn(1, T, 1, 1024, generator=g), torch.randn(1, T, 1, 1024, generator=g)
    a_u[:, N:] = a_u[:, :1]              # pad_uncond_audio = uncond_audio[:1] repeated (pipeline:175-179)
    a_c[:, N:] = a_u[:, :1]
    v_u[:, N:] = v_u[:, :1]
    v_c[:, N:] = v_u[:, :1]
    aud = torch.cat([a_u, a_u, a_c, a_c])
    vas = torch.cat([v_u, v_u, v_u, v_c])
    pose = 0.1 * torch.randn(1, T, 64, H, W, generator=g)
    added = torch.tensor([[12.5, 12.0, 20.0]] * 4)
    lower = torch.zeros(1, 1, 8 * H, 8 * W)
    lower[..., 4 * H:, :] = 1.0
    masks = (torch.ones(1, 1, 8 * H, 8 * W), lower, 1 - lower)
    backend = pl.HipBackend(unet, H, W, masks, [1, 1], added, T, fpb, imgl, ide, aud, vas, pose)
    assert backend.branch_twins() == {}
    lc = pl.LoopConfig(num_frames=N, frames_per_batch=fpb, overlap=0, shift_offset=1, num_inference_steps=25)
    plan = []
    with torch.no_grad():
        got = pl.denoise(backend, latents, lc, steps=3, plan_log=plan)
        lc4 = pl.LoopConfig(num_frames=N, frames_per_batch=fpb, overlap=0, shift_offset=1, num_inference_steps=25,
                            dedup_branches=False)
        plan4 = []
        all4 = pl.denoise(backend, latents, lc4, steps=3, plan_log=plan4)
    assert [p["units"] for p in plan] == [10, 12, 10], plan
    assert [p["units"] for p in plan4] == [12, 12, 12], plan4
    assert rel(got, all4) < 1e-2


def _oracle_loop(unet_fn, latents, imgl, ide, aud, vas, pose, added, masks, gate, N, fpb, steps):
    """oracle.denoise_loop truncated to `steps` sampler steps (same schedule)."""
    sig, ts = ref.euler_karras_tables(25)
    T = N + fpb
    lat = latents.clone()
    shift = 0
    for i in range(steps):
        pred = torch.zeros_like(lat)
        cnt = torch.zeros(1, T, 1, 1, 1)
        for index_start in range(0, T, fpb):
            s0 = index_start - shift
            idx = [(j % T) for j in range(s0, s0 + fpb)]
            x = torch.cat([lat[:, idx]] * 4) / ((sig[i] ** 2 + 1) ** 0.5)
            x = torch.cat([x, imgl[:, idx]], dim=2)
            ehs = (ide[:, idx].flatten(0, 1), [aud[:, idx].flatten(0, 1) * gate[0], vas[:, idx].flatten(0, 1) * gate[1]])
            face, mouth, expm = masks                        # pipeline:702-711
            mlist = ([mouth, expm] if gate == [1, 1] else [face, torch.zeros_like(face)] if gate == [1, 0]
                     else [torch.zeros_like(face), face])
            noise = unet_fn(x, ts[i], ehs, added, pose[:, idx].repeat(4, 1, 1, 1, 1), {"ip_adapter_masks": mlist})
            u, dav, dv, c = noise.chunk(4)
            eps = u + 2.0 * (dav - u) + 7.5 * (dv - dav) + 3.0 * (c - dv)
            out = ref.euler_step_v(eps, sig[i], sig[i + 1], lat[:, idx])
            for j in range(fpb):
                pred[:, (s0 + j) % T] += out[:, j]
                cnt[:, (s0 + j) % T] += 1
        shift = (shift + 1) % fpb
        lat = pred / cnt
    return lat
