"""GPU parity at the BASELINE geometry and over the full 25-step schedule.

* UNet forward at 576x1024 (latent 72x128), real widths 320/640/1280/1280 and heads 5/10/20/20,
  B = 1 CFG branch x F = 2 frames, four mask cases (modes 0 / 1 / 2 and half masks), against the fp32
  oracle's output on the same seeded weights and inputs (tests/golden/unet_full_*.safetensors,
  tools/gen_golden_full.py). This is the shape the reference's UNet call runs (v10:362-517) with
  S0 = 9216 spatial attention and Mamba scans of length 9249 / 2337 / 609 (mamba_layer.py:1532).
  Tolerance (bf16 activations, fp32 accumulation vs fp32 CPU): relative L2 <= 2e-2 and max |err| <=
  0.25 on an output of rms ~1 (measured values are printed and, with ACTH_PARITY_LOG set, appended
  to that file as JSON lines).
* The selective scan at the level shapes (L = 9249 / 9218 / 2337 / 609, D = 640 / 1280 / 2560) and
  flash attention at S = 9216 (5 heads) and 2304 (10 heads) against the oracle's restatements.
* The sampler loop over all 25 Karras steps (sigma 700 -> 0.002) for modes 0 / 1 / 2 against the
  oracle loop's final latents (tests/golden/loop25_*.safetensors, tools/gen_golden_loop.py).
"""
import json
import os

import pytest
import torch
import torch.nn.functional as F
from safetensors.torch import load_file

from oracle import reference_cpu as ref
from tests import golden_full as gf
from tests import golden_loop as gl

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _stats(got, want):
    got = got.float().cpu()
    want = want.float().cpu()
    d = got - want
    return dict(rel_l2=(d.norm() / want.norm()).item(), max_abs=d.abs().max().item(),
                ref_rms=want.pow(2).mean().sqrt().item())


def _log(name, st):
    print(name, json.dumps(st))
    path = os.environ.get("ACTH_PARITY_LOG")
    if path:
        with open(path, "a") as fh:
            fh.write(json.dumps(dict(test=name, **st)) + "\n")


# ------------------------------------------------------------------------------------------ UNet
@pytest.fixture(scope="module")
def full_unet(dev):
    unet = gf.build_full_unet()
    sd = unet.state_dict()
    wsum = gf.checksum(*[sd[k] for k in sorted(sd)])
    return unet.to(dev), wsum


@pytest.mark.parametrize("case", gf.CASES)
def test_unet_full_geometry_matches_oracle(dev, full_unet, case):
    unet, wsum = full_unet
    g = load_file(os.path.join(GOLD, f"unet_full_{case}.safetensors"))
    # fp64 sums over 1.8 B values: the reduction order (thread count) moves the last digits only
    torch.testing.assert_close(wsum, g["weights_checksum"], rtol=1e-6, atol=1e-6)
    sample, t, ehs, added, pose, masks = gf.case_inputs(case)
    torch.testing.assert_close(gf.checksum(sample, ehs[0], *ehs[1], pose, *masks), g["inputs_checksum"],
                               rtol=1e-6, atol=1e-6)
    out = unet(sample.to(dev), t.to(dev), (ehs[0].to(dev), [e.to(dev) for e in ehs[1]]), added.to(dev),
               spatial_condition=pose.to(dev), cross_attention_kwargs={"ip_adapter_masks": masks},
               return_dict=False)[0]
    st = _stats(out, g["out"])
    rpath = os.path.join(GOLD, f"unet_full_{case}_rounded.safetensors")
    if os.path.exists(rpath):
        # the fp16 budget (tools/gen_golden_fp16.py): the reference's shipped fp16 path (inference.yaml:66)
        # modelled as the oracle with fp16 weights / op inputs / outputs, and the same model at bf16
        rd = load_file(rpath)
        st["fp16_ref_path_rel_l2"] = _stats(rd["fp16"], g["out"])["rel_l2"]
        st["bf16_rounding_rel_l2"] = _stats(rd["bf16"], g["out"])["rel_l2"]
        st["vs_fp16_ref_path_rel_l2"] = _stats(out, rd["fp16"])["rel_l2"]
    _log(f"unet_full_{case}", st)
    assert torch.isfinite(out).all()
    assert st["rel_l2"] < 2e-2, st
    # max |err| gate ~3x the measured 0.031-0.045 on outputs of rms ~0.55-0.62 (profiles/r3_final_parity.jsonl)
    assert st["max_abs"] < 0.25 * st["ref_rms"], st
    if "bf16_rounding_rel_l2" in st:
        # stated tolerance: the HIP bf16 error stays within 1.5x of what bf16 rounding at op boundaries alone
        # costs (fp16 rounding costs ~8x less: 3 more mantissa bits)
        assert st["rel_l2"] < 1.5 * st["bf16_rounding_rel_l2"], st


@pytest.mark.parametrize("case", ["mode0", "half"])
def test_unet_full_geometry_fp16_matches_fp16_budget(dev, full_unet, case):
    """The fp16 activation path (libactalker_hip_f16.so, UNet.acth_compute_dtype = float16 -- what an fp16
    UNet selects by itself, the reference's shipped weight_dtype, Inference.py:168-173) at 576x1024 against
    the fp32 oracle. Stated tolerance: within 1.5x of the deviation the oracle itself shows when every op's
    weights / inputs / outputs are rounded to fp16 (tests/golden/unet_full_*_rounded.safetensors "fp16",
    tools/gen_golden_fp16.py) -- 1.6-1.8e-3, ~8x tighter than the bf16 bound above."""
    unet, _ = full_unet
    g = load_file(os.path.join(GOLD, f"unet_full_{case}.safetensors"))
    rd = load_file(os.path.join(GOLD, f"unet_full_{case}_rounded.safetensors"))
    sample, t, ehs, added, pose, masks = gf.case_inputs(case)
    unet.acth_compute_dtype = torch.float16
    try:
        out = unet(sample.to(dev), t.to(dev), (ehs[0].to(dev), [e.to(dev) for e in ehs[1]]), added.to(dev),
                   spatial_condition=pose.to(dev), cross_attention_kwargs={"ip_adapter_masks": masks},
                   return_dict=False)[0]
    finally:
        unet.acth_compute_dtype = None
    st = _stats(out, g["out"])
    st["fp16_ref_path_rel_l2"] = _stats(rd["fp16"], g["out"])["rel_l2"]
    st["vs_fp16_ref_path_rel_l2"] = _stats(out, rd["fp16"])["rel_l2"]
    _log(f"unet_full_{case}_fp16", st)
    assert torch.isfinite(out).all()
    assert st["rel_l2"] < 1.5 * st["fp16_ref_path_rel_l2"], st
    assert st["max_abs"] < 0.05 * st["ref_rms"], st


# ------------------------------------------------------------------------------------------ scan
def _bf(t):
    return t.to(torch.bfloat16)


@pytest.mark.parametrize("xdt", ["f32", "bf16", "bf16q"])
@pytest.mark.parametrize("S,C,n_cond", [(9216, 320, 33), (9216, 320, 2), (2304, 640, 33), (576, 1280, 33)])
def test_selective_scan_level_shapes(dev, S, C, n_cond, xdt, monkeypatch):
    """One batch element of a level's scan: L = S + n_cond (audio branch 33 = ID + 32 audio tokens,
    expression branch 2 = ID + 1 VASA token), D = d_inner = 2C, R = ceil(C / 16), outputs kept for
    the S image tokens (mamba_layer.py:1965-1969, 1505-1548). xdt: the x_proj rows fed to the scan in
    fp32 (paired-lane kernel) or bf16 (scan_quad_kernel; the reference's half-precision x_dbl,
    mamba_layer.py:1521, which the oracle then also uses)."""
    from actalker_amd import ops
    monkeypatch.setattr(ops, "SCAN_ALGO", 1 if xdt == "bf16q" else 0)
    g = torch.Generator().manual_seed(S + n_cond)
    D, R, L = 2 * C, -(-C // 16), S + n_cond
    u = _bf(torch.randn(L, D, generator=g))
    xproj = torch.randn(2 * (R + 32), D, generator=g) * D ** -0.5
    dtw = (torch.rand(2, D, R, generator=g) * 2 - 1) * R ** -0.5
    dt = torch.exp(torch.rand(2, D, generator=g) * (torch.log(torch.tensor(0.1)) - torch.log(torch.tensor(0.001)))
                   + torch.log(torch.tensor(0.001)))
    dtb = dt + torch.log(-torch.expm1(-dt))
    alog = torch.log(torch.arange(1, 17).float()).repeat(2 * D, 1) + 0.1 * torch.randn(2 * D, 16, generator=g)
    Dp = 1 + 0.1 * torch.randn(2 * D, generator=g)
    xdbl = u.float() @ _bf(xproj).float().t()
    if xdt != "f32":
        xdbl = _bf(xdbl)
    y0, y1 = ops.selective_scan(u.to(dev), xdbl.to(dev), dtw.to(dev), dtb.to(dev), alog.to(dev), Dp.to(dev),
                                nb=1, L=L, R=R, n_keep=S)
    W = R + 32
    x = u.float().t()[None]                                        # (1, D, L)
    xs = torch.stack([x, torch.flip(x, dims=[-1])], 1)
    x_dbl = torch.einsum("b k d l, k c d -> b k c l", xs, _bf(xproj).float().view(2, W, D))
    if xdt != "f32":
        x_dbl = _bf(x_dbl).float()
    dts, Bs, Cs = torch.split(x_dbl, [R, 16, 16], dim=2)
    dts = torch.einsum("b k r l, k d r -> b k d l", dts, dtw)
    out = ref.selective_scan_ref(xs.reshape(1, 2 * D, L), dts.reshape(1, 2 * D, L), -torch.exp(alog), Bs, Cs, Dp,
                                 delta_bias=dtb.reshape(-1), delta_softplus=True).view(1, 2, D, L)
    r0 = out[0, 0, :, :S].t()
    r1 = torch.flip(out[0, 1], dims=[-1])[:, :S].t()
    s0, s1 = _stats(y0, r0), _stats(y1, r1)
    _log(f"scan_L{L}_D{D}_{xdt}", dict(dir0=s0, dir1=s1))
    assert s0["rel_l2"] < 1e-2 and s1["rel_l2"] < 1e-2, (s0, s1)


@pytest.mark.parametrize("S,heads", [(9216, 5), (2304, 10)])
def test_flash_attn_level_shapes(dev, S, heads):
    from actalker_amd import ops
    g = torch.Generator().manual_seed(S)
    C = heads * 64
    qkv = _bf(torch.randn(S, 3 * C, generator=g))
    out = ops.flash_attn(qkv.to(dev), 1, S, heads)
    q, k, v = qkv.float().view(1, S, 3, heads, 64).permute(2, 0, 3, 1, 4)
    refo = F.scaled_dot_product_attention(q, k, v).permute(0, 2, 1, 3).reshape(S, C)
    st = _stats(out, refo)
    _log(f"flash_S{S}_H{heads}", st)
    assert st["rel_l2"] < 1e-2, st


# ------------------------------------------------------------------------------------------ loop
@pytest.fixture(scope="module")
def loop_unet(dev):
    import __graft_entry__ as ge
    unet, cfg = ge._tiny_unet(seed=gl.UNET_SEED)
    return unet.to(dev)


@pytest.mark.parametrize("mode", sorted(gl.GATES))
def test_pipeline_25_steps_matches_oracle(dev, loop_unet, mode):
    """All 25 Karras steps (sigma 700 -> 0.002) of the windowed 4-way-CFG loop, dedup on (modes 0 / 1
    evaluate 3 branches), vs the oracle loop's final latents. Tolerance: relative L2 <= 3e-2 on the
    final latents (bf16 UNet, fp32 latent state)."""
    from actalker_amd import pipeline as pl
    latents, imgl, ide, aud, vas, pose, added, masks = gl.loop_inputs()
    gate = gl.GATES[mode]
    T = gl.N + gl.FPB
    backend = pl.HipBackend(loop_unet, gl.H, gl.W, masks, gate, added, T, gl.FPB, imgl, ide, aud, vas, pose)
    twins = backend.branch_twins()
    assert twins == {"mode0": {3: 2}, "mode1": {2: 1}, "mode2": {}}[mode]
    lc = pl.LoopConfig(num_frames=gl.N, frames_per_batch=gl.FPB, overlap=0, shift_offset=gl.SHIFT,
                       num_inference_steps=25)
    with torch.no_grad():
        got = pl.denoise(backend, latents, lc)
    want = load_file(os.path.join(GOLD, f"loop25_{mode}.safetensors"))["latents"]
    st = _stats(got, want)
    _log(f"loop25_{mode}", st)
    assert torch.isfinite(got).all()
    assert st["rel_l2"] < 3e-2, st
    assert st["max_abs"] < 0.25 * st["ref_rms"], st


@pytest.mark.parametrize("mode", ["mode0", "mode2"])
def test_pipeline_25_steps_real_width_matches_oracle(dev, full_unet, mode):
    """The same 25-step windowed 4-way-CFG loop on the REAL-WIDTH UNet (320 / 640 / 1280 / 1280 channels,
    synthetic weights of the full-geometry cases) at a 16x32 latent, vs the fp32 oracle loop
    (tools/gen_golden_loop_full.py). Stated tolerance: the HIP bf16 loop stays within 1.5x of the deviation
    the bf16-rounded oracle loop itself accumulates over the 25 steps (every op's inputs / outputs rounded
    at its boundary, oracle/precision.py), and below 5e-2 absolute."""
    from actalker_amd import pipeline as pl
    path = os.path.join(GOLD, f"loop25_full_{mode}.safetensors")
    if not os.path.exists(path):
        pytest.skip("real-width loop fixture not generated (tools/gen_golden_loop_full.py)")
    g = load_file(path)
    unet, wsum = full_unet
    torch.testing.assert_close(wsum, g["weights_checksum"], rtol=1e-6, atol=1e-6)
    latents, imgl, ide, aud, vas, pose, added, masks = gl.loop_inputs(pose_ch=320)
    T = gl.N + gl.FPB
    backend = pl.HipBackend(unet, gl.H, gl.W, masks, gl.GATES[mode], added, T, gl.FPB, imgl, ide, aud, vas, pose)
    lc = pl.LoopConfig(num_frames=gl.N, frames_per_batch=gl.FPB, overlap=0, shift_offset=gl.SHIFT,
                       num_inference_steps=25)
    with torch.no_grad():
        got = pl.denoise(backend, latents, lc)
    want, want_b = g["latents"], g["latents_bf16"]
    st = _stats(got, want)
    st["bf16_rounding_rel_l2"] = ((want_b - want).norm() / want.norm()).item()
    _log(f"loop25_full_{mode}", st)
    assert torch.isfinite(got).all()
    assert st["rel_l2"] < 5e-2, st
    assert st["rel_l2"] < 1.5 * st["bf16_rounding_rel_l2"], st
    assert st["max_abs"] < 0.25 * st["ref_rms"], st


@pytest.mark.parametrize("act", ["bf16", "fp16"])
def test_c1_loop_matches_cpu_oracle(dev, full_unet, act):
    """BASELINE C1 end to end: mode 0, 14 frames, 25 steps, 576x576 (latent 72x72), fpb 14,
    shift 7, the full-size UNet -- the HIP loop on exactly the workload tools/gen_golden_c1.py ran through the fp32
    oracle on the CPU (tests/golden_c1.py). Stated tolerance: the bf16-rounding floor the real-width loop measures
    (1.5-1.8e-2 after 25 steps, test above) with the same 1.5x factor when the bf16-rounded C1 loop is present,
    else rel-L2 < 5e-2 (the absolute cap of the real-width loop test). ``act``: the UNet's activation dtype (fp16:
    the reference's shipped weight_dtype), held to the same bound."""
    from actalker_amd import pipeline as pl
    from tests import golden_c1 as gc
    path = os.path.join(GOLD, "c1_loop25_mode0.safetensors")
    if not os.path.exists(path):
        pytest.skip("C1 oracle loop fixture not generated (tools/gen_golden_c1.py)")
    g = load_file(path)
    unet, wsum = full_unet
    torch.testing.assert_close(wsum, g["weights_checksum"], rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(gc.inputs_checksum(), g["inputs_checksum"], rtol=1e-6, atol=1e-6)
    latents, imgl, ide, aud, vas, pose, added, masks = gc.loop_inputs()
    T = gc.N + gc.FPB
    backend = pl.HipBackend(unet, gc.H, gc.W, masks, gc.GATE, added, T, gc.FPB, imgl, ide, aud, vas, pose)
    assert backend.branch_twins() == {3: 2}
    lc = pl.LoopConfig(num_frames=gc.N, frames_per_batch=gc.FPB, overlap=gc.OVERLAP, shift_offset=gc.SHIFT,
                       num_inference_steps=25, guidance=gc.GUIDANCE)
    unet.acth_compute_dtype = torch.float16 if act == "fp16" else torch.bfloat16
    try:
        backend = pl.HipBackend(unet, gc.H, gc.W, masks, gc.GATE, added, T, gc.FPB, imgl, ide, aud, vas, pose)
        with torch.no_grad():
            got = pl.denoise(backend, latents, lc)
    finally:
        unet.acth_compute_dtype = None
    want = g["latents"]
    st = _stats(got, want)
    # No rounded C1 *loop* exists (the fp32 oracle loop alone took 19 671 s; a rounded one ~11 CPU-hours). The loop
    # is held to 1.5x the rounding floor of one C1 window call instead (tests/golden/unet_c1win14_mode0_floor:
    # the oracle under bf16 / fp16 rounding against the reference run, largest unit): the 25-step loop's own
    # deviation measured at that call floor's size (bf16 1.72e-2 vs 1.72-1.80e-2, fp16 2.20e-3 vs 2.21-2.25e-3,
    # profiles/r4_step6_window_twins_parity.jsonl, r6_c1_floor.log), capped at the former fixed bounds.
    tol = 5e-3 if act == "fp16" else 5e-2
    fpath = os.path.join(GOLD, "unet_c1win14_mode0_floor.safetensors")
    if os.path.exists(fpath):
        fl = load_file(fpath)["fp16" if act == "fp16" else "bf16"]
        st["c1_call_floor_rel_l2"] = float(fl.max())
        tol = min(tol, 1.5 * st["c1_call_floor_rel_l2"])
    if "latents_bf16" in g and act == "bf16":
        st["bf16_rounding_rel_l2"] = ((g["latents_bf16"] - want).norm() / want.norm()).item()
        tol = min(tol, 1.5 * st["bf16_rounding_rel_l2"])
    st["tol"] = tol
    _log(f"c1_loop25_mode0_{act}", st)
    assert torch.isfinite(got).all()
    assert st["rel_l2"] < tol, st
    assert st["max_abs"] < 0.25 * st["ref_rms"], st


# ------------------------------------------------------------------------------------------ reference run
@pytest.mark.parametrize("case", ["tiny_mode0", "tiny_mode1", "tiny_mode2", "tiny_half", "tiny_box", "tiny_f25_half",
                                  "tiny_f25_mode2", "full_half", "full_mode0", "full_mode2", "c1_face0"])
def test_unet_matches_reference_run(dev, request, case):
    """HIP UNet forward against the REFERENCE UNet package's own forward (v10:362-517 and everything under it,
    run unchanged on the CPU by tools/gen_golden_unet_ref.py; only the diffusers leaves and the scan math
    restated). Tolerance as the oracle comparison: bf16 activations vs fp32, rel-L2 <= 2e-2."""
    from tests import golden_unet_ref as gu
    g = load_file(os.path.join(GOLD, f"unet_ref_{case}.safetensors"))
    if case in gu.FULL_CASES:                      # the module's full-size UNet: same seed, same checksum
        unet, wsum = request.getfixturevalue("full_unet")
    else:
        unet = gu.build_hip_unet(case)
        sd = unet.state_dict()
        wsum = gf.checksum(*[sd[k] for k in sorted(sd)])
        unet = unet.to(dev)
    torch.testing.assert_close(wsum, g["weights_checksum"], rtol=1e-6, atol=1e-6)
    sample, t, ehs, added, pose, masks = gu.case_inputs(case)
    torch.testing.assert_close(gf.checksum(sample, ehs[0], *ehs[1], pose, *masks), g["inputs_checksum"],
                               rtol=1e-6, atol=1e-6)
    out = unet(sample.to(dev), t.to(dev), (ehs[0].to(dev), [e.to(dev) for e in ehs[1]]), added.to(dev),
               spatial_condition=pose.to(dev), cross_attention_kwargs={"ip_adapter_masks": masks},
               return_dict=False)[0]
    st = _stats(out, g["out"])
    _log(f"unet_ref_{case}", st)
    assert torch.isfinite(out).all()
    assert st["rel_l2"] < 2e-2, st
    # ~3x the measured max |err| (0.032-0.045 at rms ~0.57-0.62, profiles/r3_final_parity.jsonl)
    assert st["max_abs"] < 0.25 * st["ref_rms"], st


# ------------------------------------------------------------------------------------------ reference sampler run
@pytest.mark.parametrize("act", ["bf16", "fp16"])
@pytest.mark.parametrize("case", ["mode0", "mode1", "mode2", "f25_mode0", "f25_mode2"])
def test_pipeline_call_matches_reference_pipeline_run(dev, case, act):
    """The product Pose2VideoLongSVDPipeline.__call__ (actalker_amd/pipeline_svd.py: CFG stacking, add_noise,
    masks / pose plumbing, per-step guidance, the HIP loop) against the REFERENCE pipeline's own __call__
    (pipeline:351-773, run unchanged on the CPU by tools/gen_golden_pipeline_ref.py with the reference UNet
    package at the same tiny widths and the reference scheduler mirror), 25 steps, output_type="latent", the
    same deterministic VAE / ID-projection / pose-guider stand-ins (tests/golden_pipeline.py). Stated tolerance:
    within 1.5x of the deviation the bf16-rounded oracle version of the same run accumulates over the 25 steps
    (tools/gen_golden_pipeline_floor.py; the per-step guidance here reaches 7.5, so the rounding floor is higher
    than the constant-guidance loop's), and below 5e-2. ``f25_*``: the reference's shipped window, frames_per_batch =
    n_sample_frames = 25 (config/inference.yaml:4 -> Inference.py:573) with shift_offset 7, at a 8x16 latent. ``act`` fp16: the UNet with fp16 activations (the reference's
    shipped weight_dtype) held to 1.5x the fp16-rounded oracle run's deviation (``latents_fp16``) when present."""
    from actalker_amd.pipeline_svd import Pose2VideoLongSVDPipeline
    from tests import golden_pipeline as gp
    from tests import golden_unet_ref as gu
    path = os.path.join(GOLD, f"pipeline_ref_{case}.safetensors")
    if not os.path.exists(path):
        pytest.skip("reference pipeline fixture not generated (tools/gen_golden_pipeline_ref.py)")
    g = load_file(path)
    unet = gu.build_hip_unet("tiny_mode0")
    sd = unet.state_dict()
    torch.testing.assert_close(gf.checksum(*[sd[k] for k in sorted(sd)]), g["weights_checksum"], rtol=1e-6, atol=1e-6)
    gate, overlap, shift = gp.CASES[case]
    vae, idp, pg = gp.standins(gu.TINY_CFG["block_out_channels"][0])
    pipe = Pose2VideoLongSVDPipeline(vae, unet, idp, pg).to(dev)
    if act == "fp16":
        unet.acth_compute_dtype = torch.float16
    raw = gp.raw_inputs(case=case)
    with torch.no_grad():
        got = pipe(**raw, generator=torch.Generator().manual_seed(gp.GEN_SEED), output_type="latent",
                   return_dict=False, overlap=overlap, shift_offset=shift, gate=gate, **gp.call_kwargs(case))
    st = _stats(got, g["latents"])
    tol = 3e-2
    fpath = os.path.join(GOLD, f"pipeline_floor_{case}.safetensors")
    key = "latents_fp16" if act == "fp16" else "latents_bf16"
    if os.path.exists(fpath):
        fl = load_file(fpath)
        if key in fl:
            st[f"{act}_rounding_rel_l2"] = ((fl[key] - fl["latents"]).norm() / fl["latents"].norm()).item()
            tol = min(5e-2, 1.5 * st[f"{act}_rounding_rel_l2"])
    _log(f"pipeline_ref_{case}" + ("_fp16" if act == "fp16" else ""), st)
    assert torch.isfinite(got).all()
    assert st["rel_l2"] < tol, st
    assert st["max_abs"] < 0.25 * st["ref_rms"], st


# ------------------------------------------------------------------------------------------ headline window call
@pytest.mark.parametrize("mode,frames,w_px", [(0, 14, 1024), (1, 14, 1024), (2, 14, 1024), (0, 25, 1024), (0, 14, 576)])
@pytest.mark.parametrize("act", ["bf16", "fp16"])
def test_headline_window_call_matches_reference_run(dev, full_unet, act, mode, frames, w_px):
    """The call the headline times, held to the REFERENCE UNet run at that shape: one
    14-frame window at 576x1024, its mode-0 CFG branches (uncond / drop audio+vasa / drop vasa) as three units
    of ONE HipBackend.run_units call -- window-input scaling, the CFG prefix shared by branches 1 and 2, the batched
    per-call context projections, automatic units per call -- against tools/gen_golden_unet_ref.py's
    ``win14_mode0`` (the reference UNet package by path, B = 3 x F = 14, inputs stacked as pipeline:712-729 does).
    ``mode`` 2: the C4 / C5 workload's call, all four branches (no twin; branches 1-3 share the prefix) with the
    masks [mouth, exp], against ``win14_mode2``. ``mode`` 1 (expression-only): branch 2 is branch 1's twin, so the
    call evaluates branches 0, 1, 3, against ``win14_mode1`` (the reference run for those three). ``frames`` 25: the
    reference's shipped window (config/inference.yaml:4 n_sample_frames) at 576x1024, mode 0, against ``win25_mode0``:
    the temporal attention's two-block (F <= 32) kernel at the real widths. ``w_px`` 576: BASELINE C1's geometry
    (576x576), mode 0, against ``c1win14_mode0``, each unit held to 1.5x C1's own rounding floor for that unit
    (tests/golden/unet_c1win14_mode0_floor.safetensors: bf16 1.72-1.80e-2, fp16 2.2e-3 -- the 576x576 call loses
    more to bf16 rounding than the 576x1024 one's 1.40e-2), capped at 2e-2.
    Stated tolerance per unit: 1.5x the bf16 (fp16) rounding floor the oracle shows at this geometry and weights
    (tests/golden/unet_full_mode0_rounded.safetensors for mode 0, unet_full_half_rounded.safetensors -- the same
    [lower, upper] mask split with both prompts live -- for mode 2: every op's inputs / outputs rounded at its
    boundary), capped at 2e-2 as every UNet golden; max |err| < 0.25 x output rms."""
    from actalker_amd import pipeline as pl
    from tests import golden_win14 as gw
    case = f"win{frames}_mode{mode}" if w_px == 1024 else f"c1win{frames}_mode{mode}"
    H, W = gw.H_PX // 8, w_px // 8
    path = os.path.join(GOLD, f"unet_ref_{case}.safetensors")
    if not os.path.exists(path):
        pytest.skip(f"headline-window reference fixture not generated (tools/gen_golden_unet_ref.py {case})")
    g = load_file(path)
    unet, wsum = full_unet
    torch.testing.assert_close(wsum, g["weights_checksum"], rtol=1e-6, atol=1e-6)
    sample, t, ehs, added_r, pose_r, masks_r = gw.reference_inputs(mode=mode, frames=frames, w_px=w_px)
    torch.testing.assert_close(gf.checksum(sample, ehs[0], *ehs[1], pose_r, *masks_r), g["inputs_checksum"],
                               rtol=1e-6, atol=1e-6)
    nb, gate = gw.MODES[mode]["nb"], gw.MODES[mode]["gate"]
    lat, imgl, ide, aud, vas, pose, added, masks = gw.loop_tensors(mode=mode, frames=frames, w_px=w_px)
    fcase = "half" if mode == 2 else "mode0"
    floor = load_file(os.path.join(GOLD, f"unet_full_{fcase}_rounded.safetensors"))
    full = load_file(os.path.join(GOLD, f"unet_full_{fcase}.safetensors"))["out"]
    fl = _stats(floor["fp16" if act == "fp16" else "bf16"], full)["rel_l2"]
    fl_unit = None
    c1_floor = os.path.join(GOLD, f"unet_{case}_floor.safetensors")
    if w_px != 1024 and os.path.exists(c1_floor):
        # C1's own rounding floor per unit (tools/gen_golden_c1_floor.py: the rounded oracle on this call's inputs
        # against the reference run), in place of the 576x1024 one
        f1 = load_file(c1_floor)
        torch.testing.assert_close(f1["inputs_checksum"], g["inputs_checksum"], rtol=1e-6, atol=1e-6)
        fl_unit = f1["fp16" if act == "fp16" else "bf16"].tolist()
    tol = min(2e-2, 1.5 * fl)
    unet.acth_compute_dtype = torch.float16 if act == "fp16" else torch.bfloat16
    try:
        be = pl.HipBackend(unet, H, W, masks, gate, added, frames, frames, imgl, ide, aud, vas, pose)
        assert be.max_units_per_call() >= nb                 # one call, as the bench's auto split gives
        assert be.prefix_classes() == [0] + [1] * (nb - 1)   # branches 1.. share the UNet prefix
        twins = {2: 1} if mode == 1 else {}
        assert be.branch_twins() == twins
        branches = [c for c in range(nb) if c not in twins]
        win = [list(range(frames))]
        state = be.new_state(lat)
        S = H * W
        out = torch.empty((len(branches) * frames * S, 4), device=dev, dtype=torch.float32)
        be.begin_step(win)
        with torch.no_grad():
            be.run_units(state, [(0, c) for c in branches], win, float(t), gw.SIGMA, out, 0)
        torch.cuda.synchronize()
    finally:
        unet.acth_compute_dtype = None
    got = out.view(len(branches), frames, H, W, 4).permute(0, 1, 4, 2, 3)
    want = g["out"]                        # the reference run's elements, in the same order as ``branches``
    assert want.shape[0] == len(branches)
    for c in range(len(branches)):
        st = _stats(got[c], want[c])
        tol_c = tol if fl_unit is None else min(2e-2, 1.5 * fl_unit[c])
        st["rounding_floor_rel_l2"] = fl if fl_unit is None else fl_unit[c]
        st["tol"] = tol_c
        _log(f"{case}_unit{branches[c]}_{act}", st)
        assert torch.isfinite(got[c]).all()
        assert st["rel_l2"] < tol_c, (c, st)
        assert st["max_abs"] < 0.25 * st["ref_rms"], (c, st)
