"""Benchmark: denoised frames/sec of ACTalker's 25-step audio-driven denoising at 576x1024, 14 frames
per GPU (BASELINE.json metric), on 1..8 MI355X with one process per GPU.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N --steps K --warmup W

A "step" is one sampler step of the loop (pipeline:671): every window x CFG-branch UNet pass
(one 84-frame call in modes 0/1, two 56-frame calls in mode 2, at N=14 on one GPU) + guidance + Euler + window accumulation. In modes 0 / 1 the
gate zeroes the VASA / audio prompts (pipeline:724), so two of the four CFG branches receive
bitwise-identical inputs; that branch is evaluated once and read twice by guidance (identical
output; pipeline.HipBackend.branch_twins), i.e. 3 x 14-frame UNet batches per window. In every mode, a
window lying wholly in the fpb padding frames past N (every other step at N = 14, shift 7) gives branches
1-3 the same inputs -- the same ID embedding and image latents and the uncond audio / VASA pad for all
branches (pipeline:175-184) -- so there branches 2 and 3 read branch 1's prediction
(pipeline.window_twins). --no-dedup evaluates all four everywhere, as the reference does. The sampler's
steps are shape-identical, so frames/sec = N_frames / (25 * seconds_per_step). Weak scaling: each GPU
adds 14 output frames (N = 14 * world), units = (window, CFG branch) sharded contiguously, one RCCL
all-gather of noise predictions per step.

Synthetic data: seed 72589, latents/tokens ~N(0,1), pose ~N(0,0.1), masks per
mode, added_time_ids [12.5, 12, 20], guidance 2.0/7.5/3.0, shift 7, overlap 0; random-init weights of
the full SVD-XT + ACTalker v10 architecture (1.775 B params, no checkpoints offline).

Also reported: the dominant kernel's roofline (HIP events around its launches in a separate instrumented
pass after the timed loop, so the headline carries no measurement overhead), the reference's shipped
precision (fp16) and window (fpb 25) beside the headline, and the CPU baseline (the oracle restatement, fp32, on this host's cores, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0          # MI355X dense bf16 MFMA (MI355X_MICROARCH.md: ~2.5 PF dense; fp16 is the same)
PEAK_HBM_GBS = 8000.0              # MI355X HBM3E spec (MI355X_MICROARCH.md; ~6.3 TB/s achievable)
# algorithmic TFLOP per UNet frame-forward: (height, width, mode 2?)
TFLOP_PER_FRAME_FWD = {(576, 1024, True): 3.433, (576, 1024, False): 3.402, (576, 576, False): 1.779}
MODES = {0: ([1, 0], "mode=0 audio-only"), 1: ([0, 1], "mode=1 expression-only"), 2: ([1, 1], "mode=2 audio+expression")}


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def build_unet(device, seed=72589):
    from actalker_amd.synthetic import init_synthetic_
    from actalker_amd.unet_spatio_temporal_condition_mambaID_v10_two_ip import (UNetSpatioTemporalConditionModel,
                                                                               add_ip_adapters)
    with torch.device("meta"):
        unet = UNetSpatioTemporalConditionModel(num_frames=25)
    unet = unet.to_empty(device="cpu")
    add_ip_adapters(unet, [32, 32], [1.25, 1.25])
    init_synthetic_(unet, seed)
    return unet


def synthetic_inputs(N, fpb, H, W, mode, seed=72589):
    """Pipeline-internal tensors after CFG stacking (pipeline:128-184, 522-598, 636-638)."""
    g = torch.Generator().manual_seed(seed)
    T = N + fpb
    h, w = H // 8, W // 8
    ref_lat = torch.randn(1, 4, h, w, generator=g)
    noise = torch.randn(1, T, 4, h, w, generator=g)
    img_lat = torch.randn(1, 4, h, w, generator=g)
    id_tok = torch.randn(1, 1, 1024, generator=g)
    audio = torch.randn(N, 32, 1024, generator=g)
    uncond_audio = torch.randn(32, 1024, generator=g)
    vasa = torch.randn(N, 1024, generator=g) if mode != 0 else torch.zeros(N, 1024)
    uncond_vasa = torch.randn(1024, generator=g) if mode != 0 else torch.zeros(1024)
    pose = 0.1 * torch.randn(1, T, 320, h, w, generator=g)
    # CFG stacks: ID [0, id, id, id]; audio [u, u, a, a]; vasa [u, u, u, v]; +fpb uncond pad frames
    ide = torch.cat([torch.zeros(1, T, 1, 1024)] + [id_tok[:, None].expand(1, T, 1, 1024)] * 3)
    a_c = torch.cat([audio, uncond_audio[None].expand(fpb, 32, 1024)])[None]
    a_u = uncond_audio[None, None].expand(1, T, 32, 1024)
    aud = torch.cat([a_u, a_u, a_c, a_c])
    v_c = torch.cat([vasa, uncond_vasa[None].expand(fpb, 1024)])[None, :, None]
    v_u = uncond_vasa[None, None, None].expand(1, T, 1, 1024)
    vas = torch.cat([v_u, v_u, v_u, v_c])
    imgl = torch.cat([torch.zeros(1, T, 4, h, w)] + [img_lat[:, None].expand(1, T, 4, h, w)] * 3)
    sigma0 = 700.0
    latents = 0.18215 * ref_lat[:, None] + sigma0 * noise                 # scheduler.add_noise at t0
    added = torch.tensor([[12.5, 12.0, 20.0]] * 4)
    ones = torch.ones(1, 1, H, W)
    # (face, mouth, exp): without face models preprocessing falls back to a full-image face mask, and
    # Inference.py:545-546 overwrites the mouth / expression masks with ones
    masks = (ones, ones, ones)
    return dict(latents=latents, image_latents=imgl.contiguous(), image_embeddings=ide.contiguous(),
                audio_prompts=aud.contiguous(), vasa_prompts=vas.contiguous(), pose_fea=pose, added=added,
                masks=masks)


def gemm_algorithmic_bytes(a, w, M, N, K, kw):
    """HBM bytes one acth_gemm launch must move at minimum: each A source element once (an
    implicit-conv image once, not 9x), the weights, the output, and residual / mix rows."""
    esz = 2
    if kw.get("conv") is not None:
        c = kw["conv"]
        a_elems = c["B"] * c["H"] * c["W"] * (a.shape[1] + (kw["a2"].shape[1] if kw.get("a2") is not None else 0))
    elif kw.get("temporal") is not None:
        a_elems = M * (a.shape[1] + (kw["a2"].shape[1] if kw.get("a2") is not None else 0))
    else:
        a_elems = M * K
    n_out = N // 2 if kw.get("act", 0) == 2 else N
    out_b = 4 if kw.get("out_f32") else 2
    extra = (M * N * esz if kw.get("residual") is not None else 0) + (M * N * esz if kw.get("mix") is not None else 0)
    return a_elems * esz + N * K * esz + M * n_out * out_b + extra


PMC_WORKLOAD = None     # this run's workload key (set in main); PMC bytes are reported for that workload only


def workload_key(mode, height, width, frames, fpb, dtype, world=1):
    return f"mode{mode} {height}x{width} f{frames} fpb{fpb} {dtype}" + (f" world{world}" if world > 1 else "")


def pmc_traffic(family="acth_gemm"):
    """Per-kernel-family HBM bytes measured by rocprofv3 PMC passes of this command over one sampler
    step (tools/pmc_pass.sh -> tools/pmc_summary.py --json -> profiles/pmc_traffic.json), or None:
    {hbm_bytes_per_launch (per kernel dispatch), dispatches, read_bytes, write_bytes, source}. None as well
    when the counted run's workload (the file's "_workload") is not this run's."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None
    if d.get("_workload") is None or d.get("_workload") != PMC_WORKLOAD:
        return None
    from actalker_amd._lib import kernel_source_digest
    if d.get("_kernel_sources") != kernel_source_digest():     # counted on other kernels than the ones timed here
        return None
    return d.get(family)


class GemmTimer:
    """HIP events around every GEMM launch on the launch stream (torch's current stream)."""

    def __init__(self):
        self.events = []
        self.work = []                 # (flop, algorithmic bytes) per launch, parallel to events
        self.flops = 0.0
        self.bytes = 0.0
        self.launches = 0

    def install(self):
        from actalker_amd import ops
        orig = ops.gemm
        self.orig = orig

        def timed(a, w, **kw):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            out = orig(a, w, **kw)
            e1.record()
            N, K = w.shape
            M = out.shape[0] if kw.get("orow") is None else (kw.get("M") or a.shape[0])
            if kw.get("conv") is not None:
                c = kw["conv"]
                M = c["B"] * c["Ho"] * c["Wo"]
            elif kw.get("M") is not None:
                M = kw["M"]
            else:
                M = a.shape[0]
            fl, by = 2.0 * M * N * K, gemm_algorithmic_bytes(a, w, M, N, K, kw)
            self.flops += fl
            self.bytes += by
            self.launches += 1
            mode = "conv" if kw.get("conv") is not None else "temporal" if kw.get("temporal") is not None else "dense"
            self.events.append((e0, e1, (mode, M, N, K, kw.get("act", 0))))
            self.work.append((fl, by))
            return out
        ops.gemm = timed
        import actalker_amd.modules as mods
        mods.ops = ops
        return self

    def uninstall(self):
        from actalker_amd import ops
        ops.gemm = self.orig

    def total_ms(self):
        return sum(a.elapsed_time(b) for a, b, _ in self.events)

    def roofline_time(self):
        """Per-launch roofline: each launch's floor is max(FLOP / MFMA peak, algorithmic bytes / HBM peak);
        returns (sum of floors / sum of measured times, share of measured time in launches whose floor is
        the HBM one). The small-K level-0 GEMMs (K = 320: 2 FLOP per byte of A read and C written) are
        HBM-bound, which the family's single MFMA fraction does not show."""
        t_floor = t_meas = t_hbm = 0.0
        for (a, b, _), (fl, by) in zip(self.events, self.work):
            ms = a.elapsed_time(b)
            f_mfma, f_hbm = fl / (PEAK_BF16_TFLOPS * 1e9), by / (PEAK_HBM_GBS * 1e6)
            t_floor += max(f_mfma, f_hbm)
            t_meas += ms
            if f_hbm > f_mfma:
                t_hbm += ms
        return (t_floor / t_meas if t_meas else None), (t_hbm / t_meas if t_meas else None)

    def conv_family(self, step_ms_total):
        """The implicit-GEMM 3x3 convolutions (acth_gemm with A mode 1) as their own family: achieved MFMA rate,
        share of the step, algorithmic bytes (each image element once) and their PMC traffic."""
        evs = [(a, b, w) for (a, b, key), w in zip(self.events, self.work) if key[0] == "conv"]
        if not evs:
            return None
        ms = sum(a.elapsed_time(b) for a, b, _ in evs)
        fl = sum(w[0] for _, _, w in evs)
        by = sum(w[1] for _, _, w in evs)
        ach = fl / (ms / 1e3) / 1e12
        out = dict(bound="mfma", achieved=round(ach, 1), peak=PEAK_BF16_TFLOPS, unit="TFLOP/s",
                   frac=round(ach / PEAK_BF16_TFLOPS, 4), launches=len(evs), avg_launch_us=round(1000.0 * ms / len(evs), 1),
                   share_of_step=round(ms / step_ms_total, 4), algorithmic_bytes_per_launch=round(by / len(evs)),
                   flop_per_launch=round(fl / len(evs)))
        pmc = pmc_traffic("gemm_conv")
        if pmc:
            out["traffic"] = round(pmc["hbm_bytes_per_launch"])
            out["traffic_unit"] = "HBM bytes per kernel dispatch (PMC 2*FETCH_SIZE + WRITE_SIZE)"
            out["traffic_source"] = pmc.get("source")
        return out

    def shape_report(self, top=25):
        agg = {}
        for a, b, key in self.events:
            ms = a.elapsed_time(b)
            n, t = agg.get(key, (0, 0.0))
            agg[key] = (n + 1, t + ms)
        tot = sum(t for _, t in agg.values())
        lines = []
        for key, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
            mode, M, N, K, act = key
            tf = 2.0 * M * N * K * n / (t / 1000.0) / 1e12
            lines.append(f"{mode:8s} M={M:7d} N={N:5d} K={K:5d} act={act} n={n:4d} ms={t:8.1f} "
                         f"({100 * t / tot:4.1f}%) {tf:7.1f} TF/s")
        return "\n".join(lines)


class FamilyTimer:
    """HIP events around every launch of the non-GEMM kernel families on the launch stream inside the
    timed region, with each launch's algorithmic work: flash attention FLOPs (4 S^2 64 per head and
    batch), fused level-0 feed-forward FLOPs (24 M C^2), selective-scan bytes (u read once for both directions, the xdbl rows (bf16, or fp32 on the legacy path), both outputs
    written), GroupNorm / LayerNorm bytes (input read once, output written once -- the stats pass's
    second read of the input is the kernels' cost, not the algorithm's), Mamba combine + LayerNorm bytes
    (the rows each branch reads -- in_proj row or both scan directions -- and the output row)."""

    def __init__(self):
        self.ev = {}                         # family -> list of (e0, e1, work)
        self.extra = {}                      # family -> summed secondary work (selective_scan: state updates)

    def _wrap(self, mod, name, fam, work_fn):
        orig = getattr(mod, name)

        def timed(*a, **k):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            out = orig(*a, **k)
            e1.record()
            w = work_fn(*a, **k)
            if callable(w):                   # evaluated after the timed region (needs a device read)
                self.ev.setdefault(fam, []).append((e0, e1, w))
                return out
            if isinstance(w, tuple):          # (work, secondary count): the scan's state updates
                w, extra = w
                self.extra[fam] = self.extra.get(fam, 0) + extra
            self.ev.setdefault(fam, []).append((e0, e1, w))
            return out
        setattr(mod, name, timed)
        self._restore.append((mod, name, orig))

    def install(self):
        from actalker_amd import ops
        import actalker_amd.modules as mods
        self._restore = []

        def w_flash(qkv, nbatch, S, heads, out=None):
            return 4.0 * nbatch * heads * S * S * 64

        def w_scan(u, xdbl, *a, nb, L, R, n_keep, **k):
            D = u.shape[1]
            byts = nb * L * D * 2 + nb * L * xdbl.shape[1] * xdbl.element_size() + 2 * nb * n_keep * D * 2
            # state updates h = exp(dt A) h + dt u B: 16 states per channel, forward direction up to the last
            # kept token, reverse direction over all L tokens
            return byts, nb * D * 16 * (n_keep + L)

        def w_scan2(a, b):
            ra, rb = w_scan(**a), w_scan(**b)
            return ra[0] + rb[0], ra[1] + rb[1]

        def w_gn(x, *a, x2=None, residual=None, **k):
            C = x.shape[1] + (x2.shape[1] if x2 is not None else 0)
            return 2.0 * x.shape[0] * C * 2 + (x.shape[0] * C * 2 if residual is not None else 0)

        def w_ln(x, *a, add=None, sum_out=None, **k):
            return 2.0 * x.numel() * 2 + (x.numel() * 2 if sum_out is not None else 0)

        def w_ffn(x, *a, **k):
            M, C = x.shape
            return 24.0 * M * C * C                  # up 2*M*C*8C + down 2*M*4C*C

        def w_combine(branch_a, branch_e, gamma, beta, eps, M, S, C, out=None):
            # the rows each branch actually reads (its in_proj row x, or the two scan directions of a selected
            # token) plus the output row; mode-2 selections are counted after the timed region
            def rows_read(br):
                mode = br["mode"]
                if mode == 0:
                    return lambda: float(M)
                if mode == 1:
                    return lambda: 2.0 * M
                pos = br["pos"]
                return lambda: 2.0 * (M // S) * int((pos >= 0).sum()) + (M - (M // S) * int((pos >= 0).sum()))
            ra, re_ = rows_read(branch_a), rows_read(branch_e)
            return lambda: (ra() + re_() + M) * C * 2.0

        self._wrap(ops, "flash_attn", "flash_attn", w_flash)
        self._wrap(ops, "mamba_combine_ln", "mamba_combine", w_combine)
        self._wrap(ops, "geglu_ffn", "geglu_ffn", w_ffn)
        self._wrap(ops, "selective_scan", "selective_scan", w_scan)
        self._wrap(ops, "selective_scan2", "selective_scan", w_scan2)      # paired audio + expression launch
        self._wrap(ops, "groupnorm", "groupnorm", w_gn)
        self._wrap(ops, "layernorm", "layernorm", w_ln)
        mods.ops = ops
        return self

    def uninstall(self):
        for mod, name, orig in self._restore:
            setattr(mod, name, orig)

    def report(self, step_ms_total):
        peak = {"flash_attn": ("mfma", PEAK_BF16_TFLOPS, "TFLOP/s", 1e12),
                "geglu_ffn": ("mfma", PEAK_BF16_TFLOPS, "TFLOP/s", 1e12),
                "selective_scan": ("hbm", PEAK_HBM_GBS, "GB/s", 1e9),
                "groupnorm": ("hbm", PEAK_HBM_GBS, "GB/s", 1e9),
                "layernorm": ("hbm", PEAK_HBM_GBS, "GB/s", 1e9),
                "mamba_combine": ("hbm", PEAK_HBM_GBS, "GB/s", 1e9)}
        out = {}
        for fam, evs in self.ev.items():
            ms = sum(a.elapsed_time(b) for a, b, _ in evs)
            work = sum(w() if callable(w) else w for _, _, w in evs)
            bound, pk, unit, scale = peak[fam]
            ach = work / (ms / 1e3) / scale
            out[fam] = dict(bound=bound, achieved=round(ach, 1), peak=pk, unit=unit, frac=round(ach / pk, 4),
                            launches=len(evs), avg_launch_us=round(1000.0 * ms / len(evs), 1),
                            share_of_step=round(ms / step_ms_total, 4),
                            algorithmic_bytes_or_flop_per_launch=round(work / len(evs)))
            if fam == "selective_scan" and fam in self.extra:
                # the scan is VALU-issue bound, not HBM bound (PMC: ~5 cycles per VALU instruction, ~4.8 VALU
                # instructions per state update): its compute floor is one v_exp per state update at the v_exp
                # issue rate measured on gfx950 (tools/probes/valu_probe.hip: 4096 waves x 16384 v_exp in 0.239 ms)
                upd = self.extra[fam] / len(evs)
                floor_us = upd / V_EXP_PER_S * 1e6
                out[fam]["exp_floor"] = dict(
                    state_updates_per_launch=round(upd), v_exp_per_s=V_EXP_PER_S, floor_us=round(floor_us, 1),
                    frac=round(floor_us / (1000.0 * ms / len(evs)), 4),
                    source="profiles/r3_step18_valu_probe.txt (v_exp_f32, 4 waves / SIMD)")
                # the kernel's whole VALU issue, not only its exponentials: per token a lane updates 8 states with
                # 8 v_exp_f32, 8 v_pk_mul_f32, 8 v_pk_fma_f32 and ~12 single-rate VALU (u / y conversion, pair
                # reduction, D skip; the ISA of scan_pair_kernel<20,128,1,1>), priced at the probe's chip-wide
                # throughput per wave-instruction at 4 waves / SIMD
                per_512 = 8 * VALU_S["v_exp_f32"] + 8 * VALU_S["v_pk_mul_f32"] + 8 * VALU_S["v_pk_fma_f32"] + \
                    12 * VALU_S["v_fma_f32"]
                vfloor_us = upd / 512.0 * per_512 * 1e6
                out[fam]["valu_floor"] = dict(
                    floor_us=round(vfloor_us, 1), frac=round(vfloor_us / (1000.0 * ms / len(evs)), 4),
                    instructions_per_lane_token="8 v_exp + 8 v_pk_mul + 8 v_pk_fma + 12 VALU (8 states)",
                    source="profiles/r3_step18_valu_probe.txt (chip-wide time per wave-instruction, 4 waves / SIMD)")
            pmc = pmc_traffic(fam)
            if pmc:
                # PMC bytes per kernel dispatch x dispatches per op call (GroupNorm: stats + apply)
                per_call = 2 if fam == "groupnorm" else 1
                out[fam]["traffic"] = round(pmc["hbm_bytes_per_launch"] * per_call)
                out[fam]["traffic_unit"] = "HBM bytes per op call (PMC 2*FETCH_SIZE + WRITE_SIZE)"
                out[fam]["traffic_source"] = pmc.get("source")
        return out


V_EXP_PER_S = 4096 * 16384 * 64 / 0.239e-3      # gfx950 v_exp_f32 issue rate, all 1024 SIMDs (valu_probe)
# chip-wide seconds per wave-instruction at 4 waves / SIMD (valu_probe: 4096 waves x 16384 instructions)
VALU_S = {k: ms * 1e-3 / (4096 * 16384) for k, ms in
          (("v_exp_f32", 0.239), ("v_pk_mul_f32", 0.150), ("v_pk_fma_f32", 0.167), ("v_fma_f32", 0.089))}


def cpu_baseline(unet, H, W, frames=2, mode=0):
    """Oracle (fp32 CPU restatement) on a bounded sample: one UNet call, 1 CFG branch x `frames`
    frames at full resolution; frames/s extrapolated to the N=14 workload (200 frame-forwards
    per output frame = 4 CFG x 25 steps x 28/14). The HIP UNet runs the same call on the same
    weights and inputs, and the two outputs are compared (the bench line's ``parity``)."""
    from oracle import reference_cpu as ref
    sd = {k: v.detach().float().cpu() for k, v in unet.state_dict().items()}
    g = torch.Generator().manual_seed(1)
    h, w = H // 8, W // 8
    sample = torch.randn(1, frames, 8, h, w, generator=g)
    aud = torch.randn(frames, 32, 1024, generator=g) * float(mode != 1)       # gate (pipeline:724)
    vas = torch.randn(frames, 1, 1024, generator=g) * float(mode != 0)
    ehs = (torch.randn(frames, 1, 1024, generator=g), [aud, vas])
    pose = 0.1 * torch.randn(1, frames, 320, h, w, generator=g)
    one, zero = torch.ones(1, 1, H, W), torch.zeros(1, 1, H, W)
    masks = {0: [one, zero], 1: [zero, one], 2: [one, one]}[mode]             # pipeline:702-711
    t = torch.tensor(1.6)
    added = torch.tensor([[12.5, 12.0, 20.0]])
    t0 = time.perf_counter()
    with torch.no_grad():
        want = ref.unet_forward(sd, sample, t, ehs, added, pose, {"ip_adapter_masks": masks})
    dt = time.perf_counter() - t0
    dev = unet.device
    with torch.no_grad():
        got = unet(sample.to(dev), t.to(dev), (ehs[0].to(dev), [e.to(dev) for e in ehs[1]]), added.to(dev),
                   spatial_condition=pose.to(dev), cross_attention_kwargs={"ip_adapter_masks": masks},
                   return_dict=False)[0].float().cpu()
    d = got - want
    parity = dict(rel_l2=round((d.norm() / want.norm()).item(), 6), max_abs=round(d.abs().max().item(), 5),
                  ref_rms=round(want.pow(2).mean().sqrt().item(), 5), tol_rel_l2=2e-2,
                  sample=f"HIP {'fp16' if unet.compute_dtype() == torch.float16 else 'bf16'} vs oracle fp32, one UNet call (1 CFG branch x {frames} frames, {H}x{W}, "
                         f"mode {mode} masks / gated prompts), same weights and inputs")
    per_frame_fwd = dt / frames
    fps = 1.0 / (per_frame_fwd * 200.0)
    base = dict(value=fps, unit="frames/s", cores=torch.get_num_threads(), kind="port",
                sample=f"oracle fp32 UNet call, 1 CFG branch x {frames} frames at {H}x{W} ({dt:.1f} s = "
                       f"{per_frame_fwd:.2f} s/frame-forward), extrapolated x200 frame-forwards per output frame")
    return base, parity


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=25, help="timed sampler steps (25 = one full denoise)")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--mode", type=int, default=0, choices=[0, 1, 2])
    ap.add_argument("--frames-per-gpu", type=int, default=14)
    ap.add_argument("--height", type=int, default=576)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=2)
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-share-prefix", action="store_true",
                    help="run the UNet prefix before the first IP-adapter input for every CFG branch (no sharing "
                         "between the branches whose prefix inputs are equal)")
    ap.add_argument("--no-batch-ctx-proj", action="store_true",
                    help="per-module time_emb_proj / to_v(ID) GEMMs instead of the three batched ones per UNet call")
    ap.add_argument("--no-pair-scan", action="store_true",
                    help="one scan launch per Mamba branch instead of one launch for both branches")
    ap.add_argument("--no-dedup", action="store_true",
                    help="evaluate all 4 CFG branches even when two receive identical inputs (modes 0 / 1)")
    ap.add_argument("--no-four-branch-compare", action="store_true",
                    help="skip the extra timed run with all 4 CFG branches evaluated (reported beside the headline)")
    ap.add_argument("--no-other-modes", action="store_true",
                    help="skip the extra timed runs of the other BASELINE modes (C3 mode 1 / C4 mode 2 at N=1; "
                         "reported beside the headline as other_modes)")
    ap.add_argument("--units-per-call", type=int, default=0,
                    help="(window, branch) units per UNet call; 0 = auto (fewest calls within the kernels' "
                         "2 GiB buffer extents; the reference's call is 4 units = 56 frames)")
    ap.add_argument("--concurrent-calls", type=int, default=1,
                    help="run a rank's independent UNet calls of a step on this many HIP streams")
    ap.add_argument("--fpb", type=int, default=14,
                    help="frames per window (frames_per_batch); the reference ships n_sample_frames = 25 "
                         "(config/inference.yaml:4 -> Inference.py:573), the BASELINE metric is quoted at 14")
    ap.add_argument("--no-fpb25", action="store_true",
                    help="skip the extra timed run at the reference's shipped window (fpb 25, N = 25; reported "
                         "beside the headline as shipped_window)")
    ap.add_argument("--no-fp16-compare", action="store_true",
                    help="skip the extra timed run with fp16 activations (the reference's shipped weight_dtype, "
                         "config/inference.yaml:66; reported beside the bf16 headline as fp16)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16"],
                    help="activation dtype of the UNet kernels (fp16: libactalker_hip_f16.so, the reference's "
                         "shipped weight_dtype)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    # one rank per GPU; ACTH_DIST_BACKEND=gloo (with ranks sharing a device: LOCAL_RANK modulo the visible GPUs)
    # rehearses the multi-rank bench on a one-GPU box -- RCCL refuses two ranks on one device
    # (profiles/r5_rccl_same_gpu_probe.log) -- and its timings then mean nothing
    backend_name = os.environ.get("ACTH_DIST_BACKEND", "nccl")
    dev_idx = local_rank % max(1, torch.cuda.device_count()) if backend_name != "nccl" else local_rank
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    group = None
    if world > 1:
        import torch.distributed as dist
        if backend_name == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend_name)

    from actalker_amd import pipeline as pl

    gate, mode_name = MODES[args.mode]
    N = args.frames_per_gpu * world
    fpb = args.fpb
    H, W = args.height, args.width
    global PMC_WORKLOAD
    PMC_WORKLOAD = workload_key(args.mode, H, W, args.frames_per_gpu, fpb, args.dtype, world)
    if os.environ.get("ACTH_WORKLOAD_OUT") and rank == 0:     # tools/pmc_pass.sh: the key its counted run records
        with open(os.environ["ACTH_WORKLOAD_OUT"], "w") as fh:
            fh.write(PMC_WORKLOAD)
    t0 = time.time()
    unet_cpu = build_unet(dev)
    unet = unet_cpu.to(dev)
    unet.acth_batch_ctx_projections = not args.no_batch_ctx_proj
    unet.acth_compute_dtype = torch.float16 if args.dtype == "fp16" else torch.bfloat16
    if args.no_pair_scan:
        from actalker_amd import modules as _m
        for mod in unet.modules():
            if isinstance(mod, _m.SS2D_cond_v10):
                mod.acth_pair_scan = False
    log(f"model built in {time.time() - t0:.1f}s")
    inp = synthetic_inputs(N, fpb, H, W, args.mode)
    backend = pl.HipBackend(unet, H // 8, W // 8, inp["masks"], gate, inp["added"], N + fpb, fpb,
                            inp["image_latents"], inp["image_embeddings"], inp["audio_prompts"],
                            inp["vasa_prompts"], inp["pose_fea"])
    cfg = pl.LoopConfig(num_frames=N, frames_per_batch=fpb, overlap=0, shift_offset=7,
                        concurrent_calls=args.concurrent_calls, dedup_branches=not args.no_dedup,
                        units_per_call=args.units_per_call, share_cfg_prefix=not args.no_share_prefix)
    twins = backend.branch_twins() if cfg.dedup_branches else {}
    branches = [c for c in range(4) if c not in twins]
    log(f"CFG branches evaluated: {branches} (twins {twins})")

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize()

    def timed(be, latents, lc, steps, plan_log=None, warm=True):
        """One untimed warm step (``warm``), then ``steps`` timed sampler steps bracketed by barrier + synchronize."""
        if warm:
            with torch.no_grad():
                pl.denoise(be, latents, lc, rank, world, group, steps=1)
        barrier()
        t_s = time.perf_counter()
        with torch.no_grad():
            res = pl.denoise(be, latents, lc, rank, world, group, steps=steps, plan_log=plan_log)
        barrier()
        return time.perf_counter() - t_s, res

    # warmup (packs weights, builds mask tables, warms the allocator)
    with torch.no_grad():
        pl.denoise(backend, inp["latents"], cfg, rank, world, group, steps=args.warmup)
    # ACTH_TRACE_MARK=1: a spin kernel on each side of the timed loop, so a rocprofv3 kernel trace can be cut to
    # exactly the timed steps (tools/trace_gaps.py); off by default
    mark = os.environ.get("ACTH_TRACE_MARK") == "1"
    barrier()
    if mark:
        torch.cuda._sleep(1000)
    t_start = time.perf_counter()
    plan = []
    with torch.no_grad():
        out = pl.denoise(backend, inp["latents"], cfg, rank, world, group, steps=args.steps, plan_log=plan)
    if mark:
        torch.cuda._sleep(1000)
    barrier()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ok = bool(torch.isfinite(out).all())
    ms_per_step = 1000.0 * elapsed / args.steps
    fps = N / (cfg.num_inference_steps * elapsed / args.steps)

    # kernel roofline / family figures: a SEPARATE instrumented pass after the headline's timed loop (HIP events
    # around every GEMM and kernel-family launch), so the headline carries no measurement overhead. Two steps cover
    # both step kinds of the loop (with and without a padding-only window, shift 0 / 7).
    timer = ftimer = None
    inst_elapsed = None
    if not args.no_roofline:
        timer = GemmTimer().install()
        ftimer = FamilyTimer().install()
        inst_steps = min(2, args.steps)
        inst_elapsed, _ = timed(backend, inp["latents"], cfg, inst_steps, warm=False)
        timer.uninstall()
        ftimer.uninstall()

    roof = None
    if timer is not None and timer.launches:
        gemm_ms = timer.total_ms()
        if os.environ.get("ACTH_GEMM_STATS"):
            log(timer.shape_report(top=int(os.environ.get("ACTH_GEMM_STATS")) or 25))
        achieved = timer.flops / (gemm_ms / 1000.0) / 1e12
        pmc = pmc_traffic()
        roof = dict(bound="mfma", achieved=round(achieved, 2), peak=PEAK_BF16_TFLOPS, unit="TFLOP/s",
                    frac=round(achieved / PEAK_BF16_TFLOPS, 4),
                    traffic=(round(pmc["hbm_bytes_per_launch"]) if pmc else None),
                    traffic_unit="bytes/launch (PMC 2*FETCH_SIZE + WRITE_SIZE)",
                    traffic_source=(pmc or {}).get("source"),
                    algorithmic_bytes_per_launch=round(timer.bytes / timer.launches),
                    kernel="acth_gemm (gemm8p_kernel<320|256,A> + gemm256_kernel + gemm_bf16_kernel launches)",
                    launches=timer.launches, avg_launch_us=round(1000.0 * gemm_ms / timer.launches, 2),
                    flop_per_launch=round(timer.flops / timer.launches),
                    kernel_share_of_step=round(gemm_ms / (inst_elapsed * 1000.0), 3),
                    measured_in="separate instrumented pass of 2 sampler steps after the timed loop")
        rt, hbm_share = timer.roofline_time()
        if rt is not None:
            roof["per_launch_roofline"] = dict(
                time_frac=round(rt, 4), hbm_bound_time_share=round(hbm_share, 4),
                definition="sum over GEMM launches of max(FLOP / 2500 TFLOP/s, algorithmic bytes / 8000 GB/s) "
                           "divided by the sum of measured launch times")
    frame_fwds = sum(p["rank_units"] for p in plan) * fpb
    n_windows = len(range(0, N + fpb, fpb))
    units_per_step = sum(p["units"] for p in plan) / max(1, len(plan))
    # the reference-shaped figure: all four CFG branches evaluated (no twin-branch elimination), same steps
    four = None
    if cfg.dedup_branches and world == 1 and not args.no_four_branch_compare:
        cfg4 = pl.LoopConfig(num_frames=N, frames_per_batch=fpb, overlap=0, shift_offset=7,
                             concurrent_calls=args.concurrent_calls, dedup_branches=False,
                             units_per_call=args.units_per_call, share_cfg_prefix=False)
        with torch.no_grad():
            pl.denoise(backend, inp["latents"], cfg4, rank, world, group, steps=1)
        barrier()
        t4 = time.perf_counter()
        with torch.no_grad():
            pl.denoise(backend, inp["latents"], cfg4, rank, world, group, steps=args.steps)
        barrier()
        e4 = time.perf_counter() - t4
        four = dict(value=round(N / (cfg.num_inference_steps * e4 / args.steps), 4),
                    ms_per_step=round(1000.0 * e4 / args.steps, 2), cfg_branches_evaluated=4)
    # the other BASELINE single-GPU configs (C3 mode 1, C4 mode 2 = C5's per-rank workload), timed after the
    # headline on the same model: same loop settings, their own synthetic inputs / masks / gates
    other = None
    if world == 1 and not args.no_other_modes:
        other = {}
        for m in (0, 1, 2):
            if m == args.mode:
                continue
            gate_m, name_m = MODES[m]
            inp_m = synthetic_inputs(N, fpb, H, W, m)
            be_m = pl.HipBackend(unet, H // 8, W // 8, inp_m["masks"], gate_m, inp_m["added"], N + fpb, fpb,
                                 inp_m["image_latents"], inp_m["image_embeddings"], inp_m["audio_prompts"],
                                 inp_m["vasa_prompts"], inp_m["pose_fea"])
            tw_m = be_m.branch_twins() if cfg.dedup_branches else {}
            with torch.no_grad():
                pl.denoise(be_m, inp_m["latents"], cfg, rank, world, group, steps=1)
            barrier()
            tm = time.perf_counter()
            plan_m = []
            with torch.no_grad():
                out_m = pl.denoise(be_m, inp_m["latents"], cfg, rank, world, group, steps=args.steps, plan_log=plan_m)
            barrier()
            em = time.perf_counter() - tm
            other[f"mode{m}"] = dict(workload=name_m, value=round(N / (cfg.num_inference_steps * em / args.steps), 4),
                                     ms_per_step=round(1000.0 * em / args.steps, 2), steps=args.steps,
                                     cfg_branches_evaluated=4 - len(tw_m),
                                     units_per_step=round(sum(p["units"] for p in plan_m) / max(1, len(plan_m)), 2),
                                     finite=bool(torch.isfinite(out_m).all()))
            del be_m, inp_m, out_m
    # the reference's shipped precision beside the headline: fp16 activations (weight_dtype: fp16,
    # config/inference.yaml:66), same workload and loop
    fp16_cmp = None
    if world == 1 and args.dtype == "bf16" and not args.no_fp16_compare:
        prev_dtype = getattr(unet, "acth_compute_dtype", None)
        unet.acth_compute_dtype = torch.float16
        try:
            be16 = pl.HipBackend(unet, H // 8, W // 8, inp["masks"], gate, inp["added"], N + fpb, fpb,
                                 inp["image_latents"], inp["image_embeddings"], inp["audio_prompts"],
                                 inp["vasa_prompts"], inp["pose_fea"])
            e16, out16 = timed(be16, inp["latents"], cfg, args.steps)
        finally:
            unet.acth_compute_dtype = prev_dtype
        fp16_cmp = dict(dtype="fp16", value=round(N / (cfg.num_inference_steps * e16 / args.steps), 4),
                        ms_per_step=round(1000.0 * e16 / args.steps, 2), steps=args.steps,
                        finite=bool(torch.isfinite(out16).all()))
        del be16, out16
    # the reference's shipped window beside the headline: frames_per_batch = n_sample_frames = 25
    # (config/inference.yaml:4 -> Inference.py:573), N = 25 output frames (2 windows of 25 latent frames), shift 7
    shipped = None
    if world == 1 and fpb != 25 and not args.no_fpb25:
        n25 = 25
        inp25 = synthetic_inputs(n25, 25, H, W, args.mode)
        be25 = pl.HipBackend(unet, H // 8, W // 8, inp25["masks"], gate, inp25["added"], n25 + 25, 25,
                             inp25["image_latents"], inp25["image_embeddings"], inp25["audio_prompts"],
                             inp25["vasa_prompts"], inp25["pose_fea"])
        cfg25 = pl.LoopConfig(num_frames=n25, frames_per_batch=25, overlap=0, shift_offset=7,
                              concurrent_calls=args.concurrent_calls, dedup_branches=not args.no_dedup,
                              units_per_call=args.units_per_call, share_cfg_prefix=not args.no_share_prefix)
        plan25 = []
        e25, out25 = timed(be25, inp25["latents"], cfg25, args.steps, plan_log=plan25)
        shipped = dict(workload=f"{mode_name}, {H}x{W}, N = 25 frames, fpb 25 (the reference's shipped "
                                f"n_sample_frames), shift 7, 25-step EulerDiscrete, 4-way CFG",
                       value=round(n25 / (cfg25.num_inference_steps * e25 / args.steps), 4),
                       ms_per_step=round(1000.0 * e25 / args.steps, 2), steps=args.steps,
                       units_per_step=round(sum(p["units"] for p in plan25) / max(1, len(plan25)), 2),
                       finite=bool(torch.isfinite(out25).all()))
        del be25, inp25, out25
    cpu = parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, parity = cpu_baseline(unet, H, W, frames=args.cpu_frames, mode=args.mode)
    if rank == 0:
        line = {
            "metric": "denoised frames/sec, 576x1024x14f x25-step audio-driven, 1/2/4/8 MI355X",
            "value": round(fps, 4), "unit": "frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 2), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": args.dtype, "data": "synthetic",
            "config": {"workload": f"{mode_name}, {H}x{W}, {N} frames ({args.frames_per_gpu}/GPU), fpb {fpb}, "
                                   f"25-step EulerDiscrete, 4-way CFG ({len(branches)} distinct branch inputs evaluated"
                                   + (f", branch {sorted(twins)} = twin {[twins[k] for k in sorted(twins)]} under gate "
                                      f"{gate}" if twins else "")
                                   + f"; padding-only windows: branches 2, 3 = twin 1; {units_per_step:.2f} of "
                                     f"{4 * n_windows} (window x branch) units per step evaluated), units over "
                                     f"{world} GPU(s)",
                       "model": "SVD-XT UNet + ACTalker v10 dual-Mamba (1.775B, random init)",
                       "global_batch": N, "seq_len": fpb, "parallelism": f"units{world}"},
            "unet_frame_forwards_per_s_per_gpu": round(frame_fwds / elapsed, 3),
            "achieved_mfma_tflops_whole_step": (round(frame_fwds * TFLOP_PER_FRAME_FWD[(H, W, args.mode == 2)] / elapsed, 1)
                                                if (H, W, args.mode == 2) in TFLOP_PER_FRAME_FWD else None),
            "cfg_branches_evaluated": len(branches),
            "units_per_step": {"evaluated": round(units_per_step, 2), "reference": 4 * n_windows},
            "cfg_prefix_shared": cfg.share_cfg_prefix,
            "all_four_branches": four,
            "other_modes": other,
            "fp16": fp16_cmp,
            "shipped_window": shipped,
            "finite": ok,
            "roofline": roof,
            "cpu_baseline": cpu,
            "parity": parity,
            "kernel_families": ({**ftimer.report(inst_elapsed * 1000.0),
                                 **({"gemm_conv": timer.conv_family(inst_elapsed * 1000.0)} if timer is not None else {})}
                                if ftimer is not None else None),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
