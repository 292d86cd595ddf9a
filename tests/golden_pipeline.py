"""Cases of the REFERENCE-RUN sampler goldens: ``Pose2VideoLongSVDPipeline.__call__``
(src/pipelines/pipeline_svd_audio_adapter_motionexp_idembed_vasa_two_ip.py:351-773) run unchanged on the CPU by
tools/gen_golden_pipeline_ref.py with ``output_type="latent"``, around the reference UNet package at the tiny
full-topology config (tests/golden_unet_ref.py) and the reference scheduler mirror
(src/schedulers/scheduling_euler_discrete.py). So the CFG stacking and uncond padding (:128-205), the added time
ids (:207-233, :567-576), ``prepare_latents`` / ``add_noise`` (:278-317, :584-598), the mask and pose plumbing
(:600-638), the per-step guidance ``linspace`` (:640-657) and the step x window loop with ``indice_slice``
wrap, gate-dependent masks, guidance, Euler step and accumulate / average (:670-756) are all reference code.

The three models the loop only reads through (VAE encode, the ID projection, the pose guider) are deterministic
CPU/GPU stand-ins defined here with seeded weights; they are not the loop under test, and the product pipeline
(actalker_amd.pipeline_svd) is handed the same stand-ins. Each is a function of its input, so the noise
augmentation draw (:525-531) and the pose / mask images reach the loop.

Also here: ``oracle_loop_inputs`` -- the test-side restatement of :128-205 / :518-657 that turns the same raw
inputs into oracle.reference_cpu.denoise_loop's stacked tensors (checked against the reference run in
tests/test_oracle_cpu.py).
"""
import types

import torch
import torch.nn as nn
import torch.nn.functional as F

N, FPB = 4, 2
H_PX, W_PX = 128, 256
H, W = H_PX // 8, W_PX // 8
STEPS = 25
# per case: (gate, overlap, shift_offset); mode1 runs overlapping windows (accumulate / average, :748-756)
CASES = {"mode0": ([1, 0], 0, 1), "mode1": ([0, 1], 1, 1), "mode2": ([1, 1], 0, 1),
         # the reference's shipped window: frames_per_batch = n_sample_frames = 25 (config/inference.yaml:4,
         # Inference.py:573) with its shipped shift_offset 7 / overlap 0 (inference.yaml); latent 8x16
         "f25_mode0": ([1, 0], 0, 7), "f25_mode2": ([1, 1], 0, 7)}
# per case geometry (N, fpb, H_PX, W_PX); the f25 cases run 2 windows of 25 frames (T = N + fpb = 29)
GEOMETRY = {"f25_mode0": (4, 25, 64, 128), "f25_mode2": (4, 25, 64, 128)}
GUIDANCE = dict(min_guidance_scale1=1.0, max_guidance_scale1=3.0, min_guidance_scale2=2.0, max_guidance_scale2=7.5,
                min_guidance_scale3=1.5, max_guidance_scale3=3.0)
CALL = dict(height=H_PX, width=W_PX, num_frames=N, num_inference_steps=STEPS, fps=12.5, motion_bucket_id=12,
            motion_bucket_id_exp=20, noise_aug_strength=0.02, frames_per_batch=FPB, i2i_noise_strength=1.0,
            **GUIDANCE)
INPUT_SEED, GEN_SEED = 41, 7


def geometry(case=None):
    """(N, fpb, H_PX, W_PX) of ``case`` (the module defaults for the N = 4, fpb = 2 cases)."""
    return GEOMETRY.get(case, (N, FPB, H_PX, W_PX))


def call_kwargs(case=None):
    """The __call__ keyword arguments of ``case`` besides the inputs, generator, overlap, shift and gate."""
    n, fpb, hp, wp = geometry(case)
    return dict(CALL, height=hp, width=wp, num_frames=n, frames_per_batch=fpb)


class _StandIn(nn.Module):
    @property
    def dtype(self):
        return next(self.parameters()).dtype

    @property
    def device(self):
        return next(self.parameters()).device


class StandInVAE(_StandIn):
    """``encode(x).latent_dist.{mean, mode()}`` = a fixed 1x1 projection of the 8x8-average-pooled image
    (4 latent channels, the VAE's scale factor 8)."""

    def __init__(self, seed: int = 3):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.w = nn.Parameter(torch.randn(4, 3, generator=g), requires_grad=False)
        self.b = nn.Parameter(0.1 * torch.randn(4, generator=g), requires_grad=False)
        self.config = types.SimpleNamespace(block_out_channels=[128, 256, 512, 512], force_upcast=False,
                                            scaling_factor=0.18215)

    def encode(self, x):
        z = F.avg_pool2d(x.float(), 8)
        z = torch.einsum("oc,bchw->bohw", self.w, z) + self.b[:, None, None]
        return types.SimpleNamespace(latent_dist=types.SimpleNamespace(mean=z, mode=lambda: z))


class StandInIDProj(_StandIn):
    """(B, 3, h, w) image -> (B, 1, 1024): a fixed projection of its 4x4 average pool."""

    def __init__(self, seed: int = 4):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.w = nn.Parameter(torch.randn(48, 1024, generator=g) / 48 ** 0.5, requires_grad=False)

    def forward(self, x):
        return (F.adaptive_avg_pool2d(x.float(), 4).flatten(1) @ self.w)[:, None]


class StandInPoseGuider(_StandIn):
    """(1, 3, N, H, W) pose images -> (1, C, N, H/8, W/8): a fixed 1x1 projection of the 8x8 average pool."""

    def __init__(self, channels: int, seed: int = 6):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.w = nn.Parameter(0.1 * torch.randn(channels, 3, generator=g), requires_grad=False)

    def forward(self, x):
        z = F.avg_pool3d(x.float(), (1, 8, 8))
        return torch.einsum("oc,bcnhw->bonhw", self.w, z)


def raw_inputs(seed: int = INPUT_SEED, case=None):
    """The __call__ arguments the caller (Inference.py:547-577) hands the pipeline, synthetic and seeded:
    ref / clip images, N pose images (binary face boxes moving 8 px per frame: pose[0][0] is the face mask,
    :622), N expression (upper half) and mouth (lower half) mask images, N audio / uncond audio prompts
    (32, 1024), N VASA / uncond VASA prompts (1024,), and the initial noise ``latents`` (1, N + fpb, 4, h, w)."""
    N, FPB, H_PX, W_PX = geometry(case)
    H, W = H_PX // 8, W_PX // 8
    g = torch.Generator().manual_seed(seed)
    ref = torch.rand(1, 3, H_PX, W_PX, generator=g) * 2 - 1
    clip = torch.rand(1, 3, 224, 224, generator=g)
    pose = []
    for k in range(N):
        p = torch.zeros(3, H_PX, W_PX)
        p[:, H_PX // 4: 3 * H_PX // 4, W_PX // 4 + 8 * k: 3 * W_PX // 4 + 8 * k] = 1.0
        pose.append(p)
    upper = torch.zeros(3, H_PX, W_PX)
    upper[:, : H_PX // 2] = 1.0
    exp_masks = [upper.clone() for _ in range(N)]
    mouth_masks = [1.0 - upper for _ in range(N)]
    aud = [torch.randn(32, 1024, generator=g) for _ in range(N)]
    uaud = [torch.randn(32, 1024, generator=g) for _ in range(N)]
    vas = [torch.randn(1024, generator=g) for _ in range(N)]
    uvas = [torch.randn(1024, generator=g) for _ in range(N)]
    latents = torch.randn(1, N + FPB, 4, H, W, generator=g)
    return dict(ref_image=ref, clip_image=clip, pose_images=pose, exp_mask_images=exp_masks,
                mouth_mask_images=mouth_masks, audio_prompts=aud, uncond_audio_prompts=uaud, vasa_prompts=vas,
                uncond_vasa_prompts=uvas, latents=latents)


def inputs_checksum(raw):
    from tests import golden_full as gf
    return gf.checksum(raw["ref_image"], raw["clip_image"], *raw["pose_images"], *raw["exp_mask_images"],
                       *raw["mouth_mask_images"], *raw["audio_prompts"], *raw["uncond_audio_prompts"],
                       *raw["vasa_prompts"], *raw["uncond_vasa_prompts"], raw["latents"])


def standins(pose_channels: int):
    return StandInVAE(), StandInIDProj(), StandInPoseGuider(pose_channels)


def oracle_loop_inputs(raw, vae, id_proj, pose_guider, gate, case=None):
    """Restatement of pipeline:128-205 (CFG stacking, uncond pads), :518-598 (ref / image latents, add_noise at
    sigma_max with the generator's noise-augmentation draw first), :600-638 (masks, pose features) and :640-657
    (per-step guidance) -> the arguments of oracle.reference_cpu.denoise_loop."""
    from oracle.reference_cpu import euler_karras_tables
    N, FPB, _, _ = geometry(case)
    T = N + FPB
    ide = id_proj(raw["clip_image"]).unsqueeze(1).repeat(1, T, 1, 1)
    ide = torch.cat([torch.zeros_like(ide), ide, ide, ide])
    a = torch.stack(raw["audio_prompts"]).unsqueeze(0)
    ua = torch.stack(raw["uncond_audio_prompts"]).unsqueeze(0)
    v = torch.stack(raw["vasa_prompts"]).unsqueeze(0).unsqueeze(2)
    uv = torch.stack(raw["uncond_vasa_prompts"]).unsqueeze(0).unsqueeze(2)
    pa, pv = ua[:, :1].repeat(1, FPB, 1, 1), uv[:, :1].repeat(1, FPB, 1, 1)
    a, ua, v, uv = torch.cat([a, pa], 1), torch.cat([ua, pa], 1), torch.cat([v, pv], 1), torch.cat([uv, pv], 1)
    aud, vas = torch.cat([ua, ua, a, a]), torch.cat([uv, uv, uv, v])
    ref = raw["ref_image"]
    ref_lat = vae.encode(ref).latent_dist.mean * 0.18215
    aug = torch.randn(ref.shape, generator=torch.Generator().manual_seed(GEN_SEED))
    il = vae.encode(ref + CALL["noise_aug_strength"] * aug).latent_dist.mode()
    imgl = torch.cat([torch.zeros_like(il), il, il, il]).unsqueeze(1).repeat(1, T, 1, 1, 1)
    sigmas, _ = euler_karras_tables(STEPS)
    latents = ref_lat.unsqueeze(1) + raw["latents"] * sigmas[0]
    added = torch.tensor([[CALL["fps"], CALL["motion_bucket_id"], CALL["motion_bucket_id_exp"]]] * 4)
    pose_t = torch.stack(raw["pose_images"], 1)[None]                               # (1, 3, N, H, W)
    face = pose_t[0, :1, :1]
    exp = torch.stack(raw["exp_mask_images"], 1)[None][0, :1, :1]
    mouth = torch.stack(raw["mouth_mask_images"], 1)[None][0, :1, :1]
    pose_fea = pose_guider(pose_t).transpose(1, 2)
    gsched = list(zip(*[torch.linspace(CALL[f"min_guidance_scale{j}"], CALL[f"max_guidance_scale{j}"], STEPS).tolist()
                        for j in (1, 2, 3)]))
    return latents, imgl, ide, aud, vas, pose_fea, added, [face, mouth, exp], gsched


def oracle_pipeline_loop(case: str, dtype=None):
    """The oracle's version of the reference run of ``case``: tiny full-topology weights (the reference-run UNet
    goldens' seed), the restated stacking above and oracle.reference_cpu.denoise_loop. dtype (torch.bfloat16 /
    float16): every oracle op rounded at its boundary (oracle.precision) -- the rounding floor the HIP bf16 loop
    is held against."""
    import contextlib
    from oracle import reference_cpu as ref
    from tests import golden_unet_ref as gu
    unet = gu.build_hip_unet("tiny_mode0")
    sd = {k: v.detach().float() for k, v in unet.state_dict().items()}
    ctx = contextlib.nullcontext()
    if dtype is not None:
        from oracle import precision
        sd = precision.round_state_dict(sd, dtype)
        ctx = precision.rounded(dtype)
    gate, overlap, shift = CASES[case]
    N, FPB, _, _ = geometry(case)
    vae, idp, pg = standins(gu.TINY_CFG["block_out_channels"][0])
    with torch.no_grad():
        lat, imgl, ide, aud, vas, pose, added, masks, gs = oracle_loop_inputs(raw_inputs(case=case), vae, idp, pg,
                                                                              gate, case)

        def unet_fn(sample, t, ehs, added_ids, sc, cak):
            return ref.unet_forward(sd, sample, t, ehs, added_ids, sc, cak, ip_scale=(1.25, 1.25),
                                    cfg=gu.oracle_cfg("tiny_mode0"))

        with ctx:
            return ref.denoise_loop(unet_fn, lat, imgl, ide, aud, vas, pose, added, masks, gate, N, FPB,
                                    overlap=overlap, shift_offset=shift, guidance=gs, num_inference_steps=STEPS)
