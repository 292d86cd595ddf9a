"""End-to-end Pose2VideoLongSVDPipeline on the GPU (adapters -> VAE encode -> sharded loop -> VAE decode)
against the oracle composition of the same stages (oracle/reference_cpu.py: id_proj_model, pose_guider,
vae_encode_moments, denoise_loop, vae_decode), tiny widths, real topology. Exercises the reference's
own defaults that the bench path does not: overlapping windows (overlap > 0 -> counter averaging),
pose features indexed mod N while latents wrap mod N + fpb, per-step guidance schedules, and
decode_chunk_size chunking. Tolerance: relative L2 5e-2 on the decoded frames (bf16 vs fp32,
through 3 sampler steps, as tests/test_model_gpu.py's loop test)."""
import pytest
import torch

from actalker_amd.synthetic import synthetic_state_dict
from oracle import reference_cpu as ref

pytestmark = pytest.mark.gpu


def _init(m, seed):
    sd = synthetic_state_dict(seed, {k: tuple(v.shape) for k, v in m.state_dict().items()})
    m.load_state_dict(sd, strict=True)
    return sd


def test_pipeline_end_to_end_vs_oracle(dev):
    from __graft_entry__ import _tiny_unet
    from actalker_amd.adapters import IDProjModel, PoseGuider
    from actalker_amd.pipeline_svd import Pose2VideoLongSVDPipeline
    from actalker_amd.vae import AutoencoderKLTemporalDecoder

    unet, cfg = _tiny_unet()
    sd_unet = {k: v.detach().clone() for k, v in unet.state_dict().items()}
    vae = AutoencoderKLTemporalDecoder(block_out_channels=(64, 64, 128, 128))
    sd_vae = _init(vae, 51)
    idp = IDProjModel(512, 1024, 1024)
    sd_id = _init(idp, 52)
    pg = PoseGuider(64, block_out_channels=(16, 32, 96, 256))
    sd_pg = _init(pg, 53)

    N, fpb, H, W, steps = 4, 2, 128, 256, 3
    g = torch.Generator().manual_seed(9)
    ref_img = torch.rand(1, 3, H, W, generator=g) * 2 - 1
    clip = torch.randn(1, 1, 512, generator=g)
    poses = [torch.rand(3, H, W, generator=g) for _ in range(N)]
    lower = torch.zeros(1, H, W)
    lower[:, H // 2:] = 1.0
    exp_masks = [1 - lower for _ in range(N)]
    mouth_masks = [lower for _ in range(N)]
    aud = [torch.randn(32, 1024, generator=g) for _ in range(N)]
    uaud = [torch.randn(32, 1024, generator=g) for _ in range(N)]
    vas = [torch.randn(1024, generator=g) for _ in range(N)]
    uvas = [torch.randn(1024, generator=g) for _ in range(N)]
    T = N + fpb
    aug = torch.randn(1, 3, H, W, generator=torch.Generator().manual_seed(77))
    noise = torch.randn(1, T, 4, H // 8, W // 8, generator=torch.Generator().manual_seed(78))
    kw = dict(height=H, width=W, num_frames=N, num_inference_steps=steps, min_guidance_scale1=2.0,
              max_guidance_scale1=2.0, min_guidance_scale2=7.5, max_guidance_scale2=7.5, min_guidance_scale3=3.0,
              max_guidance_scale3=3.0, fps=12.5, motion_bucket_id=12, motion_bucket_id_exp=20,
              noise_aug_strength=0.02, decode_chunk_size=4, overlap=1, shift_offset=1, frames_per_batch=fpb,
              gate=[1, 1])

    pipe = Pose2VideoLongSVDPipeline(vae, unet, idp, pg).to(dev)
    gen = torch.Generator().manual_seed(77)             # first draw = the augmentation noise
    got = pipe(ref_img, clip, poses, exp_masks, mouth_masks, aud, uaud, vas, uvas, generator=gen, latents=noise,
               **kw).frames
    torch.cuda.synchronize()
    assert got.shape == (1, 3, N, H, W)

    # ---- oracle composition, same stages and order
    ide = ref.id_proj_model(sd_id, "", clip).unsqueeze(1).repeat(1, T, 1, 1)
    ide = torch.cat([torch.zeros_like(ide), ide, ide, ide])
    st = lambda xs: torch.stack(xs, 0)[None]                                     # noqa: E731
    a, ua = st(aud), st(uaud)
    v, uv = st(vas)[:, :, None], st(uvas)[:, :, None]
    pa, pv = ua[:, :1].repeat(1, fpb, 1, 1), uv[:, :1].repeat(1, fpb, 1, 1)
    a, ua, v, uv = torch.cat([a, pa], 1), torch.cat([ua, pa], 1), torch.cat([v, pv], 1), torch.cat([uv, pv], 1)
    audio_cfg, vasa_cfg = torch.cat([ua, ua, a, a]), torch.cat([uv, uv, uv, v])
    ref_lat = ref.vae_encode_moments(sd_vae, ref_img)[:, :4] * 0.18215
    img_lat = ref.vae_encode_moments(sd_vae, ref_img + 0.02 * aug)[:, :4]
    img_lat = torch.cat([torch.zeros_like(img_lat), img_lat, img_lat, img_lat]).unsqueeze(1).repeat(1, T, 1, 1, 1)
    sig, _ = ref.euler_karras_tables(steps)
    lat0 = ref_lat.unsqueeze(1) + noise * sig[0]
    pose = torch.stack(poses, 1)[None]
    pose_fea = ref.pose_guider(sd_pg, "", pose).transpose(1, 2)
    masks = (pose[0, :1, :1], lower[None], (1 - lower)[None])
    added = torch.tensor([[12.5, 12.0, 20.0]] * 4)

    def unet_fn(sample, t, ehs, added_ids, sc, cak):
        return ref.unet_forward(sd_unet, sample, t, ehs, added_ids, sc, cak, ip_scale=(1.25, 1.25),
                                cfg=dict(block_out_channels=cfg["block_out_channels"],
                                         num_attention_heads=cfg["num_attention_heads"]))

    lat = ref.denoise_loop(unet_fn, lat0, img_lat, ide, audio_cfg, vasa_cfg, pose_fea, added, masks, [1, 1], N, fpb,
                           1, 1, (2.0, 7.5, 3.0), num_inference_steps=steps)
    z = lat.flatten(0, 1) / 0.18215
    want = torch.cat([ref.vae_decode(sd_vae, z[i:i + 4], z[i:i + 4].shape[0]) for i in range(0, T, 4)])
    want = want.reshape(1, T, *want.shape[1:]).permute(0, 2, 1, 3, 4)[:, :, :N]
    err = ((got.cpu() - want).norm() / want.norm()).item()
    assert err < 5e-2, f"end-to-end rel-L2 {err:.3e}"
