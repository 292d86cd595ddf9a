"""End-to-end ACTalker generation on MI355X: the reference pipeline's ``__call__`` with every stage
on the HIP kernels (conditioning adapters -> VAE ref encode -> sharded denoising loop -> VAE decode).

Mirrors ``Pose2VideoLongSVDPipeline`` (src/pipelines/pipeline_svd_audio_adapter_motionexp_idembed_vasa_two_ip.py:
constructor :80-127, ``_clip_encode_image`` :128-184, ``_encode_vae_image`` :186-205, ``_get_add_time_ids``
:207-233, ``decode_latents`` :235-262, ``prepare_latents`` :278-317, ``__call__`` :351-773): same argument
names, defaults and meaning, same CFG branch order [uncond, drop-audio-vasa, drop-vasa, cond], same
mode gates and ip_adapter_masks, same window / shift schedule. Differences, all deliberate:
  * the loop is ``pipeline.denoise`` (window x CFG-branch units, optional multi-GPU sharding with one
    RCCL all-gather per step, fp32 latent state);
  * noise is drawn from the given (CPU) ``generator`` and moved to the device (the reference draws on
    the device RNG, which differs across vendors anyway);
  * ``output_type`` "pt" / "np" / "latent" (no PIL conversion: image I/O is out of scope).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence, Union

import torch

from .pipeline import HipBackend, LoopConfig, broadcast_from_rank0, denoise, karras_sigmas
from .vae import decode_latents


@dataclass
class Pose2VideoSVDPipelineOutput:
    frames: Union[torch.Tensor, "object"]


def _linspace(a, b, n) -> List[float]:
    return [float(v) for v in torch.linspace(a, b, n)]


class Pose2VideoLongSVDPipeline:
    vae_scale_factor = 8

    def __init__(self, vae, unet, id_proj_model, pose_guider, scheduler=None, feature_extractor=None,
                 image_encoder=None):
        self.vae, self.unet, self.id_proj_model, self.pose_guider = vae, unet, id_proj_model, pose_guider
        self.scheduler, self.feature_extractor, self.image_encoder = scheduler, feature_extractor, image_encoder

    def to(self, device=None, dtype=None):
        for m in (self.vae, self.unet, self.id_proj_model, self.pose_guider):
            if m is not None:
                m.to(device)
        return self

    @property
    def device(self):
        return self.unet.device

    # ---------------------------------------------------------------- conditioning (pipeline:128-233)
    def _clip_encode_image(self, image, audio_prompts, uncond_audio_prompts, vasa_prompts, uncond_vasa_prompts,
                           num_frames, device, frames_per_batch):
        ide = self.id_proj_model(image.to(device).float())                       # (1, seq, 1024)
        ide = ide.float().unsqueeze(1).repeat(1, num_frames, 1, 1)               # (1, T, seq, 1024)
        ide = torch.cat([torch.zeros_like(ide), ide, ide, ide])
        a = torch.stack(list(audio_prompts), 0).to(device).float().unsqueeze(0)            # (1, N, 32, 1024)
        v = torch.stack(list(vasa_prompts), 0).to(device).float().unsqueeze(0).unsqueeze(2)
        ua = torch.stack(list(uncond_audio_prompts), 0).to(device).float().unsqueeze(0)
        uv = torch.stack(list(uncond_vasa_prompts), 0).to(device).float().unsqueeze(0).unsqueeze(2)
        pad_a = ua[:, :1].repeat(1, frames_per_batch, 1, 1)
        pad_v = uv[:, :1].repeat(1, frames_per_batch, 1, 1)
        a, ua = torch.cat([a, pad_a], 1), torch.cat([ua, pad_a], 1)
        v, uv = torch.cat([v, pad_v], 1), torch.cat([uv, pad_v], 1)
        return ide, torch.cat([ua, ua, a, a]), torch.cat([uv, uv, uv, v])

    def _encode_vae_image(self, image, device):
        lat = self.vae.encode(image.to(device).float()).latent_dist.mode()
        return torch.cat([torch.zeros_like(lat), lat, lat, lat])

    def _get_add_time_ids(self, fps, motion_bucket_id, noise_aug_strength, batch_size=1):
        ids = [fps, motion_bucket_id, noise_aug_strength]
        cfg = self.unet.config
        if cfg.addition_time_embed_dim * len(ids) != self.unet.add_embedding.linear_1.in_features:
            raise ValueError("Model expects an added time embedding vector of length "
                             f"{self.unet.add_embedding.linear_1.in_features}, but a vector of "
                             f"{cfg.addition_time_embed_dim * len(ids)} was created.")
        t = torch.tensor([ids], dtype=torch.float32).repeat(batch_size, 1)
        return torch.cat([t, t, t, t])

    # ---------------------------------------------------------------- call (pipeline:351-773)
    @torch.no_grad()
    def __call__(self, ref_image, clip_image, pose_images, exp_mask_images, mouth_mask_images, audio_prompts,
                 uncond_audio_prompts, vasa_prompts, uncond_vasa_prompts, height: int = 576, width: int = 1024,
                 num_frames: Optional[int] = None, num_inference_steps: int = 25, min_guidance_scale1=1.0,
                 max_guidance_scale1=3.0, min_guidance_scale2=1.0, max_guidance_scale2=3.0, min_guidance_scale3=1.0,
                 max_guidance_scale3=3.0, fps: int = 7, motion_bucket_id: int = 127, motion_bucket_id_exp: int = 127,
                 noise_aug_strength: float = 0.02, decode_chunk_size: Optional[int] = None,
                 num_videos_per_prompt: Optional[int] = 1, generator: Optional[torch.Generator] = None,
                 latents: Optional[torch.Tensor] = None, output_type: Optional[str] = "pt",
                 callback_on_step_end=None, callback_on_step_end_tensor_inputs: Sequence[str] = ("latents",),
                 return_dict: bool = True, overlap: int = 7, shift_offset: int = 3, frames_per_batch: int = 14,
                 i2i_noise_strength: float = 1.0, gate=(1, 1), world: int = 1, rank: int = 0, group=None):
        if num_videos_per_prompt != 1:
            raise ValueError("num_videos_per_prompt > 1 is not supported")
        if i2i_noise_strength != 1.0:
            raise ValueError("i2i_noise_strength < 1 (partial schedules) is not supported by the HIP loop")
        if not isinstance(ref_image, torch.Tensor) or ref_image.dim() != 4 or ref_image.shape[0] != 1:
            raise ValueError("ref_image must be a (1, 3, H, W) tensor in [-1, 1]")
        device = self.device
        num_frames = num_frames if num_frames is not None else len(pose_images)
        decode_chunk_size = decode_chunk_size if decode_chunk_size is not None else num_frames
        T = num_frames + frames_per_batch
        h, w = height // self.vae_scale_factor, width // self.vae_scale_factor

        image_embeddings, audio_cfg, vasa_cfg = self._clip_encode_image(
            clip_image, audio_prompts, uncond_audio_prompts, vasa_prompts, uncond_vasa_prompts, T, device,
            frames_per_batch)
        added_time_ids = self._get_add_time_ids(fps, motion_bucket_id, motion_bucket_id_exp)

        sigmas, _ = karras_sigmas(num_inference_steps)
        ref = ref_image.to(device).float()
        ref_latents = self.vae.encode(ref).latent_dist.mean * 0.18215
        aug = torch.randn(ref.shape, generator=generator)
        noise = latents if latents is not None else torch.randn((1, T, 4, h, w), generator=generator)
        if world > 1:
            # every rank must condition on the same noise-augmented image and start from the same
            # latents (the loop replicates guidance / Euler per rank): rank 0's draws are broadcast, so an
            # unseeded per-rank RNG (generator=None under torchrun) cannot make the ranks diverge
            aug, noise = aug.contiguous(), noise.float().clone()
            broadcast_from_rank0(aug, group)
            broadcast_from_rank0(noise, group)
        aug = aug.to(device)
        image_latents = self._encode_vae_image(ref + noise_aug_strength * aug, device)
        image_latents = image_latents.unsqueeze(1).repeat(1, T, 1, 1, 1)

        lat0 = ref_latents.unsqueeze(1) + noise.to(device).float() * sigmas[0]          # scheduler.add_noise at t0

        pose = torch.stack([p.to(device).float() for p in pose_images], 1)[None] if isinstance(pose_images, list) \
            else pose_images.to(device).float()                                      # (1, 3, N, H, W)
        face_mask = pose[0, :1, :1]
        exp_mask = torch.stack([m.to(device).float() for m in exp_mask_images], 1)[None][0, :1, :1]
        mouth_mask = torch.stack([m.to(device).float() for m in mouth_mask_images], 1)[None][0, :1, :1]
        pose_fea = self.pose_guider(pose).transpose(1, 2)                            # (1, N, 320, h, w)

        sched = list(zip(_linspace(min_guidance_scale1, max_guidance_scale1, num_inference_steps),
                         _linspace(min_guidance_scale2, max_guidance_scale2, num_inference_steps),
                         _linspace(min_guidance_scale3, max_guidance_scale3, num_inference_steps)))
        cfg = LoopConfig(num_frames=num_frames, frames_per_batch=frames_per_batch, overlap=overlap,
                         shift_offset=shift_offset, num_inference_steps=num_inference_steps, guidance=sched[0],
                         guidance_schedule=sched)
        backend = HipBackend(self.unet, h, w, (face_mask, mouth_mask, exp_mask), list(gate), added_time_ids, T,
                             frames_per_batch, image_latents, image_embeddings, audio_cfg, vasa_cfg, pose_fea)
        cb = None
        if callback_on_step_end is not None:
            def cb(i):
                callback_on_step_end(self, i, sigmas[i], {})
        lat = denoise(backend, lat0, cfg, rank=rank, world=world, group=group, step_callback=cb)
        if output_type == "latent":
            frames = lat
        else:
            frames = decode_latents(self.vae, lat, T, decode_chunk_size)[:, :, :num_frames]
            if output_type == "np":
                frames = frames.cpu().numpy()
        if not return_dict:
            return frames
        return Pose2VideoSVDPipelineOutput(frames=frames)
