"""Drop-in ``UNetSpatioTemporalConditionModel`` for ACTalker's ``unet_cls`` config key.

Reference: src/models/base/unet_spatio_temporal_condition_mambaID_v10_two_ip.py (class at :35,
``__init__`` :73-251, ``forward`` :362-517, ``add_ip_adapters`` :519-567 — the copy in
unet_spatio_temporal_condition.py:519-566 without the ``pdb.set_trace()``, and
``load_adapter_states`` :571-592). Selected by config/inference.yaml:62 via Inference.py:54-62::

    unet_cls: 'actalker_amd.unet_spatio_temporal_condition_mambaID_v10_two_ip.UNetSpatioTemporalConditionModel'

Same constructor arguments, config fields, attribute names, parameter names/shapes and forward
signature; the forward itself runs on the MI355X kernels of libactalker_hip.so (bf16 activations,
fp32 accumulation). There is no CPU path: calling forward on a CPU module raises.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass
from typing import Sequence, Any, Dict, List, Optional, Tuple, Union

import torch
import torch.nn as nn

from . import modules, ops
from .modules import (Attention, AttnProcessor2_0, Conv2d, CrossAttnDownBlockSpatioTemporal,
                      CrossAttnUpBlockSpatioTemporal, Ctx, DownBlockSpatioTemporal, GroupNorm,
                      IPAdapterAttnProcessor2_0, Timesteps, TimestepEmbedding,
                      TransformerSpatioTemporalModel_new_mambaID_v10_two_ip, UNetMidBlockSpatioTemporal,
                      UpBlockSpatioTemporal)

TransformerSpatioTemporalModel = TransformerSpatioTemporalModel_new_mambaID_v10_two_ip


@dataclass
class UNetSpatioTemporalConditionOutput:
    sample: torch.Tensor = None


class FrozenConfig(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


def get_down_block(down_block_type, num_layers, in_channels, out_channels, temb_channels, add_downsample,
                   resnet_eps, resnet_act_fn, num_attention_heads, cross_attention_dim=None,
                   transformer_layers_per_block=1, attn_cls=None, **_):
    """unet_3d_blocks.py:205-332 (SpatioTemporal branches)."""
    if down_block_type == "DownBlockSpatioTemporal":
        return DownBlockSpatioTemporal(num_layers=num_layers, in_channels=in_channels, out_channels=out_channels,
                                       temb_channels=temb_channels, add_downsample=add_downsample)
    if down_block_type == "CrossAttnDownBlockSpatioTemporal":
        if cross_attention_dim is None:
            raise ValueError("cross_attention_dim must be specified for CrossAttnDownBlockSpatioTemporal")
        return CrossAttnDownBlockSpatioTemporal(in_channels=in_channels, out_channels=out_channels,
                                                temb_channels=temb_channels, num_layers=num_layers,
                                                transformer_layers_per_block=transformer_layers_per_block,
                                                add_downsample=add_downsample,
                                                cross_attention_dim=cross_attention_dim,
                                                num_attention_heads=num_attention_heads, attn_cls=attn_cls)
    raise ValueError(f"{down_block_type} does not exist.")


def get_up_block(up_block_type, num_layers, in_channels, out_channels, prev_output_channel, temb_channels,
                 add_upsample, resnet_eps, resnet_act_fn, num_attention_heads, resolution_idx=None,
                 cross_attention_dim=None, transformer_layers_per_block=1, attn_cls=None, **_):
    """unet_3d_blocks.py:335-473. Note: resnet_eps is NOT forwarded (reference :446-471), so the
    up blocks keep their 1e-6 default."""
    if up_block_type == "UpBlockSpatioTemporal":
        return UpBlockSpatioTemporal(num_layers=num_layers, in_channels=in_channels, out_channels=out_channels,
                                     prev_output_channel=prev_output_channel, temb_channels=temb_channels,
                                     resolution_idx=resolution_idx, add_upsample=add_upsample)
    if up_block_type == "CrossAttnUpBlockSpatioTemporal":
        if cross_attention_dim is None:
            raise ValueError("cross_attention_dim must be specified for CrossAttnUpBlockSpatioTemporal")
        return CrossAttnUpBlockSpatioTemporal(in_channels=in_channels, out_channels=out_channels,
                                              prev_output_channel=prev_output_channel, temb_channels=temb_channels,
                                              num_layers=num_layers,
                                              transformer_layers_per_block=transformer_layers_per_block,
                                              add_upsample=add_upsample, cross_attention_dim=cross_attention_dim,
                                              num_attention_heads=num_attention_heads,
                                              resolution_idx=resolution_idx, attn_cls=attn_cls)
    raise ValueError(f"{up_block_type} does not exist.")


class UNetSpatioTemporalConditionModel(nn.Module):
    _supports_gradient_checkpointing = True

    def __init__(
        self,
        sample_size: Optional[int] = None,
        in_channels: int = 8,
        out_channels: int = 4,
        down_block_types: Tuple[str] = ("CrossAttnDownBlockSpatioTemporal", "CrossAttnDownBlockSpatioTemporal",
                                        "CrossAttnDownBlockSpatioTemporal", "DownBlockSpatioTemporal"),
        up_block_types: Tuple[str] = ("UpBlockSpatioTemporal", "CrossAttnUpBlockSpatioTemporal",
                                      "CrossAttnUpBlockSpatioTemporal", "CrossAttnUpBlockSpatioTemporal"),
        block_out_channels: Tuple[int] = (320, 640, 1280, 1280),
        addition_time_embed_dim: int = 256,
        projection_class_embeddings_input_dim: int = 768,
        layers_per_block: Union[int, Tuple[int]] = 2,
        cross_attention_dim: Union[int, Tuple[int]] = 1024,
        transformer_layers_per_block: Union[int, Tuple[int], Tuple[Tuple]] = 1,
        num_attention_heads: Union[int, Tuple[int]] = (5, 10, 20, 20),
        num_frames: int = 25,
        attn_cls: nn.Module = TransformerSpatioTemporalModel,
        **_ignored,
    ):
        super().__init__()
        self.config = FrozenConfig(
            sample_size=sample_size, in_channels=in_channels, out_channels=out_channels,
            down_block_types=tuple(down_block_types), up_block_types=tuple(up_block_types),
            block_out_channels=tuple(block_out_channels), addition_time_embed_dim=addition_time_embed_dim,
            projection_class_embeddings_input_dim=projection_class_embeddings_input_dim,
            layers_per_block=layers_per_block, cross_attention_dim=cross_attention_dim,
            transformer_layers_per_block=transformer_layers_per_block, num_attention_heads=num_attention_heads,
            num_frames=num_frames)
        self.sample_size = sample_size
        if len(down_block_types) != len(up_block_types):
            raise ValueError("Must provide the same number of `down_block_types` as `up_block_types`.")
        if len(block_out_channels) != len(down_block_types):
            raise ValueError("Must provide the same number of `block_out_channels` as `down_block_types`.")
        if not isinstance(num_attention_heads, int) and len(num_attention_heads) != len(down_block_types):
            raise ValueError("Must provide the same number of `num_attention_heads` as `down_block_types`.")
        if isinstance(cross_attention_dim, list) and len(cross_attention_dim) != len(down_block_types):
            raise ValueError("Must provide the same number of `cross_attention_dim` as `down_block_types`.")
        if not isinstance(layers_per_block, int) and len(layers_per_block) != len(down_block_types):
            raise ValueError("Must provide the same number of `layers_per_block` as `down_block_types`.")

        self.conv_in = Conv2d(in_channels, block_out_channels[0], kernel_size=3, padding=1)
        time_embed_dim = block_out_channels[0] * 4
        self.time_proj = Timesteps(block_out_channels[0], True, downscale_freq_shift=0)
        self.time_embedding = TimestepEmbedding(block_out_channels[0], time_embed_dim)
        self.add_time_proj = Timesteps(addition_time_embed_dim, True, downscale_freq_shift=0)
        self.add_embedding = TimestepEmbedding(projection_class_embeddings_input_dim, time_embed_dim)

        self.down_blocks = nn.ModuleList([])
        self.up_blocks = nn.ModuleList([])
        if isinstance(num_attention_heads, int):
            num_attention_heads = (num_attention_heads,) * len(down_block_types)
        if isinstance(cross_attention_dim, int):
            cross_attention_dim = (cross_attention_dim,) * len(down_block_types)
        if isinstance(layers_per_block, int):
            layers_per_block = [layers_per_block] * len(down_block_types)
        if isinstance(transformer_layers_per_block, int):
            transformer_layers_per_block = [transformer_layers_per_block] * len(down_block_types)

        output_channel = block_out_channels[0]
        for i, down_block_type in enumerate(down_block_types):
            input_channel = output_channel
            output_channel = block_out_channels[i]
            is_final_block = i == len(block_out_channels) - 1
            self.down_blocks.append(get_down_block(
                down_block_type, num_layers=layers_per_block[i],
                transformer_layers_per_block=transformer_layers_per_block[i], in_channels=input_channel,
                out_channels=output_channel, temb_channels=time_embed_dim, add_downsample=not is_final_block,
                resnet_eps=1e-5, cross_attention_dim=cross_attention_dim[i],
                num_attention_heads=num_attention_heads[i], resnet_act_fn="silu", attn_cls=attn_cls))

        self.mid_block = UNetMidBlockSpatioTemporal(
            block_out_channels[-1], temb_channels=time_embed_dim,
            transformer_layers_per_block=transformer_layers_per_block[-1],
            cross_attention_dim=cross_attention_dim[-1], num_attention_heads=num_attention_heads[-1])

        self.num_upsamplers = 0
        rev_ch = list(reversed(block_out_channels))
        rev_heads = list(reversed(num_attention_heads))
        rev_layers = list(reversed(layers_per_block))
        rev_cross = list(reversed(cross_attention_dim))
        rev_tl = list(reversed(transformer_layers_per_block))
        output_channel = rev_ch[0]
        for i, up_block_type in enumerate(up_block_types):
            is_final_block = i == len(block_out_channels) - 1
            prev_output_channel = output_channel
            output_channel = rev_ch[i]
            input_channel = rev_ch[min(i + 1, len(block_out_channels) - 1)]
            add_upsample = not is_final_block
            if add_upsample:
                self.num_upsamplers += 1
            self.up_blocks.append(get_up_block(
                up_block_type, num_layers=rev_layers[i] + 1, transformer_layers_per_block=rev_tl[i],
                in_channels=input_channel, out_channels=output_channel, prev_output_channel=prev_output_channel,
                temb_channels=time_embed_dim, add_upsample=add_upsample, resnet_eps=1e-5, resolution_idx=i,
                cross_attention_dim=rev_cross[i], num_attention_heads=rev_heads[i], resnet_act_fn="silu",
                attn_cls=attn_cls))

        self.conv_norm_out = GroupNorm(num_channels=block_out_channels[0], num_groups=32, eps=1e-5)
        self.conv_act = nn.SiLU()
        self.conv_out = Conv2d(block_out_channels[0], out_channels, kernel_size=3, padding=1)

    # -------------------------------------------------------------------------------- API
    @property
    def dtype(self) -> torch.dtype:
        return self.conv_in.weight.dtype

    @property
    def device(self) -> torch.device:
        return self.conv_in.weight.device

    @property
    def attn_processors(self) -> Dict[str, nn.Module]:
        out = {}
        for name, mod in self.named_modules():
            if isinstance(mod, Attention):
                out[f"{name}.processor"] = mod.processor
        return out

    def set_attn_processor(self, processor):
        count = len(self.attn_processors)
        if isinstance(processor, dict) and len(processor) != count:
            raise ValueError(f"A dict of processors was passed, but the number of processors {len(processor)} "
                             f"does not match the number of attention layers: {count}.")
        for name, mod in self.named_modules():
            if isinstance(mod, Attention):
                mod.set_processor(processor if not isinstance(processor, dict) else processor[f"{name}.processor"])

    def set_default_attn_processor(self):
        self.set_attn_processor(AttnProcessor2_0())

    def invalidate_kernel_cache(self):
        """Drop every packed kernel-layout weight (call after mutating parameters in place)."""
        for m in self.modules():
            if hasattr(m, "_acth_invalidate"):
                m._acth_invalidate()

    def _apply(self, fn, *args, **kwargs):
        r = super()._apply(fn, *args, **kwargs)
        self.invalidate_kernel_cache()
        return r

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        r = super().load_state_dict(state_dict, strict=strict, assign=assign)
        self.invalidate_kernel_cache()
        return r

    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path, subfolder: Optional[str] = None,
                        variant: Optional[str] = None, **kwargs):
        """Local-directory loader for a diffusers UNet folder (config.json + safetensors/bin weights).
        Keys absent from the checkpoint (Mamba / IP-adapter) keep their initialisation, like
        diffusers' ``low_cpu_mem_usage=False`` path used at Inference.py:56-62."""
        root = pretrained_model_name_or_path if subfolder is None else os.path.join(pretrained_model_name_or_path,
                                                                                      subfolder)
        if not os.path.isdir(root):
            raise OSError(f"{root} is not a local directory (no network access in this build)")
        with open(os.path.join(root, "config.json")) as f:
            cfg = {k: v for k, v in json.load(f).items() if not k.startswith("_")}
        model = cls(**cfg)
        stem = "diffusion_pytorch_model"
        names = ([f"{stem}.{variant}.safetensors", f"{stem}.{variant}.bin"] if variant else []) + \
                [f"{stem}.safetensors", f"{stem}.bin"]
        for n in names:
            p = os.path.join(root, n)
            if os.path.exists(p):
                if p.endswith(".safetensors"):
                    from safetensors.torch import load_file
                    sd = load_file(p)
                else:
                    sd = torch.load(p, map_location="cpu", weights_only=True)
                model.load_state_dict(sd, strict=False)
                break
        else:
            raise OSError(f"no weights found in {root}")
        return model

    # -------------------------------------------------------------------------------- forward
    def _prep_ctx(self, B, F, timestep, encoder_hidden_states, added_time_ids, cross_attention_kwargs,
                  temb_only: bool = False):
        """``temb_only``: the context of a shared CFG prefix (forward_tokens ``prefix_src``), which reads only
        the ResBlock time-embedding projections -- the token projections are skipped."""
        dev = self.device
        ctx = Ctx(B, F, dev)
        if not torch.is_tensor(timestep):
            timestep = torch.tensor([float(timestep)], device=dev)
        t = timestep.reshape(-1).to(dev, torch.float32)
        if t.numel() == 1:
            t = t.expand(B).contiguous()
        t_emb = self.time_proj.run(t)                                          # (B, 320)
        emb = self.time_embedding.run(t_emb)                                   # (B, 1280)
        aug = self.add_time_proj.run(added_time_ids.reshape(-1).to(dev, torch.float32))
        aug = aug.reshape(B, -1)                                               # (B, 768)
        # silu(emb + aug_emb): the only form in which the ResBlocks consume the embedding
        ctx.temb = self.add_embedding.run(aug, residual=emb, act_out=ops.ACT_SILU)

        if isinstance(encoder_hidden_states, tuple):
            id_h, ip = encoder_hidden_states
        else:
            id_h, ip = encoder_hidden_states, None
        cak = cross_attention_kwargs or {}
        ctx.masks = cak.get("ip_adapter_masks")
        gate = cak.get("acth_gate")       # optional hint from actalker_amd.pipeline: exact-zero branches
        if gate is not None:
            ctx.audio_zero, ctx.vasa_zero = bool(gate[0] == 0), bool(gate[1] == 0)
        ctx.has_ip = ip is not None
        self._batched_temb_projections(ctx)
        srcs = (id_h,) + ((ip[0], ip[1]) if ip is not None else ())
        batch = getattr(self, "acth_batch_ctx_projections", True)
        jobs = self._ctx_token_jobs(ctx, temb_only) if batch else []
        # The token side (ID / audio / VASA rows, their frame means and every projection of them) depends only on
        # the prompt rows and the weights: the sampler hands the same row tensors to every step of a window
        # layout (pipeline._run_units), so it is computed once per (rows, packed weights) and reused.
        key = (B, F, str(ops.act_dtype()), ctx.audio_zero, ctx.vasa_zero, temb_only, batch)
        cache = self.__dict__.setdefault("_acth_tok_cache", [])
        hit = None
        # only on the device's default stream: an entry made on one stream and read (or freed) on another would need
        # cross-stream events (LoopConfig.concurrent_calls > 1 runs calls on side streams)
        use_cache = (not temb_only and dev.type == "cuda"
                     and torch.cuda.current_stream(dev) == torch.cuda.default_stream(dev))
        if use_cache:
            for i, ent in enumerate(cache):
                if (ent["key"] == key and len(ent["srcs"]) == len(srcs)
                        and all(a is b and a._version == vb for a, b, vb in zip(srcs, ent["srcs"], ent["ver"]))
                        and len(ent["ws"]) == len(jobs) and all(j[1] is w for j, w in zip(jobs, ent["ws"]))):
                    hit = cache.pop(i)                    # entries hold tensors: found by identity, not ==
                    break
        if hit is not None:
            cache.insert(0, hit)                          # most recently used first
            for k, v in hit["fields"].items():
                setattr(ctx, k, v)
            return ctx
        if id_h.shape[0] == B:
            id_h = id_h.repeat_interleave(F, dim=0)
        ctx.id_tok = id_h.reshape(B * F, -1).to(dev, ops.act_dtype()).contiguous()
        if ip is not None:
            a, v = ip[0], ip[1]
            ctx.n_audio = a.shape[-2]
            ctx.audio_tok = a.reshape(B * F * ctx.n_audio, -1).to(dev, ops.act_dtype()).contiguous()
            ctx.vasa_tok = v.reshape(B * F, -1).to(dev, ops.act_dtype()).contiguous()
            ctx.audio_mean = ops.frame_mean(ctx.audio_tok, B, F, ctx.n_audio)
            ctx.vasa_mean = ops.frame_mean(ctx.vasa_tok, B, F, 1)
        ctx.id_mean = ops.frame_mean(ctx.id_tok, B, F, 1)
        self._run_ctx_token_jobs(ctx, jobs)
        if use_cache:
            names = ("id_tok", "audio_tok", "vasa_tok", "n_audio", "id_mean", "audio_mean", "vasa_mean", "vid",
                     "ipkv", "ipvb", "mamba_proj")
            cache.insert(0, dict(key=key, srcs=srcs, ver=tuple(t._version for t in srcs),
                                 ws=tuple(j[1] for j in jobs), fields={n: getattr(ctx, n) for n in names}))
            del cache[self._ACTH_TOK_CACHE:]
        return ctx

    # window layouts the sampler cycles through (the shift offset walks a few (frames, branches) layouts per run)
    _ACTH_TOK_CACHE = 8

    def _dev_ints(self, values, device, dtype=torch.int64) -> torch.Tensor:
        """Device copy of a small host list, cached by content (the sampler repeats the same
        prefix maps every step; a pageable host -> device copy waits for the stream to drain)."""
        cache = self.__dict__.setdefault("_acth_ints", {})
        key = (tuple(values), str(device), dtype)
        t = cache.get(key)
        if t is None:
            t = cache[key] = torch.tensor(values, dtype=dtype, device=device)
        return t

    def _ctx_mods(self):
        mods = self.__dict__.get("_acth_ctx_mods")
        if mods is None:                     # module lists, walked once (the tree is fixed after __init__)
            res, sp, tp, mb = [], [], [], []
            for m in self.modules():
                if isinstance(m, (modules.ResnetBlock2D, modules.TemporalResnetBlock)) and m.time_emb_proj is not None:
                    res.append(m)
                elif isinstance(m, modules.TransformerSpatioTemporalModel):
                    sp += [blk.attn2 for blk in m.transformer_blocks]
                    tp += [blk.attn2 for blk in m.temporal_transformer_blocks]
                elif isinstance(m, modules.SS2D_cond_v10):
                    mb.append(m)
            mods = self.__dict__["_acth_ctx_mods"] = (res, sp, tp, mb)
        return mods

    def _batched_temb_projections(self, ctx):
        """``temb`` through every ResBlock's ``time_emb_proj`` (diffusers resnet.py: ~40 per call) as one GEMM over
        the concatenated weights; the results are column views handed to the blocks (``ctx.tproj``), which fall
        back to their own GEMM when absent. Each of the separate products would be a 6- or 84-row GEMM filling
        3-10 workgroups for ~25-30 us."""
        if not getattr(self, "acth_batch_ctx_projections", True):
            return
        res = self._ctx_mods()[0]
        if res:
            lins = [m.time_emb_proj for m in res]
            tensors = [t for l in lins for t in ((l.weight, l.bias) if l.bias is not None else (l.weight,))]

            def pack_t():
                w = modules._bf(torch.cat([l.weight for l in lins], 0))
                b = torch.cat([l.bias if l.bias is not None else torch.zeros(l.out_features, device=l.weight.device)
                               for l in lins]).float().contiguous()
                return w, b
            w, b = modules._versioned_pack(self, "temb_all", tensors, pack_t)
            out = ops.gemm(ctx.temb, w, bias=b, out_f32=True)
            ctx.tproj, o = {}, 0
            for m, l in zip(res, lins):
                ctx.tproj[id(m)] = out[:, o:o + l.out_features]
                o += l.out_features

    def _ctx_token_jobs(self, ctx, temb_only: bool = False):
        """The per-call token projections as GEMMs over concatenated weights: the Mamba blocks' SiLU(ID / audio /
        VASA token projections) (mamba_layer.py:1955-1960), every IP attn2's audio K|V (to_k_ip[0] | to_v_ip[0])
        and VASA V (to_v_ip[1]) on the frame tokens (spatial) or the window means (temporal), and the ID token
        through each attn2's ``to_v`` (16 spatial on ``id_tok``, 16 temporal on ``id_mean``). Returns
        [(token attribute of ctx, packed weight, activation, [(ctx dict, key, column offset, columns)])]; the
        packed weights come from modules._versioned_pack, so the same objects come back while the weights are
        unchanged (the token cache in _prep_ctx keys on them)."""
        jobs = []
        if temb_only:
            return jobs
        res, sp, tp, mb = self._ctx_mods()
        if mb:
            groups = [("id", [m.id_proj for m in mb], "id_tok")]
            if ctx.has_ip:
                groups += [("audio", [m.audio_proj for m in mb], "audio_tok"),
                           ("exp", [m.exp_proj for m in mb], "vasa_tok")]
            for key, lins, tok in groups:
                ws = [l.weight for l in lins]
                w = modules._versioned_pack(self, ("mamba", key), ws, lambda ws=ws: modules._bf(torch.cat(ws, 0)))
                asg, o = [], 0
                for l in lins:
                    asg.append(("mamba_proj", id(l), o, l.out_features))
                    o += l.out_features
                jobs.append((tok, w, ops.ACT_SILU, asg))
        if ctx.has_ip:
            for key, attns, atok, vtok in (("s", sp, "audio_tok", "vasa_tok"), ("t", tp, "audio_mean", "vasa_mean")):
                ip = [(a, a.processor) for a in attns if modules.is_ip_processor(a.processor)]
                kv_procs = [(a, pr) for a, pr in ip if len(pr.to_k_ip) > 0 and len(pr.to_v_ip) > 0]
                vb_procs = [(a, pr) for a, pr in ip if len(pr.to_v_ip) > 1]
                for dst, zero, tok, procs, srcs in (
                        ("ipkv", ctx.audio_zero, atok, kv_procs,
                         [(pr.to_k_ip[0].weight, pr.to_v_ip[0].weight) for _, pr in kv_procs]),
                        ("ipvb", ctx.vasa_zero, vtok, vb_procs, [(pr.to_v_ip[1].weight,) for _, pr in vb_procs])):
                    if zero or not procs:
                        continue
                    flat = [t for ws in srcs for t in ws]
                    w = modules._versioned_pack(self, ("ip", key, len(srcs[0])), flat,
                                                lambda flat=flat: modules._bf(torch.cat(flat, 0)))
                    asg, o = [], 0
                    for (a, _), ws in zip(procs, srcs):
                        n = sum(t.shape[0] for t in ws)
                        asg.append((dst, id(a), o, n))
                        o += n
                    jobs.append((tok, w, ops.ACT_NONE, asg))
        for key, attns, tok in (("vid_s", sp, "id_tok"), ("vid_t", tp, "id_mean")):
            if not attns:
                continue
            ws = [a.to_v.weight for a in attns]
            w = modules._versioned_pack(self, key, ws, lambda ws=ws: modules._bf(torch.cat(ws, 0)))
            asg, o = [], 0
            for a, wt in zip(attns, ws):
                asg.append(("vid", id(a), o, wt.shape[0]))
                o += wt.shape[0]
            jobs.append((tok, w, ops.ACT_NONE, asg))
        return jobs

    def _run_ctx_token_jobs(self, ctx, jobs):
        ctx.mamba_proj, ctx.ipkv, ctx.ipvb, ctx.vid = {}, {}, {}, {}
        for tok, w, act, asg in jobs:
            t = getattr(ctx, tok)
            if t is None:
                continue
            out = ops.gemm(t, w, act=act)
            for dst, k, o, n in asg:
                getattr(ctx, dst)[k] = out[:, o:o + n]

    def compute_dtype(self) -> torch.dtype:
        """Activation dtype of the HIP path: ``acth_compute_dtype`` when set (torch.bfloat16 / torch.float16),
        otherwise fp16 for a UNet whose weights are fp16 -- the dtype the reference runs its UNet in
        (Inference.py:168-173, ``weight_dtype: fp16`` in its config) -- and bf16 for any other weight dtype.
        Weights are packed per dtype (modules._pk), so both paths can run on one module tree."""
        d = getattr(self, "acth_compute_dtype", None)
        if d is None:
            d = torch.float16 if self.conv_in.weight.dtype == torch.float16 else torch.bfloat16
        return d

    def forward_tokens(self, x_tok: torch.Tensor, B: int, F: int, H: int, W: int, timestep, encoder_hidden_states,
                       added_time_ids, spatial_condition_tok: Optional[torch.Tensor] = None,
                       cross_attention_kwargs: Optional[Dict[str, Any]] = None,
                       spatial_condition_rmap: Optional[torch.Tensor] = None, out_f32: bool = True,
                       spatial_condition_rmap_max: Optional[int] = None,
                       prefix_src: Optional[Sequence[int]] = None, out: Optional[torch.Tensor] = None):
        """Token-major entry: x_tok (B*F*H*W, in_channels) -> (B*F*H*W, out_channels), computed with
        ``compute_dtype()`` activations (token inputs in another dtype are converted on entry).
        ``spatial_condition_rmap`` (device int32, one entry per frame) remaps frame rows of
        ``spatial_condition_tok``; ``spatial_condition_rmap_max`` is the host-side bound on its entries.

        ``prefix_src`` (host list, one entry per batch element): batch element b computes the UNet prefix
        that reads no IP-adapter input -- conv_in, the first down block's first ResBlock, the first
        transformer's GroupNorm / proj_in and its first block's attn1 -- as element prefix_src[b] <= b
        does. The caller guarantees those elements' latent rows, spatial condition rows, timestep and
        added time ids are equal (the pipeline's CFG branches 1-3 of one window differ only in the audio /
        VASA / ID prompts, pipeline:162-200); the prefix then runs once per distinct element and its
        rows are copied out (exact: every op there is per batch element).

        ``out`` (optional, (B*F*H*W, out_channels) rows of the output dtype): conv_out writes there directly."""
        if self.device.type != "cuda":
            raise RuntimeError("UNetSpatioTemporalConditionModel (actalker_amd) runs on the MI355X HIP kernels "
                               "only; move it to a GPU device first")
        dt = self.compute_dtype()
        with ops.compute_dtype(dt):
            if x_tok.dtype != dt:
                x_tok = x_tok.to(dt)
            if spatial_condition_tok is not None and spatial_condition_tok.dtype != dt:
                spatial_condition_tok = spatial_condition_tok.to(dt)
            return self._forward_tokens(x_tok, B, F, H, W, timestep, encoder_hidden_states, added_time_ids,
                                        spatial_condition_tok, cross_attention_kwargs, spatial_condition_rmap,
                                        out_f32, spatial_condition_rmap_max, prefix_src, out)

    def _forward_tokens(self, x_tok, B, F, H, W, timestep, encoder_hidden_states, added_time_ids,
                        spatial_condition_tok, cross_attention_kwargs, spatial_condition_rmap, out_f32,
                        spatial_condition_rmap_max, prefix_src, out=None):
        ctx = self._prep_ctx(B, F, timestep, encoder_hidden_states, added_time_ids, cross_attention_kwargs)
        S0 = H * W
        uniq = None
        if prefix_src is not None and len(prefix_src) == B and self._prefix_capable():
            if any(prefix_src[b] > b or prefix_src[prefix_src[b]] != prefix_src[b] for b in range(B)):
                raise ValueError("prefix_src[b] must be <= b and name a distinct element")
            uniq = [b for b in range(B) if prefix_src[b] == b]
            if len(uniq) == B:
                uniq = None
        prefix = None
        if uniq is not None:
            Bu = len(uniq)
            pos = {b: i for i, b in enumerate(uniq)}
            ui = self._dev_ints(uniq, x_tok.device)
            ui32 = self._dev_ints(uniq, x_tok.device, torch.int32)
            inv_h = [pos[prefix_src[b]] for b in range(B)]
            inv = self._dev_ints(inv_h, x_tok.device, torch.int32)

            def take(t, per):                # rows of the distinct elements (t holds B x per rows)
                if t.is_cuda and t.is_contiguous() and (t.numel() // B * t.element_size()) % 16 == 0:
                    return ops.gather_blocks(t, B, ui32, max(uniq))
                return t.reshape(B, per, *t.shape[1:]).index_select(0, ui).reshape(Bu * per, *t.shape[1:])

            def expand(t):                   # distinct-element rows -> the full batch (one block-gather launch)
                return ops.gather_blocks(t.contiguous(), Bu, inv, max(inv_h))

            if isinstance(encoder_hidden_states, tuple):
                ehs_u = (take(encoder_hidden_states[0], F), [take(e, F) for e in encoder_hidden_states[1]])
            else:
                ehs_u = take(encoder_hidden_states, F)
            added_u = added_time_ids.reshape(B, -1).index_select(0, ui.to(added_time_ids.device))
            t_u = timestep
            if torch.is_tensor(timestep) and timestep.numel() == B:
                t_u = timestep.reshape(-1).index_select(0, ui.to(timestep.device))
            ctx_u = self._prep_ctx(Bu, F, t_u, ehs_u, added_u, cross_attention_kwargs, temb_only=True)
            prefix = (ctx_u, expand)
            x_in = take(x_tok, F * S0)
            rmap_in = take(spatial_condition_rmap, F) if spatial_condition_rmap is not None else None
            sc_in = spatial_condition_tok
            if sc_in is not None and rmap_in is None and sc_in.shape[0] == B * F * S0:
                sc_in = take(sc_in, F * S0)            # per-element rows (no frame remap)
            B_in = Bu
        else:
            x_in, rmap_in, sc_in, B_in = x_tok, spatial_condition_rmap, spatial_condition_tok, B
        # conv_in (+ spatial_condition add fused as the residual)
        cols = ops.im2col3x3(x_in, B_in * F, H, W)
        kw = {}
        if sc_in is not None:
            kw = dict(residual=sc_in)
            if rmap_in is not None:
                # row (u*F + f)*S0 + s reads spatial_condition row rmap[u*F + f]*S0 + s
                if spatial_condition_rmap_max is None:
                    raise ValueError("spatial_condition_rmap needs spatial_condition_rmap_max")
                kw.update(rmap=rmap_in, r_div=S0, r_mod=rmap_in.numel(), rmap_max=spatial_condition_rmap_max)
        h = ops.gemm(cols, self._conv_in_w(), bias=self.conv_in.b(), **kw)
        del cols
        BF = B * F
        if prefix is not None:
            skips = [expand(h)]
            h, outs, H, W = self.down_blocks[0].run(ctx, h, H, W, prefix=prefix)
            skips.extend(outs)
            rest = self.down_blocks[1:]
        else:
            skips = [h]
            rest = self.down_blocks
        for blk in rest:
            h, outs, H, W = blk.run(ctx, h, H, W)
            skips.extend(outs)
        h = self.mid_block.run(ctx, h, H, W)
        for blk in self.up_blocks:
            h, H, W = blk.run(ctx, h, skips, H, W)
        g, b = self.conv_norm_out.gb()
        n = ops.groupnorm(h, g, b, self.conv_norm_out.eps, H * W, silu=True)
        return ops.conv3x3(n, self.conv_out.w3(), BF, H, W, bias=self.conv_out.b(), out_f32=out_f32, out=out)

    def _prefix_capable(self) -> bool:
        from .modules import CrossAttnDownBlockSpatioTemporal
        b0 = self.down_blocks[0]
        return isinstance(b0, CrossAttnDownBlockSpatioTemporal) and len(b0.attentions) > 0

    def _conv_in_w(self):
        # conv_in has Cin = 8 < 64: explicit im2col + dense GEMM, weight as (Cout, 9*Cin)
        return self.conv_in.w3()

    def forward(self, sample: torch.Tensor, timestep: Union[torch.Tensor, float, int], encoder_hidden_states,
                added_time_ids: torch.Tensor, spatial_condition: Optional[torch.Tensor] = None,
                cross_attention_kwargs: Optional[Dict[str, Any]] = None, return_dict: bool = True):
        B, F = sample.shape[:2]
        H, W = sample.shape[-2:]
        with torch.no_grad(), ops.compute_dtype(self.compute_dtype()):
            x = ops.nchw_to_tokens(sample.to(self.device))
            sc = ops.nchw_to_tokens(spatial_condition.to(self.device)) if spatial_condition is not None else None
            out = self.forward_tokens(x, B, F, H, W, timestep, encoder_hidden_states, added_time_ids, sc,
                                      cross_attention_kwargs)
            out = ops.tokens_to_nchw(out, B * F, H, W, out_dtype=torch.float32)
        out = out.reshape(B, F, *out.shape[1:]).to(sample.dtype)
        if not return_dict:
            return (out,)
        return UNetSpatioTemporalConditionOutput(sample=out)


# ------------------------------------------------------------------------------------------
def add_ip_adapters(unet, num_adapter_embeds=[32, ], scale=[1.0, ]):
    """unet_spatio_temporal_condition.py:519-566: attn1 -> AttnProcessor2_0, attn2 ->
    IPAdapterAttnProcessor2_0 whose to_k_ip / to_v_ip start as copies of to_k / to_v."""
    assert len(num_adapter_embeds) == len(scale)
    attn_procs = {}
    unet_sd = unet.state_dict()
    for name in unet.attn_processors.keys():
        cross_attention_dim = None if name.endswith("attn1.processor") else unet.config.cross_attention_dim
        if name.startswith("mid_block"):
            hidden_size = unet.config.block_out_channels[-1]
        elif name.startswith("up_blocks"):
            block_id = int(name[len("up_blocks.")])
            hidden_size = list(reversed(unet.config.block_out_channels))[block_id]
        elif name.startswith("down_blocks"):
            block_id = int(name[len("down_blocks.")])
            hidden_size = unet.config.block_out_channels[block_id]
        if cross_attention_dim is None:
            attn_procs[name] = AttnProcessor2_0()
        else:
            attn_procs[name] = IPAdapterAttnProcessor2_0(hidden_size=hidden_size,
                                                         cross_attention_dim=cross_attention_dim,
                                                         num_tokens=num_adapter_embeds, scale=scale
                                                         ).to(device=unet.device, dtype=unet.dtype)
            layer_name = name.split(".processor")[0]
            weights = {}
            for i in range(len(num_adapter_embeds)):
                weights[f"to_k_ip.{i}.weight"] = unet_sd[layer_name + ".to_k.weight"]
                weights[f"to_v_ip.{i}.weight"] = unet_sd[layer_name + ".to_v.weight"]
            attn_procs[name].load_state_dict(weights)
    unet.set_attn_processor(attn_procs)
    return torch.nn.ModuleList([m for m in unet.attn_processors.values()
                                if isinstance(m, IPAdapterAttnProcessor2_0)])


def load_adapter_states(adapter_modules, state_dict_list):
    """unet_spatio_temporal_condition.py:570-591: merge adapter state dicts, renumbering the
    adapter index (key field 2) on collisions; loads with strict=False."""
    assert len(state_dict_list) > 0
    merged = {}
    for state_dict in state_dict_list:
        for k, v in state_dict.items():
            if k in merged:
                k_split = k.split('.')
                idx = int(k_split[2]) + 1
                k_split[2] = str(idx)
                new_k = '.'.join(k_split)
                while new_k in merged:
                    idx += 1
                    k_split[2] = str(idx)
                    new_k = '.'.join(k_split)
                merged[new_k] = v
            else:
                merged[k] = v
    info = adapter_modules.load_state_dict(merged, strict=False)
    for m in adapter_modules.modules():
        if hasattr(m, "_acth_invalidate"):
            m._acth_invalidate()
    return info
