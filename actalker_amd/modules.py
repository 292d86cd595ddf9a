"""Parameter containers and token-major HIP forward passes for the SVD-XT spatio-temporal UNet
with ACTalker's masked dual-Mamba branches.

Module names, attribute names and parameter shapes mirror the reference (and the diffusers
0.29.2 building blocks it instantiates) exactly, so reference ``state_dict``s load with
``strict=True``. The forward passes do not: activations stay token-major ``(B*F*h*w, C)`` in
bf16 end to end (no NCHW<->NHWC permutes), every contraction / norm / attention / scan runs in
libactalker_hip.so, and weights are re-packed once into the kernels' layouts.

Reference map (file:line under /root/reference/src/models/base unless noted):
  SpatioTemporalResBlock / ResnetBlock2D / TemporalResnetBlock   diffusers.models.resnet (0.29.2)
  Downsample2D / Upsample2D / TimestepEmbedding / FeedForward     diffusers (0.29.2)
  AlphaBlender                        TransformerSTmodel.py:116-197
  BasicTransformerBlock               attention.py:29-343
  TemporalBasicTransformerBlock       attention.py:347-473
  AttnProcessor2_0                    attention_processor.py:1518-1605
  IPAdapterAttnProcessor2_0           attention_processor.py:2704-2934
  SS2D_Unit / SS2D_cond_v10           mamba_layer.py:1394-1553 / 1902-1986
  TransformerSpatioTemporalModel      TransformerSTmodel.py:200-421
  ..._new_mambaID_v10_two_ip          TransformerSTmodel.py:3908-4155
  *BlockSpatioTemporal                unet_3d_blocks.py:2047-2592
"""
from __future__ import annotations

import math
import weakref
import os
from typing import List, Optional

import torch
import torch.nn as nn

from . import ops
from .masks import mask_info


# ------------------------------------------------------------------------------------------
# packing helpers (weights -> kernel layouts, cached per module until invalidated)
class Packed(nn.Module):
    """Mixin: per-module cache of kernel-layout weights."""

    def _pk(self, key, fn):
        # kernel layouts are per activation dtype (bf16 / fp16 builds, ops.compute_dtype)
        key = (key, ops.act_dtype())
        cache = self.__dict__.setdefault("_acth_cache", {})
        v = cache.get(key)
        if v is None:
            with torch.no_grad():
                v = fn()
            cache[key] = v
        return v

    def _acth_invalidate(self):
        self.__dict__["_acth_cache"] = {}


def _bf(w: torch.Tensor) -> torch.Tensor:
    """A weight in the current activation dtype (bf16, or fp16 inside ops.compute_dtype(torch.float16))."""
    return w.detach().to(ops.act_dtype()).contiguous()


def _f32(b: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    return None if b is None else b.detach().to(torch.float32).contiguous()


def pack_conv3x3(w: torch.Tensor) -> torch.Tensor:
    """(Cout, Cin, 3, 3) -> (Cout, 9*Cin) with k = (ky*3 + kx)*Cin + c."""
    return _bf(w.permute(0, 2, 3, 1).reshape(w.shape[0], -1))


def pack_conv3d_t(w: torch.Tensor) -> torch.Tensor:
    """(Cout, Cin, 3, 1, 1) -> (Cout, 3*Cin) with k = kf*Cin + c."""
    return _bf(w[:, :, :, 0, 0].permute(0, 2, 1).reshape(w.shape[0], -1))


GEGLU_G = 16   # GEGLU granule: the GEMM epilogues pair hidden column j with gate column j + 16


def pack_geglu(w: torch.Tensor, b: torch.Tensor):
    """GEGLU proj (2*I, C) [hidden; gate] -> rows interleaved in 16-row granules [h16, g16, h16, ...], so
    every 32 consecutive GEMM output columns hold 16 hidden and their 16 gate columns (the 16x16 MFMA
    fragment width): the GELU gate fuses into the GEMM epilogue."""
    inner = w.shape[0] // 2
    G = GEGLU_G
    hw, gw = w[:inner], w[inner:]
    hb, gb = b[:inner], b[inner:]
    wi = torch.stack([hw.view(inner // G, G, -1), gw.view(inner // G, G, -1)], 1).reshape(2 * inner, -1)
    bi = torch.stack([hb.view(inner // G, G), gb.view(inner // G, G)], 1).reshape(-1)
    return _bf(wi), _f32(bi)


def ffn_w2_perm(inner: int) -> torch.Tensor:
    """Column order of the fused feed-forward's W2 (acth_geglu_ffn): within each 16-unit granule, column
    8 hi + e holds unit 8 (e // 4) + 4 hi + e % 4 -- the order in which lane (token, hi) of the
    up projection's 32x32 MFMA fragment holds its 8 gated units, i.e. the down projection's K order."""
    hi, e = torch.arange(2).view(2, 1), torch.arange(8).view(1, 8)
    local = (8 * (e // 4) + 4 * hi + e % 4).reshape(16)
    return (torch.arange(0, inner, 16).view(-1, 1) + local.view(1, 16)).reshape(-1)


def pack_ffn_w2(w: torch.Tensor) -> torch.Tensor:
    """FeedForward output Linear (C, I) -> columns permuted by ffn_w2_perm, times 0.5 (the kernel
    carries 2 h gelu(g); scaling by a power of two is exact in bf16)."""
    return _bf(0.5 * w[:, ffn_w2_perm(w.shape[1]).to(w.device)].float())


FUSED_FFN = os.environ.get("ACTH_FUSED_FFN", "1") != "0"
# the fused IP-adapter cross attention block (acth_ip_fold + acth_xattn) where its shape allows; 0 = the
# unfused norm2 / to_q / ip_attn / to_out / norm3 ops (A/B benchmarks, tests)
FUSED_XATTN = os.environ.get("ACTH_FUSED_XATTN", "1") != "0"
# the blocks' "LayerNorm -> FeedForward" pairs (norm3 -> ff, norm_in (+ pos_emb) -> ff_in) as one kernel: the
# LayerNorm runs in acth_geglu_ffn's prologue; 0 = a separate acth_layernorm pass (A/B benchmarks, tests)
FUSED_FFN_LN = os.environ.get("ACTH_FUSED_FFN_LN", "1") != "0"


# ------------------------------------------------------------------------------------------
class Ctx:
    """Per-UNet-call state shared by all blocks."""

    def __init__(self, B: int, F: int, device):
        self.B, self.F, self.BF = B, F, B * F
        self.device = device
        self.temb = None            # silu(emb): (B, 1280) bf16
        self.id_tok = None          # (BF, 1024)
        self.audio_tok = None       # (BF*32, 1024)
        self.vasa_tok = None        # (BF, 1024)
        self.n_audio = 32
        self.id_mean = None         # (B, 1024)
        self.audio_mean = None      # (B*32, 1024)
        self.vasa_mean = None       # (B, 1024)
        self.masks = None           # [mask_audio, mask_exp] (1,1,H,W) or None
        self.audio_zero = False     # gate hints: tokens known to be exactly zero
        self.vasa_zero = False
        self.has_ip = True
        self.tproj = {}             # id(ResBlock) -> its time_emb_proj(temb) (B, C) f32 view (batched GEMM)
        self.vid = {}               # id(attn2) -> its to_v(ID token) (rows, C) bf16 view (batched GEMM)
        self.ipkv = {}              # id(attn2) -> IP audio K|V (rows, 2C) view (batched GEMM)
        self.ipvb = {}              # id(attn2) -> IP VASA V (rows, C) view (batched GEMM)
        self.mamba_proj = {}        # id(Mamba id / audio / exp Linear) -> SiLU(tokens @ W^T) view (batched)

    def temb_proj(self, blk):
        tp = self.tproj.get(id(blk))
        if tp is None:
            tp = ops.gemm(self.temb, blk.time_emb_proj.w(), bias=blk.time_emb_proj.b(), out_f32=True)
        return tp

    def mask(self, k: int, S: int):
        if self.masks is None:
            return None
        return mask_info(self.masks[k], S, self.device)


# ------------------------------------------------------------------------------------------
class Linear(nn.Linear, Packed):
    def w(self):
        return self._pk("w", lambda: _bf(self.weight))

    def b(self):
        return self._pk("b", lambda: _f32(self.bias))


class Conv2d(nn.Conv2d, Packed):
    def w3(self):
        return self._pk("w3", lambda: pack_conv3x3(self.weight))

    def w1(self):
        return self._pk("w1", lambda: _bf(self.weight[:, :, 0, 0]))

    def b(self):
        return self._pk("b", lambda: _f32(self.bias))


class Conv3d(nn.Conv3d, Packed):
    def wt(self):
        return self._pk("wt", lambda: pack_conv3d_t(self.weight))

    def w1(self):
        return self._pk("w1", lambda: _bf(self.weight[:, :, 0, 0, 0]))

    def b(self):
        return self._pk("b", lambda: _f32(self.bias))


class GroupNorm(nn.GroupNorm, Packed):
    def gb(self):
        return self._pk("gb", lambda: (_f32(self.weight), _f32(self.bias)))


class LayerNorm(nn.LayerNorm, Packed):
    def gb(self):
        return self._pk("gb", lambda: (_f32(self.weight), _f32(self.bias)))


# ------------------------------------------------------------------------------------------
class Timesteps(nn.Module):
    def __init__(self, num_channels: int, flip_sin_to_cos: bool, downscale_freq_shift: float, scale: int = 1):
        super().__init__()
        self.num_channels = num_channels
        self.flip_sin_to_cos = flip_sin_to_cos
        self.downscale_freq_shift = downscale_freq_shift
        self.scale = scale

    def run(self, t: torch.Tensor) -> torch.Tensor:
        return ops.timestep_embedding(t, self.num_channels, self.flip_sin_to_cos, self.downscale_freq_shift,
                                      self.scale)


class TimestepEmbedding(nn.Module):
    def __init__(self, in_channels: int, time_embed_dim: int, out_dim: Optional[int] = None):
        super().__init__()
        self.linear_1 = Linear(in_channels, time_embed_dim)
        self.act = nn.SiLU()
        self.linear_2 = Linear(time_embed_dim, out_dim if out_dim is not None else time_embed_dim)

    def run(self, x, residual=None, act_out=ops.ACT_NONE):
        h = ops.gemm(x, self.linear_1.w(), bias=self.linear_1.b(), act=ops.ACT_SILU)
        return ops.gemm(h, self.linear_2.w(), bias=self.linear_2.b(), residual=residual, act=act_out)


class AlphaBlender(Packed):
    def __init__(self, alpha: float, merge_strategy: str = "learned_with_images",
                 switch_spatial_to_temporal_mix: bool = False):
        super().__init__()
        self.merge_strategy = merge_strategy
        self.switch_spatial_to_temporal_mix = switch_spatial_to_temporal_mix
        self.register_parameter("mix_factor", nn.Parameter(torch.Tensor([alpha])))

    def alpha(self) -> float:
        # image_only_indicator is all zeros in the UNet (v10:454): alpha = sigmoid(mix_factor);
        # read once per weight load (host float) so the forward never syncs
        def f():
            a = torch.sigmoid(self.mix_factor.detach().float()).item()
            return 1.0 - a if self.switch_spatial_to_temporal_mix else a
        return self._pk("alpha", f)


# ------------------------------------------------------------------------------------------
class ResnetBlock2D(nn.Module):
    def __init__(self, in_channels, out_channels, temb_channels, eps):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.norm1 = GroupNorm(32, in_channels, eps=eps, affine=True)
        self.conv1 = Conv2d(in_channels, out_channels, 3, 1, 1)
        # temb_channels=None: no time embedding (the VAE's blocks, diffusers resnet.py)
        self.time_emb_proj = Linear(temb_channels, out_channels) if temb_channels is not None else None
        self.norm2 = GroupNorm(32, out_channels, eps=eps, affine=True)
        self.dropout = nn.Dropout(0.0)
        self.conv2 = Conv2d(out_channels, out_channels, 3, 1, 1)
        self.nonlinearity = nn.SiLU()
        self.use_in_shortcut = in_channels != out_channels
        self.conv_shortcut = Conv2d(in_channels, out_channels, 1, 1, 0) if self.use_in_shortcut else None

    def run(self, ctx: Ctx, x, x2, H, W):
        S = H * W
        g1, b1 = self.norm1.gb()
        n1 = ops.groupnorm(x, g1, b1, self.norm1.eps, S, x2=x2, silu=True)
        tp = ctx.temb_proj(self)
        h = ops.conv3x3(n1, self.conv1.w3(), ctx.BF, H, W, bias=self.conv1.b(), rowbias=tp, rb_div=ctx.F * S)
        del n1
        g2, b2 = self.norm2.gb()
        n2 = ops.groupnorm(h, g2, b2, self.norm2.eps, S, silu=True)
        del h
        if self.conv_shortcut is not None:
            sc = ops.gemm(x, self.conv_shortcut.w1(), a2=x2, bias=self.conv_shortcut.b())
        else:
            sc = x
        return ops.conv3x3(n2, self.conv2.w3(), ctx.BF, H, W, bias=self.conv2.b(), residual=sc)


class TemporalResnetBlock(nn.Module):
    def __init__(self, in_channels, out_channels, temb_channels, eps):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.norm1 = GroupNorm(32, in_channels, eps=eps, affine=True)
        self.conv1 = Conv3d(in_channels, out_channels, kernel_size=(3, 1, 1), stride=1, padding=(1, 0, 0))
        self.time_emb_proj = Linear(temb_channels, out_channels) if temb_channels is not None else None
        self.norm2 = GroupNorm(32, out_channels, eps=eps, affine=True)
        self.dropout = nn.Dropout(0.0)
        self.conv2 = Conv3d(out_channels, out_channels, kernel_size=(3, 1, 1), stride=1, padding=(1, 0, 0))
        self.nonlinearity = nn.SiLU()
        self.use_in_shortcut = in_channels != out_channels
        self.conv_shortcut = (Conv3d(in_channels, out_channels, kernel_size=1, stride=1, padding=0)
                              if self.use_in_shortcut else None)

    def run(self, ctx: Ctx, x, S, mix, mix_alpha):
        FS = ctx.F * S
        g1, b1 = self.norm1.gb()
        n1 = ops.groupnorm(x, g1, b1, self.norm1.eps, FS, silu=True)
        tp = ctx.temb_proj(self)
        t = ops.gemm(n1, self.conv1.wt(), temporal=dict(F=ctx.F, S=S), bias=self.conv1.b(), rowbias=tp, rb_div=FS)
        del n1
        g2, b2 = self.norm2.gb()
        n2 = ops.groupnorm(t, g2, b2, self.norm2.eps, FS, silu=True)
        del t
        sc = x if self.conv_shortcut is None else ops.gemm(x, self.conv_shortcut.w1(), bias=self.conv_shortcut.b())
        # output = input + conv2(...); AlphaBlender: a * x_spatial + (1 - a) * output
        return ops.gemm(n2, self.conv2.wt(), temporal=dict(F=ctx.F, S=S), bias=self.conv2.b(), residual=sc,
                        mix=mix, mix_alpha=mix_alpha)


class SpatioTemporalResBlock(nn.Module):
    def __init__(self, in_channels, out_channels=None, temb_channels=512, eps=1e-6, temporal_eps=None,
                 merge_factor=0.5, merge_strategy="learned_with_images", switch_spatial_to_temporal_mix=False):
        super().__init__()
        out_channels = in_channels if out_channels is None else out_channels
        self.spatial_res_block = ResnetBlock2D(in_channels, out_channels, temb_channels, eps)
        self.temporal_res_block = TemporalResnetBlock(out_channels, out_channels, temb_channels,
                                                      temporal_eps if temporal_eps is not None else eps)
        self.time_mixer = AlphaBlender(merge_factor, merge_strategy, switch_spatial_to_temporal_mix)

    def run(self, ctx: Ctx, x, H, W, x2=None):
        hs = self.spatial_res_block.run(ctx, x, x2, H, W)
        return self.temporal_res_block.run(ctx, hs, H * W, hs, self.time_mixer.alpha())


class Downsample2D(nn.Module):
    def __init__(self, channels, use_conv=True, out_channels=None, padding=1, name="conv"):
        super().__init__()
        out_channels = out_channels or channels
        self.conv = Conv2d(channels, out_channels, 3, stride=2, padding=padding)

    def run(self, ctx, x, H, W):
        return ops.conv3x3(x, self.conv.w3(), ctx.BF, H, W, stride=2, bias=self.conv.b())


class Upsample2D(nn.Module):
    def __init__(self, channels, use_conv=True, out_channels=None):
        super().__init__()
        out_channels = out_channels or channels
        self.conv = Conv2d(channels, out_channels, 3, padding=1)

    def run(self, ctx, x, H, W):
        return ops.conv3x3(x, self.conv.w3(), ctx.BF, H, W, upsample=True, bias=self.conv.b())


# ------------------------------------------------------------------------------------------
class AttnProcessor2_0(nn.Module):
    """Plain SDPA processor (no parameters)."""


class IPAdapterAttnProcessor2_0(Packed):
    def __init__(self, hidden_size, cross_attention_dim=None, num_tokens=(4,), scale=1.0):
        super().__init__()
        self.hidden_size = hidden_size
        self.cross_attention_dim = cross_attention_dim
        if not isinstance(num_tokens, (tuple, list)):
            num_tokens = [num_tokens]
        self.num_tokens = num_tokens
        if not isinstance(scale, (tuple, list)):
            scale = [scale] * len(num_tokens)
        if len(scale) != len(num_tokens):
            raise ValueError("`scale` should be a list of integers with the same length as `num_tokens`.")
        self.scale = scale
        self.to_k_ip = nn.ModuleList([Linear(cross_attention_dim, hidden_size, bias=False) for _ in num_tokens])
        self.to_v_ip = nn.ModuleList([Linear(cross_attention_dim, hidden_size, bias=False) for _ in num_tokens])

    def w_kv(self, i):
        """to_k_ip[i] | to_v_ip[i] fused as one (2C, cross_dim) weight."""
        return ip_w_kv(self, i)


def _scale_value(s) -> float:
    return float(s[0]) if isinstance(s, (list, tuple)) else float(s)


def is_ip_processor(proc) -> bool:
    """An IP-adapter processor: ours, or the reference's own IPAdapterAttnProcessor2_0 object that the
    reference's unmodified ``add_ip_adapters`` (unet_spatio_temporal_condition.py:519-566) installs
    through ``set_attn_processor`` -- anything with ``to_k_ip`` / ``to_v_ip`` lists and ``scale``."""
    return hasattr(proc, "to_k_ip") and hasattr(proc, "to_v_ip") and hasattr(proc, "scale")


def _versioned_pack(mod: nn.Module, key, tensors, fn):
    """Kernel-layout pack cached on ``mod`` and keyed on the source tensors' in-place version counters,
    so a later ``load_state_dict`` into a foreign processor (the reference's ``load_adapter_states``)
    invalidates it without any hook of ours. The entry also holds weak references to the source tensors
    themselves: a replaced Parameter (a fresh tensor that the caching allocator may place at the freed
    address, with _version 0 again) never matches a stale entry."""
    cache = mod.__dict__.setdefault("_acth_vcache", {})
    key = (key, ops.act_dtype())         # one layout per activation dtype (ops.compute_dtype)
    ver = tuple((t.data_ptr(), t._version) for t in tensors)
    hit = cache.get(key)
    if hit is None or hit[0] != ver or any(r() is not t for r, t in zip(hit[2], tensors)):
        with torch.no_grad():
            hit = (ver, fn(), tuple(weakref.ref(t) for t in tensors))
        cache[key] = hit
    return hit[1]


def ip_w_kv(proc, i):
    """to_k_ip[i] | to_v_ip[i] fused as one (2C, cross_dim) bf16 weight."""
    k, v = proc.to_k_ip[i].weight, proc.to_v_ip[i].weight
    return _versioned_pack(proc, ("kv", i), (k, v), lambda: _bf(torch.cat([k, v], 0)))


def ip_w_v(proc, i):
    v = proc.to_v_ip[i].weight
    return _versioned_pack(proc, ("v", i), (v,), lambda: _bf(v))


class Attention(Packed):
    def __init__(self, query_dim, cross_attention_dim=None, heads=8, dim_head=64, dropout=0.0, bias=False,
                 upcast_attention=False, out_bias=True):
        super().__init__()
        inner = heads * dim_head
        self.heads = heads
        self.is_cross = cross_attention_dim is not None
        kv_dim = cross_attention_dim if cross_attention_dim is not None else query_dim
        self.to_q = Linear(query_dim, inner, bias=bias)
        self.to_k = Linear(kv_dim, inner, bias=bias)
        self.to_v = Linear(kv_dim, inner, bias=bias)
        self.to_out = nn.ModuleList([Linear(inner, query_dim, bias=out_bias), nn.Dropout(dropout)])
        self.processor = AttnProcessor2_0()

    def set_processor(self, processor):
        self.processor = processor
        self._acth_invalidate()

    def w_qkv(self):
        return self._pk("qkv", lambda: _bf(torch.cat([self.to_q.weight, self.to_k.weight, self.to_v.weight], 0)))

    # -- spatial / temporal self-attention: out = to_out(attn(LN(x))) + x
    def run_self(self, ctx: Ctx, n, x_res, S, temporal: bool):
        C = self.heads * 64
        qkv = ops.gemm(n, self.w_qkv())
        if temporal:
            a = ops.temporal_attn(qkv, ctx.B, ctx.F, S, self.heads)
        else:
            a = ops.flash_attn(qkv, ctx.BF, S, self.heads)
        del qkv
        return ops.gemm(a, self.to_out[0].w(), bias=self.to_out[0].b(), residual=x_res)

    # -- cross attention (ID token + IP-adapter audio / VASA tokens)
    def run_cross(self, ctx: Ctx, n, x_res, S, temporal: bool):
        M = n.shape[0]
        if temporal:
            id_tok, audio, vasa, rows_per_ctx = ctx.id_mean, ctx.audio_mean, ctx.vasa_mean, ctx.F * S
            ma = mb = None
            use_a, use_b = not ctx.audio_zero, not ctx.vasa_zero
        else:
            id_tok, audio, vasa, rows_per_ctx = ctx.id_tok, ctx.audio_tok, ctx.vasa_tok, S
            ia, ib = ctx.mask(0, S), ctx.mask(1, S)
            ma = None if (ia is None or ia.all_one) else ia.weights
            mb = None if (ib is None or ib.all_one) else ib.weights
            use_a = not ctx.audio_zero and not (ia is not None and ia.all_zero)
            use_b = not ctx.vasa_zero and not (ib is not None and ib.all_zero)
        # softmax over a single key is exactly 1: the ID attention is to_v(ID) broadcast
        v_id = ctx.vid.get(id(self))
        if v_id is None or v_id.shape[0] != id_tok.shape[0]:
            v_id = ops.gemm(id_tok, self.to_v.w())
        proc = self.processor
        if is_ip_processor(proc):
            sa, sb = _scale_value(proc.scale[0]), _scale_value(proc.scale[1])
            q = kv = vb = None
            if use_a and sa != 0.0:
                q = ops.gemm(n, self.to_q.w())
                kv = ctx.ipkv.get(id(self))                    # batched per call (UNet._batched_ctx_projections)
                if kv is None or kv.shape[0] != audio.shape[0]:
                    kv = ops.gemm(audio, ip_w_kv(proc, 0))
            if use_b and sb != 0.0:
                vb = ctx.ipvb.get(id(self))
                if vb is None or vb.shape[0] != vasa.shape[0]:
                    vb = ops.gemm(vasa, ip_w_v(proc, 1))
            comb = ops.ip_attn(v_id, M, self.heads, rows_per_ctx, S, q=q, kv=kv, nkeys=ctx.n_audio, vb=vb,
                               mask_a=ma, mask_b=mb, sa=sa, sb=sb)
        else:
            comb = ops.ip_attn(v_id, M, self.heads, rows_per_ctx, S)
        return ops.gemm(comb, self.to_out[0].w(), bias=self.to_out[0].b(), residual=x_res)


    # -- the fused form: norm2 -> cross attention (+ residual) -> norm3 in one kernel (acth_xattn), with to_q /
    # to_out folded into the per-context audio keys / values (acth_ip_fold). Returns (h', norm3(h')) or None
    # when the shape or processor is not one the fused kernel covers (the caller then runs the unfused ops).
    def run_cross_fused(self, ctx: Ctx, h, S, temporal: bool, norm2, norm3):
        M, C = h.shape
        proc = self.processor
        rows_per_ctx = ctx.F * S if temporal else S
        if (not FUSED_XATTN or C not in ops.XATTN_C or not is_ip_processor(proc) or len(proc.to_k_ip) < 2
                or rows_per_ctx % ops.XATTN_ROWS or M % rows_per_ctx or ctx.n_audio != 32 or C != self.heads * 64):
            return None
        if temporal:
            id_tok, audio, vasa = ctx.id_mean, ctx.audio_mean, ctx.vasa_mean
            ma = mb = None
            use_a, use_b = not ctx.audio_zero, not ctx.vasa_zero
        else:
            id_tok, audio, vasa = ctx.id_tok, ctx.audio_tok, ctx.vasa_tok
            ia, ib = ctx.mask(0, S), ctx.mask(1, S)
            ma = None if (ia is None or ia.all_one) else ia.weights
            mb = None if (ib is None or ib.all_one) else ib.weights
            use_a = not ctx.audio_zero and not (ia is not None and ia.all_zero)
            use_b = not ctx.vasa_zero and not (ib is not None and ib.all_zero)
        if id_tok.shape[0] != M // rows_per_ctx:
            return None
        sa, sb = _scale_value(proc.scale[0]), _scale_value(proc.scale[1])
        use_a, use_b = use_a and sa != 0.0, use_b and sb != 0.0
        v_id = ctx.vid.get(id(self))
        if v_id is None or v_id.shape[0] != id_tok.shape[0]:
            v_id = ops.gemm(id_tok, self.to_v.w())
        kv = vb = None
        if use_a:
            kv = ctx.ipkv.get(id(self))
            if kv is None or kv.shape[0] != audio.shape[0]:
                kv = ops.gemm(audio, ip_w_kv(proc, 0))
        if use_b:
            vb = ctx.ipvb.get(id(self))
            if vb is None or vb.shape[0] != vasa.shape[0]:
                vb = ops.gemm(vasa, ip_w_v(proc, 1))
        woT = self.to_out[0]._pk("wT", lambda: _bf(self.to_out[0].weight.t()))
        kp, vp, gb, base, vbw = ops.ip_fold(self.to_q.w(), woT, self.to_out[0].b(), v_id, kv=kv, vb=vb,
                                            heads=self.heads, norm2=norm2.gb())
        return ops.xattn(h, norm2.eps, None if norm3 is None else (*norm3.gb(), norm3.eps), base, heads=self.heads,
                         rows_per_ctx=rows_per_ctx, S=S, kp=kp, vp=vp, gb=gb, vbw=vbw, mask_a=ma, mask_b=mb, sa=sa, sb=sb)


class GEGLU(Packed):
    def __init__(self, dim_in, dim_out, bias=True):
        super().__init__()
        self.proj = Linear(dim_in, dim_out * 2, bias=bias)

    def packed(self):
        return self._pk("geglu", lambda: pack_geglu(self.proj.weight, self.proj.bias))


class FeedForward(Packed):
    def __init__(self, dim, dim_out=None, mult=4, dropout=0.0, activation_fn="geglu", final_dropout=False,
                 inner_dim=None, bias=True):
        super().__init__()
        inner_dim = int(dim * mult) if inner_dim is None else inner_dim
        dim_out = dim_out if dim_out is not None else dim
        self.net = nn.ModuleList([GEGLU(dim, inner_dim, bias=bias), nn.Dropout(dropout),
                                  Linear(inner_dim, dim_out, bias=bias)])

    def fusable(self, C: int) -> bool:
        out = self.net[2]
        return (FUSED_FFN and C in ops.FFN_FUSED_C and out.in_features == 4 * C and out.out_features == C
                and self.net[0].proj.in_features == C)

    def run(self, n, residual, mix=None, mix_alpha: float = 0.0):
        """net[2](GEGLU(n)) + residual [AlphaBlender with ``mix``]; one fused kernel at C = 320."""
        w, b = self.net[0].packed()
        if self.fusable(n.shape[1]):
            w2 = self._pk("w2perm", lambda: pack_ffn_w2(self.net[2].weight))
            return ops.geglu_ffn(n, w, b, w2, self.net[2].b(), residual=residual, mix=mix, mix_alpha=mix_alpha)
        g = ops.gemm(n, w, bias=b, act=ops.ACT_GEGLU)
        return ops.gemm(g, self.net[2].w(), bias=self.net[2].b(), residual=residual, mix=mix,
                        mix_alpha=mix_alpha)

    def ln_fusable(self, C: int) -> bool:
        return FUSED_FFN_LN and self.fusable(C)

    def run_ln(self, x, ln, mix=None, mix_alpha: float = 0.0, add=None, add_div: int = 1):
        """net[2](GEGLU(ln(x'))) + x' [AlphaBlender with ``mix``], x' = x [+ add[row // add_div]] -- the
        blocks' "norm -> ff -> + residual" (attention.py:330-343, 449-457); one kernel at C = 320."""
        # the fused kernel takes the row add only with add_div % 64 == 0 and not together with a mix operand
        # (acth_geglu_ffn): other shapes take the LayerNorm + two-GEMM path below
        if self.ln_fusable(x.shape[1]) and (add is None or (add_div % 64 == 0 and mix is None)):
            w, b = self.net[0].packed()
            w2 = self._pk("w2perm", lambda: pack_ffn_w2(self.net[2].weight))
            return ops.geglu_ffn(x, w, b, w2, self.net[2].b(), residual=x, mix=mix, mix_alpha=mix_alpha,
                                 ln=(*ln.gb(), ln.eps), add=add, add_div=add_div)
        if add is not None:
            xs = torch.empty_like(x)
            n = ops.layernorm(x, *ln.gb(), ln.eps, add=add, add_div=add_div, sum_out=xs)
            return self.run(n, xs, mix=mix, mix_alpha=mix_alpha)
        return self.run(ops.layernorm(x, *ln.gb(), ln.eps), x, mix=mix, mix_alpha=mix_alpha)


class BasicTransformerBlock(nn.Module):
    def __init__(self, dim, num_attention_heads, attention_head_dim, cross_attention_dim=None):
        super().__init__()
        self.norm1 = LayerNorm(dim, eps=1e-5)
        self.attn1 = Attention(dim, None, num_attention_heads, attention_head_dim)
        self.norm2 = LayerNorm(dim, eps=1e-5)
        self.attn2 = Attention(dim, cross_attention_dim, num_attention_heads, attention_head_dim)
        self.norm3 = LayerNorm(dim, eps=1e-5)
        self.ff = FeedForward(dim, activation_fn="geglu")

    def run(self, ctx: Ctx, h, S):
        return self.run_after_attn1(ctx, self.run_attn1(ctx, h, S), S)

    def run_attn1(self, ctx: Ctx, h, S):
        """attn1(norm1(h)) + h: the part that reads no IP-adapter (audio / VASA / ID) input."""
        n = ops.layernorm(h, *self.norm1.gb(), self.norm1.eps)
        return self.attn1.run_self(ctx, n, h, S, temporal=False)

    def run_after_attn1(self, ctx: Ctx, h, S):
        ln3 = self.ff.ln_fusable(h.shape[1])
        fused = self.attn2.run_cross_fused(ctx, h, S, False, self.norm2, None if ln3 else self.norm3)
        if fused is not None:
            h, n = fused
            return self.ff.run_ln(h, self.norm3) if n is None else self.ff.run(n, h)
        n = ops.layernorm(h, *self.norm2.gb(), self.norm2.eps)
        h = self.attn2.run_cross(ctx, n, h, S, temporal=False)
        del n
        return self.ff.run_ln(h, self.norm3)


class TemporalBasicTransformerBlock(nn.Module):
    def __init__(self, dim, time_mix_inner_dim, num_attention_heads, attention_head_dim, cross_attention_dim=None):
        super().__init__()
        self.is_res = dim == time_mix_inner_dim
        self.norm_in = LayerNorm(dim)
        self.ff_in = FeedForward(dim, dim_out=time_mix_inner_dim, activation_fn="geglu")
        self.norm1 = LayerNorm(time_mix_inner_dim)
        self.attn1 = Attention(time_mix_inner_dim, None, num_attention_heads, attention_head_dim)
        self.norm2 = LayerNorm(time_mix_inner_dim)
        self.attn2 = Attention(time_mix_inner_dim, cross_attention_dim, num_attention_heads, attention_head_dim)
        self.norm3 = LayerNorm(time_mix_inner_dim)
        self.ff = FeedForward(time_mix_inner_dim, activation_fn="geglu")

    def run(self, ctx: Ctx, h_spatial, pos_emb, S, mix_alpha):
        """x = h + pos_emb[frame]; temporal block; AlphaBlender(h, x_temporal) fused in the last GEMM."""
        if not self.is_res:
            raise NotImplementedError("time_mix_inner_dim != dim is not used by the SVD UNet")
        t = self.ff_in.run_ln(h_spatial, self.norm_in, add=pos_emb, add_div=S)
        n = ops.layernorm(t, *self.norm1.gb(), self.norm1.eps)
        t = self.attn1.run_self(ctx, n, t, S, temporal=True)
        ln3 = self.ff.ln_fusable(t.shape[1])
        fused = self.attn2.run_cross_fused(ctx, t, S, True, self.norm2, None if ln3 else self.norm3)
        if fused is not None:
            t, n = fused
            if n is None:
                return self.ff.run_ln(t, self.norm3, mix=h_spatial, mix_alpha=mix_alpha)
            return self.ff.run(n, t, mix=h_spatial, mix_alpha=mix_alpha)
        n = ops.layernorm(t, *self.norm2.gb(), self.norm2.eps, out=n)
        t = self.attn2.run_cross(ctx, n, t, S, temporal=True)
        del n
        return self.ff.run_ln(t, self.norm3, mix=h_spatial, mix_alpha=mix_alpha)


# ------------------------------------------------------------------------------------------
class SS2D_Unit(nn.Module):
    """Parameters of one bidirectional selective-scan unit (mamba_layer.py:1394-1553)."""

    def __init__(self, d_model, d_cond, cond_size=0, d_state=16, d_conv=3, expand=2, dt_rank="auto",
                 dt_min=0.001, dt_max=0.1, dt_init="random", dt_scale=1.0, dt_init_floor=1e-4, dropout=0.,
                 conv_bias=True, bias=False, device=None, dtype=None, size=8, scan_type='scan',
                 num_direction=8, **kwargs):
        super().__init__()
        if d_state != 16:
            raise ValueError("the HIP scan is specialised for d_state == 16 (the reference's setting)")
        if num_direction != 2 or scan_type != "sweep":
            raise ValueError("ACTalker v10 uses scan_type='sweep', num_direction=2")
        self.d_model, self.d_state, self.d_conv, self.expand = d_model, d_state, d_conv, expand
        self.d_inner = int(expand * d_model)
        self.dt_rank = math.ceil(d_model / 16) if dt_rank == "auto" else dt_rank
        self.d_cond = d_cond
        self.num_direction = num_direction
        self.scan_type = scan_type
        K, Din, R, N = num_direction, self.d_inner, self.dt_rank, d_state
        self.x_proj_weight = nn.Parameter(torch.empty(K, R + 2 * N, Din))
        self.dt_projs_weight = nn.Parameter(torch.empty(K, Din, R))
        self.dt_projs_bias = nn.Parameter(torch.empty(K, Din))
        a = torch.arange(1, N + 1, dtype=torch.float32).repeat(K * Din, 1)
        self.A_logs = nn.Parameter(torch.log(a))
        self.Ds = nn.Parameter(torch.ones(K * Din))
        self._init_dt(dt_scale, dt_min, dt_max, dt_init_floor)
        nn.init.uniform_(self.x_proj_weight, -1.0 / math.sqrt(Din), 1.0 / math.sqrt(Din))

    def _init_dt(self, dt_scale, dt_min, dt_max, floor):
        std = self.dt_rank ** -0.5 * dt_scale
        with torch.no_grad():
            nn.init.uniform_(self.dt_projs_weight, -std, std)
            dt = torch.exp(torch.rand(self.dt_projs_bias.shape) * (math.log(dt_max) - math.log(dt_min))
                           + math.log(dt_min)).clamp(min=floor)
            self.dt_projs_bias.copy_(dt + torch.log(-torch.expm1(-dt)))

    def packed(self):
        c = self.__dict__.setdefault("_acth_cache", {})
        key = ("p", ops.act_dtype())
        if key not in c:
            with torch.no_grad():
                K, R, Din = self.num_direction, self.dt_rank, self.d_inner
                R4 = (R + 3) // 4 * 4
                xw = self.x_proj_weight.detach()
                if R4 != R:      # [dt (R) | 0 (R4 - R) | B | C] per direction: 8-byte aligned bf16 rows
                    pad = torch.zeros((K, R4 - R, Din), device=xw.device, dtype=xw.dtype)
                    xw = torch.cat([xw[:, :R], pad, xw[:, R:]], dim=1)
                c[key] = dict(
                    xproj=_bf(self.x_proj_weight.reshape(-1, self.d_inner)),
                    xproj_pad=_bf(xw.reshape(-1, Din)),
                    dt_w=_f32(self.dt_projs_weight),
                    dt_b=_f32(self.dt_projs_bias),
                    A_log=_f32(self.A_logs),
                    D=_f32(self.Ds))
        return c[key]

    def _acth_invalidate(self):
        self.__dict__["_acth_cache"] = {}

    # x_proj output rows in bf16 (the reference's x_dbl dtype, mamba_layer.py:1521), scanned by the paired-lane
    # kernel's bf16-row instantiation by default (scan_quad_kernel only with ACTH_SCAN_QUAD=1); False: fp32 rows
    # (ACTH_SCAN_XDBL_F32=1)
    acth_xdbl_bf16 = os.environ.get("ACTH_SCAN_XDBL_F32", "0") != "1"

    def scan_args(self, u, nb, L, n_keep):
        """x_proj of u (the GEMM ahead of the scan) and the scan's arguments."""
        p = self.packed()
        if self.acth_xdbl_bf16:
            xdbl = ops.gemm(u, p["xproj_pad"])
        else:
            xdbl = ops.gemm(u, p["xproj"], out_f32=True)
        return dict(u=u, xdbl=xdbl, dt_w=p["dt_w"], dt_b=p["dt_b"], A_log=p["A_log"], Dskip=p["D"], nb=nb, L=L,
                    R=self.dt_rank, n_keep=n_keep)

    def scan(self, u, nb, L, n_keep):
        """u: (nb*L, d_inner) bf16 token-major sequence -> (y_dir0, y_dir1) for l < n_keep."""
        return ops.selective_scan(**self.scan_args(u, nb, L, n_keep))


class SS2D_cond_v10(nn.Module):
    def __init__(self, d_model, d_cond, cond_size=0, d_state=16, d_conv=3, expand=2, dt_rank="auto",
                 dt_min=0.001, dt_max=0.1, dt_init="random", dt_scale=1.0, dt_init_floor=1e-4, dropout=0.,
                 conv_bias=True, bias=False, device=None, dtype=None, size=8, scan_type='scan', num_direction=8,
                 **kwargs):
        super().__init__()
        args = (d_model, d_cond, cond_size, d_state, d_conv, expand, dt_rank, dt_min, dt_max, dt_init, dt_scale,
                dt_init_floor, dropout, conv_bias, bias, device, dtype, size, scan_type, num_direction)
        self.audio_unit = SS2D_Unit(*args)
        self.exp_unit = SS2D_Unit(*args)
        self.d_model, self.d_state, self.d_conv, self.expand = d_model, d_state, d_conv, expand
        self.d_inner = int(expand * d_model)
        self.dt_rank = math.ceil(d_model / 16) if dt_rank == "auto" else dt_rank
        self.d_cond = d_cond
        self.audio_proj = Linear(d_cond, self.d_inner, bias=bias)
        self.exp_proj = Linear(d_cond, self.d_inner, bias=bias)
        self.id_proj = Linear(d_cond, self.d_inner, bias=bias)
        self.in_proj1 = Linear(d_model, self.d_inner, bias=bias)
        self.in_proj2 = Linear(d_model, self.d_inner, bias=bias)
        self.act1 = nn.SiLU()
        self.act2 = nn.SiLU()
        self.num_direction = num_direction
        self.out_norm = LayerNorm(self.d_inner)
        self.out_proj = Linear(self.d_inner, d_model, bias=bias)
        self.scan_type = scan_type

    # both branches' scans in one launch (acth_selective_scan2); False: one launch per branch
    acth_pair_scan = True

    def _branch(self, ctx: Ctx, h, S, info, in_proj: Linear, cond_proj: Linear, cond_tok, n_cond, unit,
                defer=False):
        """One masked branch: select tokens -> [tokens, ID, cond] -> bidirectional scan. defer: return the
        scan's arguments under "scan" instead of running it (run() pairs the two branches)."""
        BF, Din = ctx.BF, self.d_inner
        n_sel = S if info is None else info.n_sel
        identity = info is None or info.identity
        if n_sel == 0:
            # nothing selected: the scan runs on [ID, cond] only and its output is discarded
            return dict(mode=0, x=ops.gemm(h, in_proj.w()))
        L = n_sel + 1 + n_cond
        u = torch.empty((BF * L, Din), device=h.device, dtype=ops.act_dtype())
        br = {}
        if identity:
            ops.gemm(h, in_proj.w(), out=u, orow=(S, L, 0))
            br["mode"] = 1
        else:
            xz = ops.gemm(h, in_proj.w())
            ops.gather_rows(xz, info.idx, BF, S, u, L)
            br.update(mode=2, x=xz, pos=info.pos)
        uv = u.view(BF, L, Din)
        idp = ctx.mamba_proj.get(id(self.id_proj))            # batched per call (UNet._batched_ctx_projections)
        if idp is not None and idp.shape[0] == BF:
            uv[:, n_sel].copy_(idp)
        else:
            ops.gemm(ctx.id_tok, self.id_proj.w(), act=ops.ACT_SILU, out=u, orow=(1, L, n_sel))
        cp = ctx.mamba_proj.get(id(cond_proj))
        if cp is not None and cp.shape[0] == cond_tok.shape[0]:
            uv[:, n_sel + 1:n_sel + 1 + n_cond].copy_(cp.view(BF, n_cond, Din))
        else:
            ops.gemm(cond_tok, cond_proj.w(), act=ops.ACT_SILU, out=u, orow=(n_cond, L, n_sel + 1))
        br["L"] = n_sel          # scan outputs hold n_sel rows per batch element
        if defer:
            br["scan"] = unit.scan_args(u, BF, L, n_sel)
        else:
            br["y0"], br["y1"] = unit.scan(u, BF, L, n_sel)
        return br

    def run(self, ctx: Ctx, h, S):
        ia, ie = ctx.mask(0, S), ctx.mask(1, S)
        pair = self.acth_pair_scan
        ba = self._branch(ctx, h, S, ia, self.in_proj1, self.audio_proj, ctx.audio_tok, ctx.n_audio,
                          self.audio_unit, defer=pair)
        be = self._branch(ctx, h, S, ie, self.in_proj2, self.exp_proj, ctx.vasa_tok, 1, self.exp_unit,
                          defer=pair)
        if "scan" in ba and "scan" in be:
            (ba["y0"], ba["y1"]), (be["y0"], be["y1"]) = ops.selective_scan2(ba.pop("scan"), be.pop("scan"))
        for br in (ba, be):
            if "scan" in br:
                br["y0"], br["y1"] = ops.selective_scan(**br.pop("scan"))
        g, b = self.out_norm.gb()
        y = ops.mamba_combine_ln(ba, be, g, b, self.out_norm.eps, h.shape[0], S, self.d_inner)
        return ops.gemm(y, self.out_proj.w())


# ------------------------------------------------------------------------------------------
class TransformerSpatioTemporalModel(nn.Module):
    """Plain spatio-temporal transformer (mid block), TransformerSTmodel.py:200-421."""

    has_mamba = False

    def __init__(self, num_attention_heads=16, attention_head_dim=88, in_channels=320, out_channels=None,
                 num_layers=1, cross_attention_dim=None):
        super().__init__()
        self.num_attention_heads = num_attention_heads
        self.attention_head_dim = attention_head_dim
        if attention_head_dim != 64:
            raise ValueError("the HIP attention kernels are specialised for head_dim 64 (SVD's value)")
        inner_dim = num_attention_heads * attention_head_dim
        self.inner_dim = inner_dim
        self.in_channels = in_channels
        self.norm = GroupNorm(num_groups=32, num_channels=in_channels, eps=1e-6)
        self.proj_in = Linear(in_channels, inner_dim)
        self.transformer_blocks = nn.ModuleList([
            BasicTransformerBlock(inner_dim, num_attention_heads, attention_head_dim,
                                  cross_attention_dim=cross_attention_dim) for _ in range(num_layers)])
        self._build_mamba(in_channels, cross_attention_dim, num_layers)
        self.temporal_transformer_blocks = nn.ModuleList([
            TemporalBasicTransformerBlock(inner_dim, inner_dim, num_attention_heads, attention_head_dim,
                                          cross_attention_dim=cross_attention_dim) for _ in range(num_layers)])
        time_embed_dim = in_channels * 4
        self.time_pos_embed = TimestepEmbedding(in_channels, time_embed_dim, out_dim=in_channels)
        self.time_proj = Timesteps(in_channels, True, 0)
        self.time_mixer = AlphaBlender(alpha=0.5, merge_strategy="learned_with_images")
        self.out_channels = in_channels if out_channels is None else out_channels
        self.proj_out = Linear(inner_dim, in_channels)

    def _build_mamba(self, in_channels, cross_attention_dim, num_layers):
        pass

    def _pos_emb(self, ctx: Ctx):
        """time_pos_embed(Timesteps(C)(frame index)) for frames 0..F-1 of every batch element: (BF, C).
        A function of the weights and (B, F) only -- the same in every UNet call of a run -- so it is
        cached, keyed on the TimestepEmbedding tensors' versions (two 84-row GEMMs per transformer and
        call otherwise)."""
        te = self.time_pos_embed
        tensors = [t for t in (te.linear_1.weight, te.linear_1.bias, te.linear_2.weight, te.linear_2.bias)
                   if t is not None]

        def make():
            fidx = torch.arange(ctx.F, device=ctx.device, dtype=torch.float32).repeat(ctx.B)
            return te.run(self.time_proj.run(fidx))
        return _versioned_pack(self, ("pos_emb", ctx.B, ctx.F, str(ctx.device)), tensors, make)

    def run(self, ctx: Ctx, x, H, W, prefix=None):
        """``prefix`` = (ctx_u, expand): ``x`` holds only the batch elements of ``ctx_u`` (the distinct
        CFG-prefix inputs, see UNet.forward_tokens); everything before the first IP-adapter input (GroupNorm,
        proj_in, the first block's attn1) runs on them, then ``expand`` copies the rows out to ``ctx``'s
        full batch."""
        S = H * W
        g, b = self.norm.gb()
        cin = ctx if prefix is None else prefix[0]
        n = ops.groupnorm(x, g, b, self.norm.eps, S)
        h = ops.gemm(n, self.proj_in.w(), bias=self.proj_in.b())
        del n
        if prefix is not None:
            h = prefix[1](self.transformer_blocks[0].run_attn1(cin, h, S))
            x = prefix[1](x)
        pos = self._pos_emb(ctx)
        alpha = self.time_mixer.alpha()
        for i, (blk, tblk) in enumerate(zip(self.transformer_blocks, self.temporal_transformer_blocks)):
            h = blk.run_after_attn1(ctx, h, S) if (prefix is not None and i == 0) else blk.run(ctx, h, S)
            if self.has_mamba:
                h = self.mamba_blocks[i].run(ctx, h, S)
            h = tblk.run(ctx, h, pos, S, alpha)
        return ops.gemm(h, self.proj_out.w(), bias=self.proj_out.b(), residual=x)


class TransformerSpatioTemporalModel_new_mambaID_v10_two_ip(TransformerSpatioTemporalModel):
    """Spatio-temporal transformer with the masked dual-Mamba block, TransformerSTmodel.py:3908-4155."""

    has_mamba = True

    def _build_mamba(self, in_channels, cross_attention_dim, num_layers):
        self.mamba_blocks = nn.ModuleList([
            SS2D_cond_v10(d_model=in_channels, d_cond=cross_attention_dim, cond_size=32, dropout=0.1, d_state=16,
                          size=int(72 / (in_channels / 320)), scan_type='sweep', num_direction=2)
            for _ in range(num_layers)])


# ------------------------------------------------------------------------------------------
class UNetMidBlockSpatioTemporal(nn.Module):
    def __init__(self, in_channels, temb_channels, num_layers=1, transformer_layers_per_block=1,
                 num_attention_heads=1, cross_attention_dim=1280):
        super().__init__()
        self.has_cross_attention = True
        self.num_attention_heads = num_attention_heads
        if isinstance(transformer_layers_per_block, int):
            transformer_layers_per_block = [transformer_layers_per_block] * num_layers
        resnets = [SpatioTemporalResBlock(in_channels, in_channels, temb_channels, eps=1e-5)]
        attentions = []
        for i in range(num_layers):
            attentions.append(TransformerSpatioTemporalModel(
                num_attention_heads, in_channels // num_attention_heads, in_channels=in_channels,
                num_layers=transformer_layers_per_block[i], cross_attention_dim=cross_attention_dim))
            resnets.append(SpatioTemporalResBlock(in_channels, in_channels, temb_channels, eps=1e-5))
        self.attentions = nn.ModuleList(attentions)
        self.resnets = nn.ModuleList(resnets)

    def run(self, ctx, h, H, W):
        h = self.resnets[0].run(ctx, h, H, W)
        for attn, res in zip(self.attentions, self.resnets[1:]):
            h = attn.run(ctx, h, H, W)
            h = res.run(ctx, h, H, W)
        return h


class DownBlockSpatioTemporal(nn.Module):
    def __init__(self, in_channels, out_channels, temb_channels, num_layers=1, add_downsample=True):
        super().__init__()
        self.resnets = nn.ModuleList([
            SpatioTemporalResBlock(in_channels if i == 0 else out_channels, out_channels, temb_channels, eps=1e-5)
            for i in range(num_layers)])
        self.downsamplers = (nn.ModuleList([Downsample2D(out_channels, use_conv=True, out_channels=out_channels,
                                                         name="op")]) if add_downsample else None)

    def run(self, ctx, h, H, W):
        outs = []
        for res in self.resnets:
            h = res.run(ctx, h, H, W)
            outs.append(h)
        if self.downsamplers is not None:
            h = self.downsamplers[0].run(ctx, h, H, W)
            H, W = (H + 1) // 2, (W + 1) // 2
            outs.append(h)
        return h, outs, H, W


class CrossAttnDownBlockSpatioTemporal(nn.Module):
    def __init__(self, in_channels, out_channels, temb_channels, num_layers=1, transformer_layers_per_block=1,
                 num_attention_heads=1, cross_attention_dim=1280, add_downsample=True, attn_cls=None):
        super().__init__()
        self.has_cross_attention = True
        self.num_attention_heads = num_attention_heads
        if isinstance(transformer_layers_per_block, int):
            transformer_layers_per_block = [transformer_layers_per_block] * num_layers
        cls = attn_cls if attn_cls is not None else TransformerSpatioTemporalModel
        resnets, attentions = [], []
        for i in range(num_layers):
            resnets.append(SpatioTemporalResBlock(in_channels if i == 0 else out_channels, out_channels,
                                                  temb_channels, eps=1e-6))
            attentions.append(cls(num_attention_heads, out_channels // num_attention_heads, in_channels=out_channels,
                                  num_layers=transformer_layers_per_block[i], cross_attention_dim=cross_attention_dim))
        self.attentions = nn.ModuleList(attentions)
        self.resnets = nn.ModuleList(resnets)
        self.downsamplers = (nn.ModuleList([Downsample2D(out_channels, use_conv=True, out_channels=out_channels,
                                                         padding=1, name="op")]) if add_downsample else None)

    def run(self, ctx, h, H, W, prefix=None):
        """``prefix``: see TransformerSpatioTemporalModel.run -- ``h`` then holds the distinct-prefix batch
        and the first resnet runs on it too."""
        outs = []
        for i, (res, attn) in enumerate(zip(self.resnets, self.attentions)):
            if prefix is not None and i == 0:
                h = res.run(prefix[0], h, H, W)
                h = attn.run(ctx, h, H, W, prefix=prefix)
            else:
                h = res.run(ctx, h, H, W)
                h = attn.run(ctx, h, H, W)
            outs.append(h)
        if self.downsamplers is not None:
            h = self.downsamplers[0].run(ctx, h, H, W)
            H, W = (H + 1) // 2, (W + 1) // 2
            outs.append(h)
        return h, outs, H, W


class UpBlockSpatioTemporal(nn.Module):
    def __init__(self, in_channels, prev_output_channel, out_channels, temb_channels, resolution_idx=None,
                 num_layers=1, resnet_eps=1e-6, add_upsample=True):
        super().__init__()
        resnets = []
        for i in range(num_layers):
            res_skip = in_channels if (i == num_layers - 1) else out_channels
            res_in = prev_output_channel if i == 0 else out_channels
            resnets.append(SpatioTemporalResBlock(res_in + res_skip, out_channels, temb_channels, eps=resnet_eps))
        self.resnets = nn.ModuleList(resnets)
        self.upsamplers = (nn.ModuleList([Upsample2D(out_channels, use_conv=True, out_channels=out_channels)])
                           if add_upsample else None)
        self.resolution_idx = resolution_idx

    def run(self, ctx, h, skips: List[torch.Tensor], H, W):
        for res in self.resnets:
            skip = skips.pop()
            h = res.run(ctx, h, H, W, x2=skip)
        if self.upsamplers is not None:
            h = self.upsamplers[0].run(ctx, h, H, W)
            H, W = 2 * H, 2 * W
        return h, H, W


class CrossAttnUpBlockSpatioTemporal(nn.Module):
    def __init__(self, in_channels, out_channels, prev_output_channel, temb_channels, resolution_idx=None,
                 num_layers=1, transformer_layers_per_block=1, resnet_eps=1e-6, num_attention_heads=1,
                 cross_attention_dim=1280, add_upsample=True, attn_cls=None):
        super().__init__()
        self.has_cross_attention = True
        self.num_attention_heads = num_attention_heads
        if isinstance(transformer_layers_per_block, int):
            transformer_layers_per_block = [transformer_layers_per_block] * num_layers
        cls = attn_cls if attn_cls is not None else TransformerSpatioTemporalModel
        resnets, attentions = [], []
        for i in range(num_layers):
            res_skip = in_channels if (i == num_layers - 1) else out_channels
            res_in = prev_output_channel if i == 0 else out_channels
            resnets.append(SpatioTemporalResBlock(res_in + res_skip, out_channels, temb_channels, eps=resnet_eps))
            attentions.append(cls(num_attention_heads, out_channels // num_attention_heads, in_channels=out_channels,
                                  num_layers=transformer_layers_per_block[i], cross_attention_dim=cross_attention_dim))
        self.attentions = nn.ModuleList(attentions)
        self.resnets = nn.ModuleList(resnets)
        self.upsamplers = (nn.ModuleList([Upsample2D(out_channels, use_conv=True, out_channels=out_channels)])
                           if add_upsample else None)
        self.resolution_idx = resolution_idx

    def run(self, ctx, h, skips: List[torch.Tensor], H, W):
        for res, attn in zip(self.resnets, self.attentions):
            skip = skips.pop()
            h = res.run(ctx, h, H, W, x2=skip)
            h = attn.run(ctx, h, H, W)
        if self.upsamplers is not None:
            h = self.upsamplers[0].run(ctx, h, H, W)
            H, W = 2 * H, 2 * W
        return h, H, W
