"""AutoencoderKLTemporalDecoder on HIP: the ref-image encode before the denoising loop and the
temporal decode after it.

Reference call sites: ``vae.encode(ref_image).latent_dist.mean`` and ``_encode_vae_image``
(src/pipelines/pipeline_svd_audio_adapter_motionexp_idembed_vasa_two_ip.py:235-249, :520-536) and
``decode_latents`` (:264-290, called at :766) on diffusers 0.29.2's AutoencoderKLTemporalDecoder
(Inference.py:41-44; diffusers is not installed here, its published 0.29.2 structure is restated:
``Encoder`` with DownEncoderBlock2D / UNetMidBlock2D, ``quant_conv``, ``TemporalDecoder`` with
MidBlockTemporalDecoder / UpBlockTemporalDecoder of SpatioTemporalResBlocks, ``time_conv_out``).
Module and parameter names follow diffusers so an SVD ``vae`` state dict loads with strict=True.

MI355X mapping (token-major NHWC rows, bf16 activations, fp32 accumulation):
  * 3x3 convs with Cin % 64 == 0 -> MFMA implicit GEMM (acth_gemm amode 1, nearest-x2 upsample
    fused into the loader); the narrow conv_in (Cin 3 / 4), conv_out (Cout 3) and time_conv_out
    (3 -> 3) and the encoder's bottom/right-padded stride-2 downsamplers -> acth_conv_direct;
  * Conv3d (3,1,1) -> acth_gemm amode 2 when the window fits one launch; at full resolution
    (F*H*W >= 2^22 rows) the same contraction as two dense launches over a frame-padded copy
    of the GroupNorm output: [x(f-1) | x(f)] . [W0 | W1]^T, then + x(f+1) . W2^T in place;
  * GroupNorm(+SiLU) -> acth_groupnorm (temporal statistics span all frames of the window);
  * mid-block attention (1 head of 512) -> materialised per frame: S^T-free scores GEMM (fp32),
    acth_softmax_rows, and one P . V' GEMM whose V' = n . (W_o W_v)^T and bias W_o b_v + b_o fold
    the value and output projections (rows of P sum to 1), with the residual in its epilogue.
Launches are split over frames / rows to keep every launch below the kernels' 2^22-row and
2^31-byte operand limits.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import torch
import torch.nn as nn

from . import ops
from .modules import (Conv2d, Conv3d, GroupNorm, Linear, Packed, ResnetBlock2D, SpatioTemporalResBlock, _bf, _f32,
                      pack_conv3x3)

MAXROWS = (1 << 22) - 1
MAXBYTES = (1 << 31) - 1


# ------------------------------------------------------------------------------------------ launch helpers
def _conv3x3(x, w, b, nfr, H, W, *, stride=1, upsample=False, residual=None, act=ops.ACT_NONE):
    if upsample:
        Ho, Wo = 2 * H, 2 * W
    else:
        Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    ld = x.stride(0)
    per = max(1, min(MAXROWS // (Ho * Wo), MAXBYTES // (H * W * ld * 2)))
    out = torch.empty((nfr * Ho * Wo, w.shape[0]), device=x.device, dtype=torch.bfloat16)
    for f0 in range(0, nfr, per):
        n = min(per, nfr - f0)
        ri, ro = slice(f0 * H * W, (f0 + n) * H * W), slice(f0 * Ho * Wo, (f0 + n) * Ho * Wo)
        ops.conv3x3(x[ri], w, n, H, W, stride=stride, upsample=upsample, bias=b,
                    residual=None if residual is None else residual[ro], act=act, out=out[ro])
    return out


def _gemm_rows(a, w, *, bias=None, out_f32=False):
    M = a.shape[0]
    per = max(1, min(MAXROWS, MAXBYTES // (a.stride(0) * 2)))
    out = torch.empty((M, w.shape[0]), device=a.device, dtype=torch.float32 if out_f32 else torch.bfloat16)
    for r0 in range(0, M, per):
        r = slice(r0, min(M, r0 + per))
        ops.gemm(a[r], w, bias=bias, out=out[r], out_f32=out_f32)
    return out


class _FramePadded:
    """(B*(F+2)*S, C) buffer whose first and last frame of each batch are zero: the GroupNorm writes
    the middle F frames, the temporal contraction reads frame f-1 / f / f+1 as plain row ranges."""

    def __init__(self, B, F, S, C, device):
        self.B, self.F, self.S = B, F, S
        self.buf = torch.empty((B * (F + 2) * S, C), device=device, dtype=torch.bfloat16)
        for b in range(B):
            base = b * (F + 2) * S
            self.buf[base:base + S].zero_()
            self.buf[base + (F + 1) * S:base + (F + 2) * S].zero_()

    def body(self, b):
        base = b * (self.F + 2) * self.S
        return self.buf[base + self.S:base + (self.F + 1) * self.S]


def _temporal_conv(src: _FramePadded, wt, bias, *, residual=None, mix=None, mix_alpha=0.0, force_split=False):
    """Conv3d (3,1,1), pad (1,0,0) over frames on rows (b, f, s); wt packed (Cout, 3*Cin)."""
    B, F, S = src.B, src.F, src.S
    Cout, K = wt.shape
    Cin = K // 3
    FS = F * S
    out = torch.empty((B * FS, Cout), device=src.buf.device, dtype=torch.bfloat16)
    fits = FS <= MAXROWS and FS * src.buf.stride(0) * 2 <= MAXBYTES
    for b in range(B):
        ob = slice(b * FS, (b + 1) * FS)
        if fits and not force_split:
            ops.gemm(src.body(b), wt, temporal=dict(F=F, S=S), bias=bias,
                     residual=None if residual is None else residual[ob], mix=None if mix is None else mix[ob],
                     mix_alpha=mix_alpha, out=out[ob])
            continue
        base = b * (F + 2) * S
        xp = src.buf
        per = max(1, min(MAXROWS, MAXBYTES // (xp.stride(0) * 2)))
        for r0 in range(0, FS, per):
            m = min(per, FS - r0)
            o = out[b * FS + r0:b * FS + r0 + m]
            a0 = xp[base + r0:base + r0 + m]                       # frame f-1 (padded index f)
            a1 = xp[base + S + r0:base + S + r0 + m]               # frame f
            a2 = xp[base + 2 * S + r0:base + 2 * S + r0 + m]       # frame f+1
            res = None if residual is None else residual[b * FS + r0:b * FS + r0 + m]
            mx = None if mix is None else mix[b * FS + r0:b * FS + r0 + m]
            ops.gemm(a0, wt[:, :2 * Cin], a2=a1, k1=Cin, bias=bias, residual=res, out=o)
            ops.gemm(a2, wt[:, 2 * Cin:], residual=o, mix=mx, mix_alpha=mix_alpha, out=o)
    return out


# ------------------------------------------------------------------------------------------ blocks
def _resnet2d(blk: ResnetBlock2D, x, nfr, H, W):
    """diffusers ResnetBlock2D without time embedding (VAE), output_scale_factor 1."""
    S = H * W
    g1, b1 = blk.norm1.gb()
    n1 = ops.groupnorm(x, g1, b1, blk.norm1.eps, S, silu=True)
    h = _conv3x3(n1, blk.conv1.w3(), blk.conv1.b(), nfr, H, W)
    del n1
    g2, b2 = blk.norm2.gb()
    n2 = ops.groupnorm(h, g2, b2, blk.norm2.eps, S, silu=True)
    del h
    sc = x if blk.conv_shortcut is None else _gemm_rows(x, blk.conv_shortcut.w1(), bias=blk.conv_shortcut.b())
    return _conv3x3(n2, blk.conv2.w3(), blk.conv2.b(), nfr, H, W, residual=sc)


def _st_resblock(blk: SpatioTemporalResBlock, x, B, F, H, W, force_split=False):
    """diffusers SpatioTemporalResBlock (temb None): spatial ResnetBlock2D, TemporalResnetBlock over
    the F frames of each batch, AlphaBlender (learned, switch_spatial_to_temporal_mix)."""
    S = H * W
    hs = _resnet2d(blk.spatial_res_block, x, B * F, H, W)
    t = blk.temporal_res_block
    C = hs.shape[1]
    g1, b1 = t.norm1.gb()
    p1 = _FramePadded(B, F, S, C, hs.device)
    for b in range(B):
        ops.groupnorm(hs[b * F * S:(b + 1) * F * S], g1, b1, t.norm1.eps, F * S, silu=True, out=p1.body(b))
    h1 = _temporal_conv(p1, t.conv1.wt(), t.conv1.b(), force_split=force_split)
    del p1
    g2, b2 = t.norm2.gb()
    p2 = _FramePadded(B, F, S, t.out_channels, hs.device)
    for b in range(B):
        ops.groupnorm(h1[b * F * S:(b + 1) * F * S], g2, b2, t.norm2.eps, F * S, silu=True, out=p2.body(b))
    del h1
    sc = hs if t.conv_shortcut is None else _gemm_rows(hs, t.conv_shortcut.w1(), bias=t.conv_shortcut.b())
    return _temporal_conv(p2, t.conv2.wt(), t.conv2.b(), residual=sc, mix=hs, mix_alpha=blk.time_mixer.alpha(),
                          force_split=force_split)


class Attention(Packed):
    """diffusers Attention as the VAE mid blocks build it: group_norm, 1 head of ``dim_head`` = C,
    q/k/v/out with bias, residual_connection, upcast_softmax (AttnProcessor2_0 on 4-D input)."""

    def __init__(self, query_dim, heads=1, dim_head=512, eps=1e-6, norm_num_groups=32, bias=True):
        super().__init__()
        inner = heads * dim_head
        self.heads, self.dim_head = heads, dim_head
        self.scale = dim_head ** -0.5
        self.group_norm = GroupNorm(norm_num_groups, query_dim, eps=eps, affine=True)
        self.to_q = Linear(query_dim, inner, bias=bias)
        self.to_k = Linear(query_dim, inner, bias=bias)
        self.to_v = Linear(query_dim, inner, bias=bias)
        self.to_out = nn.ModuleList([Linear(inner, query_dim, bias=True), nn.Dropout(0.0)])

    def _packs(self):
        def f():
            wq, wk, wv, wo = (m.weight.detach().float() for m in (self.to_q, self.to_k, self.to_v, self.to_out[0]))
            z = lambda m: m.bias.detach().float() if m.bias is not None else torch.zeros(m.out_features,  # noqa: E731
                                                                                         device=m.weight.device)
            bqk = torch.cat([z(self.to_q), z(self.to_k)])
            w_ov = wo @ wv                                   # V' = n (W_o W_v)^T
            b_o = self.to_out[0].bias.detach().float() + wo @ z(self.to_v)
            return _bf(torch.cat([wq, wk], 0)), bqk.contiguous(), _bf(w_ov), b_o.contiguous()
        return self._pk("packs", f)

    def run(self, x, nfr, S):
        if self.heads != 1:
            raise ValueError("VAE attention: the HIP path implements the single-head (dim_head = C) mid block")
        C = x.shape[1]
        w_qk, b_qk, w_ov, b_o = self._packs()
        g, b = self.group_norm.gb()
        n = ops.groupnorm(x, g, b, self.group_norm.eps, S)
        qk = _gemm_rows(n, w_qk, bias=b_qk)
        out = torch.empty_like(x)
        scores = torch.empty((S, S), device=x.device, dtype=torch.float32)
        P = torch.empty((S, S), device=x.device, dtype=torch.bfloat16)
        for f in range(nfr):
            r = slice(f * S, (f + 1) * S)
            ops.gemm(qk[r, :C], qk[r, C:], out=scores, out_f32=True)
            ops.softmax_rows(scores, self.scale, out=P)
            vt = ops.gemm(w_ov, n[r])                       # (C, S) = V'^T
            ops.gemm(P, vt, bias=b_o, residual=x[r], out=out[r])
        return out


# ------------------------------------------------------------------------------------------ decoder
class MidBlockTemporalDecoder(nn.Module):
    def __init__(self, in_channels, out_channels, attention_head_dim=512, num_layers=1):
        super().__init__()
        self.resnets = nn.ModuleList([
            SpatioTemporalResBlock(in_channels if i == 0 else out_channels, out_channels, temb_channels=None,
                                   eps=1e-6, temporal_eps=1e-5, merge_factor=0.0, merge_strategy="learned",
                                   switch_spatial_to_temporal_mix=True) for i in range(num_layers)])
        self.attentions = nn.ModuleList([Attention(in_channels, heads=in_channels // attention_head_dim,
                                                   dim_head=attention_head_dim, eps=1e-6)])


class Upsample2D(nn.Module):
    def __init__(self, channels, use_conv=True, out_channels=None):
        super().__init__()
        self.conv = Conv2d(channels, out_channels or channels, 3, padding=1)


class UpBlockTemporalDecoder(nn.Module):
    def __init__(self, in_channels, out_channels, num_layers=1, add_upsample=True):
        super().__init__()
        self.resnets = nn.ModuleList([
            SpatioTemporalResBlock(in_channels if i == 0 else out_channels, out_channels, temb_channels=None,
                                   eps=1e-6, temporal_eps=1e-5, merge_factor=0.0, merge_strategy="learned",
                                   switch_spatial_to_temporal_mix=True) for i in range(num_layers)])
        self.upsamplers = nn.ModuleList([Upsample2D(out_channels, out_channels=out_channels)]) if add_upsample else None


class DirectConv(Packed):
    """Mixin: fp32 (taps*Cin, Cout) pack for acth_conv_direct."""

    def wd(self):
        return self._pk("wd", lambda: ops.pack_conv_direct(self.weight))


class Conv2dD(nn.Conv2d, DirectConv):
    def b(self):
        return self._pk("b", lambda: _f32(self.bias))


class Conv3dD(nn.Conv3d, DirectConv):
    def b(self):
        return self._pk("b", lambda: _f32(self.bias))


class TemporalDecoder(nn.Module):
    def __init__(self, in_channels=4, out_channels=3, block_out_channels=(128, 256, 512, 512), layers_per_block=2):
        super().__init__()
        self.layers_per_block = layers_per_block
        self.conv_in = Conv2dD(in_channels, block_out_channels[-1], kernel_size=3, stride=1, padding=1)
        self.mid_block = MidBlockTemporalDecoder(block_out_channels[-1], block_out_channels[-1],
                                                 attention_head_dim=block_out_channels[-1], num_layers=layers_per_block)
        self.up_blocks = nn.ModuleList([])
        rev = list(reversed(block_out_channels))
        out_ch = rev[0]
        for i in range(len(block_out_channels)):
            prev, out_ch = out_ch, rev[i]
            self.up_blocks.append(UpBlockTemporalDecoder(prev, out_ch, num_layers=layers_per_block + 1,
                                                         add_upsample=i != len(block_out_channels) - 1))
        self.conv_norm_out = GroupNorm(num_channels=block_out_channels[0], num_groups=32, eps=1e-6)
        self.conv_act = nn.SiLU()
        self.conv_out = Conv2dD(block_out_channels[0], out_channels, kernel_size=3, padding=1)
        self.time_conv_out = Conv3dD(out_channels, out_channels, kernel_size=(3, 1, 1), padding=(1, 0, 0))

    def run(self, z_tokens, B, F, H, W, force_split=False):
        """z rows (B*F*H*W, 4) bf16 -> fp32 rows (B*F*8H*8W, 3)."""
        nfr = B * F
        x = ops.conv_direct(z_tokens, self.conv_in.wd(), self.conv_in.b(), B=nfr, H=H, W=W)
        mb = self.mid_block
        x = _st_resblock(mb.resnets[0], x, B, F, H, W, force_split)
        for resnet, attn in zip(mb.resnets[1:], mb.attentions):
            x = attn.run(x, nfr, H * W)
            x = _st_resblock(resnet, x, B, F, H, W, force_split)
        for up in self.up_blocks:
            for resnet in up.resnets:
                x = _st_resblock(resnet, x, B, F, H, W, force_split)
            if up.upsamplers is not None:
                c = up.upsamplers[0].conv
                x = _conv3x3(x, c.w3(), c.b(), nfr, H, W, upsample=True)
                H, W = 2 * H, 2 * W
        g, b = self.conv_norm_out.gb()
        x = ops.groupnorm(x, g, b, self.conv_norm_out.eps, H * W, silu=True)
        x = ops.conv_direct(x, self.conv_out.wd(), self.conv_out.b(), B=nfr, H=H, W=W)
        x = ops.conv_direct(x, self.time_conv_out.wd(), self.time_conv_out.b(), B=B, temporal=dict(F=F, S=H * W),
                            out_f32=True)
        return x, H, W


# ------------------------------------------------------------------------------------------ encoder
class Downsample2D(nn.Module):
    def __init__(self, channels, use_conv=True, out_channels=None, padding=0, name="op"):
        super().__init__()
        self.padding = padding
        self.conv = Conv2dD(channels, out_channels or channels, 3, stride=2, padding=padding)


class DownEncoderBlock2D(nn.Module):
    def __init__(self, in_channels, out_channels, num_layers=2, add_downsample=True):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(in_channels if i == 0 else out_channels, out_channels, None, 1e-6)
                                      for i in range(num_layers)])
        self.downsamplers = nn.ModuleList([Downsample2D(out_channels, out_channels=out_channels, padding=0)]) \
            if add_downsample else None


class UNetMidBlock2D(nn.Module):
    def __init__(self, in_channels, attention_head_dim=512, num_layers=1):
        super().__init__()
        self.attentions = nn.ModuleList([Attention(in_channels, heads=in_channels // attention_head_dim,
                                                   dim_head=attention_head_dim, eps=1e-6) for _ in range(num_layers)])
        self.resnets = nn.ModuleList([ResnetBlock2D(in_channels, in_channels, None, 1e-6)
                                      for _ in range(num_layers + 1)])


class Encoder(nn.Module):
    def __init__(self, in_channels=3, out_channels=4, block_out_channels=(128, 256, 512, 512), layers_per_block=2,
                 double_z=True):
        super().__init__()
        self.layers_per_block = layers_per_block
        self.conv_in = Conv2dD(in_channels, block_out_channels[0], kernel_size=3, stride=1, padding=1)
        self.down_blocks = nn.ModuleList([])
        out_ch = block_out_channels[0]
        for i in range(len(block_out_channels)):
            in_ch, out_ch = out_ch, block_out_channels[i]
            self.down_blocks.append(DownEncoderBlock2D(in_ch, out_ch, num_layers=layers_per_block,
                                                       add_downsample=i != len(block_out_channels) - 1))
        self.mid_block = UNetMidBlock2D(block_out_channels[-1], attention_head_dim=block_out_channels[-1])
        self.conv_norm_out = GroupNorm(num_channels=block_out_channels[-1], num_groups=32, eps=1e-6)
        self.conv_act = nn.SiLU()
        self.conv_out = Conv2d(block_out_channels[-1], 2 * out_channels if double_z else out_channels, 3, padding=1)

    def run(self, x, nimg, H, W):
        x = ops.conv_direct(x, self.conv_in.wd(), self.conv_in.b(), B=nimg, H=H, W=W)
        for blk in self.down_blocks:
            for resnet in blk.resnets:
                x = _resnet2d(resnet, x, nimg, H, W)
            if blk.downsamplers is not None:
                c = blk.downsamplers[0].conv
                x = ops.conv_direct(x, c.wd(), c.b(), B=nimg, H=H, W=W, stride=2, pad0=True)
                H, W = (H - 2) // 2 + 1, (W - 2) // 2 + 1
        mb = self.mid_block
        x = _resnet2d(mb.resnets[0], x, nimg, H, W)
        for attn, resnet in zip(mb.attentions, mb.resnets[1:]):
            x = attn.run(x, nimg, H * W)
            x = _resnet2d(resnet, x, nimg, H, W)
        g, b = self.conv_norm_out.gb()
        x = ops.groupnorm(x, g, b, self.conv_norm_out.eps, H * W, silu=True)
        return _conv3x3(x, self.conv_out.w3(), self.conv_out.b(), nimg, H, W), H, W


# ------------------------------------------------------------------------------------------ autoencoder
class DiagonalGaussianDistribution:
    """diffusers DiagonalGaussianDistribution over moments (B, 2*C, h, w)."""

    def __init__(self, parameters: torch.Tensor):
        self.parameters = parameters
        self.mean, self.logvar = torch.chunk(parameters, 2, dim=1)
        self.logvar = torch.clamp(self.logvar, -30.0, 20.0)
        self.std = torch.exp(0.5 * self.logvar)

    def mode(self) -> torch.Tensor:
        return self.mean

    def sample(self, generator: Optional[torch.Generator] = None) -> torch.Tensor:
        eps = torch.randn(self.mean.shape, generator=generator, device=self.mean.device, dtype=self.mean.dtype)
        return self.mean + self.std * eps


@dataclass
class AutoencoderKLOutput:
    latent_dist: DiagonalGaussianDistribution


@dataclass
class DecoderOutput:
    sample: torch.Tensor


class _Config(dict):
    __getattr__ = dict.__getitem__


class AutoencoderKLTemporalDecoder(nn.Module):
    def __init__(self, in_channels=3, out_channels=3, down_block_types=("DownEncoderBlock2D",) * 4,
                 block_out_channels=(128, 256, 512, 512), layers_per_block=2, latent_channels=4, sample_size=768,
                 scaling_factor=0.18215, force_upcast=True, **_):
        super().__init__()
        self.config = _Config(in_channels=in_channels, out_channels=out_channels,
                              block_out_channels=tuple(block_out_channels), layers_per_block=layers_per_block,
                              latent_channels=latent_channels, sample_size=sample_size,
                              scaling_factor=scaling_factor, force_upcast=force_upcast)
        self.encoder = Encoder(in_channels, latent_channels, block_out_channels, layers_per_block, double_z=True)
        self.decoder = TemporalDecoder(latent_channels, out_channels, block_out_channels, layers_per_block)
        self.quant_conv = Conv2d(2 * latent_channels, 2 * latent_channels, 1)

    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path, subfolder: Optional[str] = None,
                        variant: Optional[str] = None, **kwargs):
        """Local diffusers folder loader (config.json + safetensors / bin weights, strict), as
        ``AutoencoderKLTemporalDecoder.from_pretrained(path, subfolder="vae", variant="fp16")``
        (Inference.py:41-44). Weights are read with safetensors or torch.load(weights_only=True)."""
        import json
        import os
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
                model.load_state_dict(sd, strict=True)
                return model
        raise OSError(f"no weights found in {root}")

    @property
    def dtype(self):
        return self.decoder.conv_in.weight.dtype

    @property
    def device(self):
        return self.decoder.conv_in.weight.device

    def invalidate_kernel_cache(self):
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

    def encode(self, x: torch.Tensor, return_dict: bool = True):
        """(B, 3, H, W) -> latent_dist over (B, 4, H/8, W/8) (fp32 moments)."""
        Bn, _, H, W = x.shape
        t = ops.nchw_to_tokens(x)
        h, h_, w_ = self.encoder.run(t, Bn, H, W)
        mom = _gemm_rows(h, self.quant_conv.w1(), bias=self.quant_conv.b(), out_f32=True)
        moments = ops.tokens_to_nchw(mom, Bn, h_, w_)
        post = DiagonalGaussianDistribution(moments)
        return AutoencoderKLOutput(latent_dist=post) if return_dict else (post,)

    def decode(self, z: torch.Tensor, num_frames: int, return_dict: bool = True, force_split: bool = False):
        """(B*num_frames, 4, h, w) -> (B*num_frames, 3, 8h, 8w) fp32."""
        BF, _, h, w = z.shape
        B = BF // num_frames
        if B * num_frames != BF:
            raise ValueError(f"decode: {BF} latents are not a multiple of num_frames={num_frames}")
        t = ops.nchw_to_tokens(z)
        y, H, W = self.decoder.run(t, B, num_frames, h, w, force_split=force_split)
        out = ops.tokens_to_nchw(y, BF, H, W)
        return DecoderOutput(sample=out) if return_dict else (out,)

    def forward(self, sample, num_frames: int = 1):
        return self.decode(self.encode(sample).latent_dist.mode(), num_frames)


def decode_latents(vae: AutoencoderKLTemporalDecoder, latents: torch.Tensor, num_frames: int,
                   decode_chunk_size: int = 14) -> torch.Tensor:
    """Pipeline ``decode_latents`` (pipeline:264-290): (b, f, 4, h, w) -> (b, 3, f, H, W) fp32,
    decoding ``decode_chunk_size`` frames at a time with num_frames = the chunk length."""
    lat = latents.flatten(0, 1) * (1.0 / vae.config.scaling_factor)
    frames = []
    for i in range(0, lat.shape[0], decode_chunk_size):
        chunk = lat[i:i + decode_chunk_size]
        frames.append(vae.decode(chunk, num_frames=chunk.shape[0]).sample)
    frames = torch.cat(frames, 0)
    frames = frames.reshape(-1, num_frames, *frames.shape[1:]).permute(0, 2, 1, 3, 4)
    return frames.float()


def encode_ref_image(vae: AutoencoderKLTemporalDecoder, ref_image: torch.Tensor) -> torch.Tensor:
    """``vae.encode(ref).latent_dist.mean * 0.18215`` (pipeline:520-521)."""
    return vae.encode(ref_image).latent_dist.mean * 0.18215


__all__ = ["AutoencoderKLTemporalDecoder", "decode_latents", "encode_ref_image", "Attention", "TemporalDecoder",
           "Encoder"]
