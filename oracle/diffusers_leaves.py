"""ORACLE — test infrastructure only (tools/ golden generators, tests/). Never imported by actalker_amd.

CPU ``nn.Module`` stand-ins for the diffusers 0.29.2 building blocks the reference UNet package imports
(diffusers is absent from this container): same constructor signatures and parameter names as the
pinned version, forward passes delegated to the oracle's functional restatements
(``oracle.reference_cpu``). They let the reference's OWN orchestration code --
unet_spatio_temporal_condition_mambaID_v10_two_ip.py, unet_3d_blocks.py, TransformerSTmodel.py,
attention.py, attention_processor.py, mamba_layer.py -- run unchanged on the CPU, so a golden made with
them pins everything those files define and leaves only these leaves restated.

diffusers 0.29.2 sources restated (module : class):
  models/embeddings.py : Timesteps, TimestepEmbedding
  models/resnet.py     : ResnetBlock2D, TemporalResnetBlock, SpatioTemporalResBlock, AlphaBlender,
                         Downsample2D, Upsample2D
  models/attention.py  : FeedForward, GEGLU
Reference call sites: unet_3d_blocks.py:24-31 (imports), :2068, 2089, 2174, 2187, 2274, 2303, 2399, 2410,
2499, 2526; attention.py:22 (FeedForward), :374, :394, :406; v10 UNet :12, :141-147;
TransformerSTmodel.py:25, :3989-3990.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from oracle import reference_cpu as ref


def _sd(module: nn.Module, p: str = "m"):
    return {f"{p}.{k}": v for k, v in module.state_dict().items()}


class Timesteps(nn.Module):
    """embeddings.py Timesteps: sinusoidal projection, no weights."""

    def __init__(self, num_channels: int, flip_sin_to_cos: bool, downscale_freq_shift: float, scale: int = 1):
        super().__init__()
        self.num_channels = num_channels
        self.flip_sin_to_cos = flip_sin_to_cos
        self.downscale_freq_shift = downscale_freq_shift
        self.scale = scale

    def forward(self, timesteps):
        return ref.timestep_embedding(timesteps, self.num_channels, self.flip_sin_to_cos, self.downscale_freq_shift,
                                      self.scale)


class TimestepEmbedding(nn.Module):
    """embeddings.py TimestepEmbedding (act_fn silu, no cond_proj / post_act): linear_1 -> SiLU -> linear_2."""

    def __init__(self, in_channels: int, time_embed_dim: int, act_fn: str = "silu", out_dim: int = None,
                 post_act_fn: Optional[str] = None, cond_proj_dim=None, sample_proj_bias=True):
        super().__init__()
        assert act_fn == "silu" and post_act_fn is None and cond_proj_dim is None
        self.linear_1 = nn.Linear(in_channels, time_embed_dim, sample_proj_bias)
        self.act = nn.SiLU()
        self.linear_2 = nn.Linear(time_embed_dim, out_dim if out_dim is not None else time_embed_dim, sample_proj_bias)

    def forward(self, sample, condition=None):
        assert condition is None
        return ref.timestep_embedding_mlp(_sd(self), "m", sample)


class ResnetBlock2D(nn.Module):
    """resnet.py ResnetBlock2D, the configuration SpatioTemporalResBlock builds (default time embedding
    norm, swish, pre-norm, 1x1 shortcut when the widths differ, output scale 1)."""

    def __init__(self, *, in_channels: int, out_channels: Optional[int] = None, conv_shortcut: bool = False,
                 dropout: float = 0.0, temb_channels: int = 512, groups: int = 32, groups_out: Optional[int] = None,
                 pre_norm: bool = True, eps: float = 1e-6, non_linearity: str = "swish", skip_time_act: bool = False,
                 time_embedding_norm: str = "default", kernel=None, output_scale_factor: float = 1.0,
                 use_in_shortcut: Optional[bool] = None, up: bool = False, down: bool = False,
                 conv_shortcut_bias: bool = True, conv_2d_out_channels: Optional[int] = None):
        super().__init__()
        assert time_embedding_norm == "default" and non_linearity == "swish" and not (up or down)
        assert output_scale_factor == 1.0 and groups == 32 and groups_out in (None, 32) and not conv_shortcut
        out_channels = in_channels if out_channels is None else out_channels
        self.eps = eps
        self.norm1 = nn.GroupNorm(groups, in_channels, eps=eps, affine=True)
        self.conv1 = nn.Conv2d(in_channels, out_channels, 3, 1, 1)
        self.time_emb_proj = nn.Linear(temb_channels, out_channels)
        self.norm2 = nn.GroupNorm(groups, out_channels, eps=eps, affine=True)
        self.conv2 = nn.Conv2d(out_channels, conv_2d_out_channels or out_channels, 3, 1, 1)
        self.use_in_shortcut = (in_channels != (conv_2d_out_channels or out_channels)
                                if use_in_shortcut is None else use_in_shortcut)
        self.conv_shortcut = (nn.Conv2d(in_channels, conv_2d_out_channels or out_channels, 1, 1, 0,
                                        bias=conv_shortcut_bias) if self.use_in_shortcut else None)

    def forward(self, input_tensor, temb, *args, **kwargs):
        return ref.resnet_block_2d(_sd(self), "m", input_tensor, temb, self.eps)


class TemporalResnetBlock(nn.Module):
    """resnet.py TemporalResnetBlock: GN-SiLU-Conv3d(3,1,1) + temb + GN-SiLU-Conv3d(3,1,1) + skip on
    (B, C, F, H, W); the GroupNorm statistics span all F frames."""

    def __init__(self, in_channels: int, out_channels: Optional[int] = None, temb_channels: int = 512,
                 eps: float = 1e-6):
        super().__init__()
        out_channels = in_channels if out_channels is None else out_channels
        self.eps = eps
        self.norm1 = nn.GroupNorm(32, in_channels, eps=eps, affine=True)
        self.conv1 = nn.Conv3d(in_channels, out_channels, (3, 1, 1), 1, (1, 0, 0))
        self.time_emb_proj = nn.Linear(temb_channels, out_channels) if temb_channels is not None else None
        self.norm2 = nn.GroupNorm(32, out_channels, eps=eps, affine=True)
        self.conv2 = nn.Conv3d(out_channels, out_channels, (3, 1, 1), 1, (1, 0, 0))
        self.conv_shortcut = (nn.Conv3d(in_channels, out_channels, 1, 1, 0) if in_channels != out_channels else None)

    def forward(self, input_tensor, temb):
        return ref.temporal_resnet_block(_sd(self), "m", input_tensor, temb, self.eps)


class AlphaBlender(nn.Module):
    """resnet.py AlphaBlender, 'learned_with_images': alpha = 1 where image_only_indicator is set, else
    sigmoid(mix_factor)."""

    def __init__(self, alpha: float, merge_strategy: str = "learned_with_images",
                 switch_spatial_to_temporal_mix: bool = False):
        super().__init__()
        assert merge_strategy == "learned_with_images" and not switch_spatial_to_temporal_mix
        self.mix_factor = nn.Parameter(torch.tensor([float(alpha)]))

    def forward(self, x_spatial, x_temporal, image_only_indicator):
        alpha = torch.where(image_only_indicator.bool(), torch.ones(1, 1), torch.sigmoid(self.mix_factor)[..., None])
        alpha = alpha[:, None, :, None, None] if x_spatial.ndim == 5 else alpha.reshape(-1)[:, None, None]
        return alpha * x_spatial + (1.0 - alpha) * x_temporal


class SpatioTemporalResBlock(nn.Module):
    """resnet.py SpatioTemporalResBlock: ResnetBlock2D per frame, TemporalResnetBlock over the frames of
    each batch element, AlphaBlender between them."""

    def __init__(self, in_channels: int, out_channels: Optional[int] = None, temb_channels: int = 512,
                 eps: float = 1e-6, temporal_eps: Optional[float] = None, merge_factor: float = 0.5,
                 merge_strategy="learned_with_images", switch_spatial_to_temporal_mix: bool = False):
        super().__init__()
        self.spatial_res_block = ResnetBlock2D(in_channels=in_channels, out_channels=out_channels,
                                               temb_channels=temb_channels, eps=eps)
        oc = out_channels if out_channels is not None else in_channels
        self.temporal_res_block = TemporalResnetBlock(in_channels=oc, out_channels=oc, temb_channels=temb_channels,
                                                      eps=temporal_eps if temporal_eps is not None else eps)
        self.time_mixer = AlphaBlender(alpha=merge_factor, merge_strategy=merge_strategy,
                                       switch_spatial_to_temporal_mix=switch_spatial_to_temporal_mix)

    def forward(self, hidden_states, temb=None, image_only_indicator=None):
        num_frames = image_only_indicator.shape[-1]
        hidden_states = self.spatial_res_block(hidden_states, temb)
        bf, c, h, w = hidden_states.shape
        b = bf // num_frames
        mix = hidden_states[None, :].reshape(b, num_frames, c, h, w).permute(0, 2, 1, 3, 4)
        if temb is not None:
            temb = temb.reshape(b, num_frames, -1)
        x_t = self.temporal_res_block(mix, temb)
        out = self.time_mixer(x_spatial=mix, x_temporal=x_t, image_only_indicator=image_only_indicator)
        return out.permute(0, 2, 1, 3, 4).reshape(bf, c, h, w)


class Downsample2D(nn.Module):
    """resnet.py Downsample2D (use_conv, padding 1): 3x3 stride-2 conv. Any name other than 'conv' /
    'Conv2d_0' still registers the conv as ``conv`` (the reference passes name='op')."""

    def __init__(self, channels: int, use_conv: bool = False, out_channels: Optional[int] = None, padding: int = 1,
                 name: str = "conv", kernel_size=3, norm_type=None, eps=None, elementwise_affine=None, bias=True):
        super().__init__()
        assert use_conv and padding == 1 and norm_type is None and kernel_size == 3
        self.conv = nn.Conv2d(channels, out_channels or channels, 3, 2, padding, bias=bias)

    def forward(self, hidden_states, *args, **kwargs):
        return ref.downsample_2d(_sd(self), "m", hidden_states)


class Upsample2D(nn.Module):
    """resnet.py Upsample2D (use_conv, no transpose): nearest x2 then 3x3 conv."""

    def __init__(self, channels: int, use_conv: bool = False, use_conv_transpose: bool = False,
                 out_channels: Optional[int] = None, name: str = "conv", kernel_size=None, padding=1, norm_type=None,
                 eps=None, elementwise_affine=None, bias=True, interpolate=True):
        super().__init__()
        assert use_conv and not use_conv_transpose and norm_type is None and interpolate and name == "conv"
        self.conv = nn.Conv2d(channels, out_channels or channels, kernel_size or 3, padding=padding, bias=bias)

    def forward(self, hidden_states, output_size=None, *args, **kwargs):
        assert output_size is None
        return ref.upsample_2d(_sd(self), "m", hidden_states)


class GEGLU(nn.Module):
    """attention.py / activations.py GEGLU: one Linear to 2 x dim_out, split hidden | gate."""

    def __init__(self, dim_in: int, dim_out: int, bias: bool = True):
        super().__init__()
        self.proj = nn.Linear(dim_in, dim_out * 2, bias=bias)


class FeedForward(nn.Module):
    """attention.py FeedForward(activation_fn='geglu'): net = [GEGLU, Dropout, Linear]."""

    def __init__(self, dim: int, dim_out: Optional[int] = None, mult: int = 4, dropout: float = 0.0,
                 activation_fn: str = "geglu", final_dropout: bool = False, inner_dim=None, bias: bool = True):
        super().__init__()
        assert activation_fn == "geglu" and not final_dropout
        inner_dim = int(dim * mult) if inner_dim is None else inner_dim
        self.net = nn.ModuleList([GEGLU(dim, inner_dim, bias), nn.Dropout(dropout),
                                  nn.Linear(inner_dim, dim_out if dim_out is not None else dim, bias=bias)])

    def forward(self, hidden_states, *args, **kwargs):
        return ref.feed_forward(_sd(self), "m", hidden_states)
