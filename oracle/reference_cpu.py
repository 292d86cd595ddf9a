"""ORACLE — test infrastructure only. Never imported by the product package (actalker_amd).

CPU fp32 restatement of ACTalker's denoising path, written as plain functions over a state dict
so it shares no code with the HIP implementation. It follows the reference files line by line
(NCHW layout, the reference's permutes, torch SDPA, a per-step selective-scan loop); each function
cites the reference file:line it restates. Third-party pieces the reference calls but that are not
in /root/reference are restated from their pinned versions:
  * mamba-ssm 1.2.0.post1 ``selective_scan_ref`` (environment.yaml:43)
  * diffusers 0.29.2 (requirements.txt:10): ResnetBlock2D, TemporalResnetBlock, SpatioTemporalResBlock,
    Downsample2D, Upsample2D, Attention (to_q/k/v, to_out), FeedForward/GEGLU, TimestepEmbedding,
    IPAdapterMaskProcessor.downsample, EulerDiscreteScheduler (Karras sigmas, v-prediction).
Pinning: SS2D_cond_v10 / SS2D_Unit (mamba_layer.py) are checked against golden vectors produced by
the reference module itself (tests/golden, tools/gen_golden.py). The UNet blocks, attention
processors and scheduler have no reference test or fixture: their parity is unpinned beyond this
restatement.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

SD = Dict[str, torch.Tensor]


# ============================================================================ third party
def selective_scan_ref(u, delta, A, B, C, D=None, z=None, delta_bias=None, delta_softplus=False,
                       return_last_state=False):
    """mamba-ssm 1.2.0 selective_scan_interface.selective_scan_ref (real A, variable B/C)."""
    dtype_in = u.dtype
    u = u.float()
    delta = delta.float()
    if delta_bias is not None:
        delta = delta + delta_bias[..., None].float()
    if delta_softplus:
        delta = F.softplus(delta)
    batch, dim, dstate = u.shape[0], A.shape[0], A.shape[1]
    B = B.float()
    C = C.float()
    x = A.new_zeros((batch, dim, dstate))
    ys = []
    deltaA = torch.exp(torch.einsum('bdl,dn->bdln', delta, A))
    if B.dim() == 3:
        deltaB_u = torch.einsum('bdl,bnl,bdl->bdln', delta, B, u)
    else:
        Bx = B.repeat_interleave(dim // B.shape[1], dim=1)
        deltaB_u = torch.einsum('bdl,bdnl,bdl->bdln', delta, Bx, u)
    if C.dim() == 4:
        C = C.repeat_interleave(dim // C.shape[1], dim=1)
    last_state = None
    for i in range(u.shape[2]):
        x = deltaA[:, :, i] * x + deltaB_u[:, :, i]
        if C.dim() == 3:
            y = torch.einsum('bdn,bn->bd', x, C[:, :, i])
        else:
            y = torch.einsum('bdn,bdn->bd', x, C[:, :, :, i])
        if i == u.shape[2] - 1:
            last_state = x
        ys.append(y)
    y = torch.stack(ys, dim=2)
    out = y if D is None else y + u * D[:, None]
    if z is not None:
        out = out * F.silu(z)
    out = out.to(dtype=dtype_in)
    return out if not return_last_state else (out, last_state)


def mask_downsample(mask, batch_size, num_queries, value_embed_dim):
    """diffusers 0.29.2 IPAdapterMaskProcessor.downsample; mask (1, H, W)."""
    o_h, o_w = mask.shape[1], mask.shape[2]
    ratio = o_w / o_h
    mask_h = int(math.sqrt(num_queries / ratio))
    mask_h = int(mask_h) + int((num_queries % int(mask_h)) != 0)
    mask_w = num_queries // mask_h
    md = F.interpolate(mask.unsqueeze(0), size=(mask_h, mask_w), mode="bicubic").squeeze(0)
    if md.shape[0] < batch_size:
        md = md.repeat(batch_size, 1, 1)
    md = md.view(md.shape[0], -1)
    area = mask_h * mask_w
    if area < num_queries:
        md = F.pad(md, (0, num_queries - md.shape[1]), value=0.0)
    if area > num_queries:
        md = md[:, :num_queries]
    return md.view(md.shape[0], md.shape[1], 1).repeat(1, 1, value_embed_dim)


def timestep_embedding(timesteps, embedding_dim, flip_sin_to_cos=False, downscale_freq_shift=1.0, scale=1.0,
                       max_period=10000):
    """TransformerSTmodel.py:43-96 (== diffusers get_timestep_embedding)."""
    half_dim = embedding_dim // 2
    exponent = -math.log(max_period) * torch.arange(0, half_dim, dtype=torch.float32)
    exponent = exponent / (half_dim - downscale_freq_shift)
    emb = torch.exp(exponent)
    emb = timesteps[:, None].float() * emb[None, :]
    emb = scale * emb
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=-1)
    if flip_sin_to_cos:
        emb = torch.cat([emb[:, half_dim:], emb[:, :half_dim]], dim=-1)
    if embedding_dim % 2 == 1:
        emb = F.pad(emb, (0, 1, 0, 0))
    return emb


def linear(sd: SD, p: str, x):
    return F.linear(x, sd[p + ".weight"], sd.get(p + ".bias"))


def timestep_embedding_mlp(sd: SD, p: str, x):
    """diffusers TimestepEmbedding: linear_1 -> SiLU -> linear_2."""
    return linear(sd, p + ".linear_2", F.silu(linear(sd, p + ".linear_1", x)))


def group_norm(sd: SD, p: str, x, eps, groups=32):
    return F.group_norm(x, groups, sd[p + ".weight"], sd[p + ".bias"], eps)


def layer_norm(sd: SD, p: str, x, eps=1e-5):
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".weight"], sd[p + ".bias"], eps)


# ---- diffusers 0.29.2 resnet.py
def resnet_block_2d(sd: SD, p: str, x, temb, eps):
    h = F.silu(group_norm(sd, p + ".norm1", x, eps))
    h = F.conv2d(h, sd[p + ".conv1.weight"], sd[p + ".conv1.bias"], padding=1)
    t = linear(sd, p + ".time_emb_proj", F.silu(temb))[:, :, None, None]
    h = h + t
    h = F.silu(group_norm(sd, p + ".norm2", h, eps))
    h = F.conv2d(h, sd[p + ".conv2.weight"], sd[p + ".conv2.bias"], padding=1)
    if p + ".conv_shortcut.weight" in sd:
        x = F.conv2d(x, sd[p + ".conv_shortcut.weight"], sd[p + ".conv_shortcut.bias"])
    return x + h


def temporal_resnet_block(sd: SD, p: str, x, temb, eps):
    """x: (B, C, F, H, W); temb: (B, F, Ct)."""
    h = F.silu(group_norm(sd, p + ".norm1", x, eps))
    h = F.conv3d(h, sd[p + ".conv1.weight"], sd[p + ".conv1.bias"], padding=(1, 0, 0))
    t = linear(sd, p + ".time_emb_proj", F.silu(temb))[:, :, :, None, None].permute(0, 2, 1, 3, 4)
    h = h + t
    h = F.silu(group_norm(sd, p + ".norm2", h, eps))
    h = F.conv3d(h, sd[p + ".conv2.weight"], sd[p + ".conv2.bias"], padding=(1, 0, 0))
    if p + ".conv_shortcut.weight" in sd:
        x = F.conv3d(x, sd[p + ".conv_shortcut.weight"], sd[p + ".conv_shortcut.bias"])
    return x + h


def alpha_blend(sd: SD, p: str, x_spatial, x_temporal):
    """AlphaBlender 'learned_with_images' with image_only_indicator == 0 (TransformerSTmodel.py:116-197)."""
    a = torch.sigmoid(sd[p + ".mix_factor"])
    return a * x_spatial + (1.0 - a) * x_temporal


def spatio_temporal_res_block(sd: SD, p: str, x, temb, num_frames, eps):
    h = resnet_block_2d(sd, p + ".spatial_res_block", x, temb, eps)
    bf, c, hh, ww = h.shape
    b = bf // num_frames
    h_mix = h[None].reshape(b, num_frames, c, hh, ww).permute(0, 2, 1, 3, 4)
    h5 = h_mix
    t = temb.reshape(b, num_frames, -1)
    h5 = temporal_resnet_block(sd, p + ".temporal_res_block", h5, t, eps)
    out = alpha_blend(sd, p + ".time_mixer", h_mix, h5)
    return out.permute(0, 2, 1, 3, 4).reshape(bf, c, hh, ww)


def downsample_2d(sd: SD, p: str, x):
    return F.conv2d(x, sd[p + ".conv.weight"], sd[p + ".conv.bias"], stride=2, padding=1)


def upsample_2d(sd: SD, p: str, x):
    x = F.interpolate(x, scale_factor=2.0, mode="nearest")
    return F.conv2d(x, sd[p + ".conv.weight"], sd[p + ".conv.bias"], padding=1)


def feed_forward(sd: SD, p: str, x):
    """diffusers FeedForward(geglu): GEGLU proj -> hidden * gelu(gate) -> Linear."""
    h, g = linear(sd, p + ".net.0.proj", x).chunk(2, dim=-1)
    return linear(sd, p + ".net.2", h * F.gelu(g))


# ============================================================================ attention
def _sdpa(q, k, v, heads):
    b = q.shape[0]
    hd = q.shape[-1] // heads
    q = q.view(b, -1, heads, hd).transpose(1, 2)
    k = k.view(b, -1, heads, hd).transpose(1, 2)
    v = v.view(b, -1, heads, hd).transpose(1, 2)
    o = F.scaled_dot_product_attention(q, k, v)
    return o.transpose(1, 2).reshape(b, -1, heads * hd)


def attn_processor(sd: SD, p: str, x, heads, context=None):
    """AttnProcessor2_0 (attention_processor.py:1528-1605)."""
    ctx = x if context is None else context
    o = _sdpa(linear(sd, p + ".to_q", x), linear(sd, p + ".to_k", ctx), linear(sd, p + ".to_v", ctx), heads)
    return linear(sd, p + ".to_out.0", o)


def ip_attn_processor(sd: SD, p: str, x, heads, ehs, scale: Sequence[float], masks=None):
    """IPAdapterAttnProcessor2_0 (attention_processor.py:2747-2934). ehs = (context, [ip_0, ip_1])."""
    context, ip_states = ehs
    b = x.shape[0]
    q = linear(sd, p + ".to_q", x)
    hs = _sdpa(q, linear(sd, p + ".to_k", context), linear(sd, p + ".to_v", context), heads)
    for i, ip in enumerate(ip_states):
        if ip.dim() == 4:
            ip = ip[:, 0]
        k = linear(sd, f"{p}.processor.to_k_ip.{i}", ip)
        v = linear(sd, f"{p}.processor.to_v_ip.{i}", ip)
        o = _sdpa(q, k, v, heads)
        if masks is not None:
            md = mask_downsample(masks[i][:, 0, :, :], b, o.shape[1], o.shape[2])
            hs = hs + scale[i] * (o * md)
        else:
            hs = hs + scale[i] * o
    return linear(sd, p + ".to_out.0", hs)


def _attn2(sd, p, x, heads, ehs, ip_scale, masks):
    if ip_scale is None:  # no IP processor installed: plain cross attention to the first context
        return attn_processor(sd, p, x, heads, ehs[0] if isinstance(ehs, tuple) else ehs)
    return ip_attn_processor(sd, p, x, heads, ehs, ip_scale, masks)


def basic_transformer_block(sd: SD, p: str, h, heads, ehs, ip_scale, masks):
    """attention.py:223-343 (layer_norm variant)."""
    n = layer_norm(sd, p + ".norm1", h)
    h = attn_processor(sd, p + ".attn1", n, heads) + h
    n = layer_norm(sd, p + ".norm2", h)
    h = _attn2(sd, p + ".attn2", n, heads, ehs, ip_scale, masks) + h
    n = layer_norm(sd, p + ".norm3", h)
    return feed_forward(sd, p + ".ff", n) + h


def temporal_basic_transformer_block(sd: SD, p: str, h, num_frames, heads, ehs_time, ip_scale):
    """attention.py:418-473."""
    bf, s, c = h.shape
    b = bf // num_frames
    h = h[None].reshape(b, num_frames, s, c).permute(0, 2, 1, 3).reshape(b * s, num_frames, c)
    res = h
    h = feed_forward(sd, p + ".ff_in", layer_norm(sd, p + ".norm_in", h)) + res
    h = attn_processor(sd, p + ".attn1", layer_norm(sd, p + ".norm1", h), heads) + h
    h = _attn2(sd, p + ".attn2", layer_norm(sd, p + ".norm2", h), heads, ehs_time, ip_scale, None) + h
    h = feed_forward(sd, p + ".ff", layer_norm(sd, p + ".norm3", h)) + h
    return h[None].reshape(b, s, num_frames, c).permute(0, 2, 1, 3).reshape(b * num_frames, s, c)


# ============================================================================ Mamba
def ss2d_unit(sd: SD, p: str, x):
    """SS2D_Unit.forward_core (mamba_layer.py:1505-1548), scan_type='sweep', num_direction=2.
    x: (B, d_inner, L)."""
    B, C, L = x.shape
    K = 2
    xpw = sd[p + ".x_proj_weight"]
    dtw = sd[p + ".dt_projs_weight"]
    R = dtw.shape[-1]
    N = (xpw.shape[1] - R) // 2
    xs = x.view(B, 1, -1, L)                                   # HSCANS 'sweep' encode = identity
    xs = torch.cat([xs, torch.flip(xs, dims=[-1])], dim=1)
    x_dbl = torch.einsum("b k d l, k c d -> b k c l", xs.view(B, K, -1, L), xpw)
    dts, Bs, Cs = torch.split(x_dbl, [R, N, N], dim=2)
    dts = torch.einsum("b k r l, k d r -> b k d l", dts.view(B, K, -1, L), dtw)
    xs = xs.view(B, -1, L)
    dts = dts.contiguous().view(B, -1, L)
    As = -torch.exp(sd[p + ".A_logs"].float()).view(-1, N)
    out_y = selective_scan_ref(xs, dts, As, Bs.view(B, K, -1, L), Cs.view(B, K, -1, L), sd[p + ".Ds"].float().view(-1),
                               z=None, delta_bias=sd[p + ".dt_projs_bias"].float().view(-1), delta_softplus=True)
    out_y = out_y.view(B, K, -1, L)
    inv_y = torch.flip(out_y[:, 1:2], dims=[-1]).view(B, 1, -1, L)
    return out_y[:, 0] + inv_y[:, 0]


def ss2d_cond_v10(sd: SD, p: str, x, id_emb, conds, masks):
    """SS2D_cond_v10.forward (mamba_layer.py:1955-1986). x: (B, L, C); conds: (B, 33, d_cond)."""
    audio_cond = conds[:, :-1]
    exp_cond = conds[:, -1:]
    id_e = F.silu(linear(sd, p + ".id_proj", id_emb))
    xz1 = linear(sd, p + ".in_proj1", x)
    am = mask_downsample(masks[0][:, 0, :, :], masks[0].shape[0], xz1.shape[1], 1)
    idx = am.view(-1).int().nonzero().view(-1)
    sel = xz1[:, idx, :]
    n = sel.shape[1]
    audio_input = torch.cat([sel, id_e, F.silu(linear(sd, p + ".audio_proj", audio_cond))], dim=1)
    out = ss2d_unit(sd, p + ".audio_unit", audio_input.permute(0, 2, 1)).to(xz1.dtype)
    xz1 = xz1.clone()
    xz1[:, idx, :] = out[:, :, :n].permute(0, 2, 1)

    xz2 = linear(sd, p + ".in_proj2", x)
    em = mask_downsample(masks[1][:, 0, :, :], masks[1].shape[0], xz2.shape[1], 1)
    idx = em.view(-1).int().nonzero().view(-1)
    sel = xz2[:, idx, :]
    n = sel.shape[1]
    exp_input = torch.cat([sel, id_e, F.silu(linear(sd, p + ".exp_proj", exp_cond))], dim=1)
    out = ss2d_unit(sd, p + ".exp_unit", exp_input.permute(0, 2, 1)).to(xz2.dtype)
    xz2 = xz2.clone()
    xz2[:, idx, :] = out[:, :, :n].permute(0, 2, 1)

    y = layer_norm(sd, p + ".out_norm", xz2 + xz1)
    return linear(sd, p + ".out_proj", y)


# ============================================================================ transformer
def transformer_st(sd: SD, p: str, x, ehs, cak, num_frames, heads, ip_scale, mamba: bool):
    """TransformerSpatioTemporalModel (TransformerSTmodel.py:276-421) and the v10 variant
    (:4001-4155, Mamba after the spatial block, no residual around it)."""
    bf, _, hh, ww = x.shape
    b = bf // num_frames

    def spatial2time(t):
        t = t.reshape(b, num_frames, t.shape[-2], t.shape[-1])
        t = t.mean(dim=(1,), keepdim=True)
        t = t.repeat(1, hh * ww, 1, 1)
        return t.reshape(b * hh * ww, -1, t.shape[-1])

    if isinstance(ehs, tuple):
        ehs_time = (spatial2time(ehs[0]), [spatial2time(s) for s in ehs[1]])
    else:
        ehs_time = spatial2time(ehs)
    res = x
    h = group_norm(sd, p + ".norm", x, 1e-6)
    c = h.shape[1]
    h = h.permute(0, 2, 3, 1).reshape(bf, hh * ww, c)
    h = linear(sd, p + ".proj_in", h)
    fidx = torch.arange(num_frames).repeat(b, 1).reshape(-1)
    emb = timestep_embedding_mlp(sd, p + ".time_pos_embed", timestep_embedding(fidx, c, True, 0))[:, None, :]
    masks = cak.get("ip_adapter_masks") if cak else None
    h = basic_transformer_block(sd, p + ".transformer_blocks.0", h, heads, ehs, ip_scale, masks)
    if mamba:
        conds = torch.cat([ehs[1][0].reshape(bf, -1, ehs[1][0].shape[-1]),
                           ehs[1][1].reshape(bf, -1, ehs[1][1].shape[-1])], dim=1)
        h = ss2d_cond_v10(sd, p + ".mamba_blocks.0", h, ehs[0], conds, masks)
    hm = h + emb
    hm = temporal_basic_transformer_block(sd, p + ".temporal_transformer_blocks.0", hm, num_frames, heads, ehs_time,
                                          ip_scale)
    h = alpha_blend(sd, p + ".time_mixer", h, hm)
    h = linear(sd, p + ".proj_out", h)
    h = h.reshape(bf, hh, ww, c).permute(0, 3, 1, 2)
    return h + res


# ============================================================================ UNet
DEFAULT_CFG = dict(in_channels=8, out_channels=4, block_out_channels=(320, 640, 1280, 1280),
                   num_attention_heads=(5, 10, 20, 20), layers_per_block=2, cross_attention_dim=1024)


def unet_forward(sd: SD, sample, timestep, encoder_hidden_states, added_time_ids, spatial_condition=None,
                 cross_attention_kwargs=None, ip_scale: Optional[Sequence[float]] = (1.25, 1.25), cfg=None):
    """UNetSpatioTemporalConditionModel.forward (unet_spatio_temporal_condition_mambaID_v10_two_ip.py:362-517)
    with down/mid/up blocks of unet_3d_blocks.py:2047-2592. Returns (B, F, out_ch, h, w)."""
    cfg = dict(DEFAULT_CFG, **(cfg or {}))
    ch = cfg["block_out_channels"]
    heads = cfg["num_attention_heads"]
    B, Fn = sample.shape[:2]
    t = timestep if torch.is_tensor(timestep) else torch.tensor([timestep], dtype=torch.float32)
    t = t.reshape(-1).float().expand(B)
    emb = timestep_embedding_mlp(sd, "time_embedding", timestep_embedding(t, ch[0], True, 0))
    aug = timestep_embedding(added_time_ids.flatten().float(), 256, True, 0).reshape(B, -1)
    emb = emb + timestep_embedding_mlp(sd, "add_embedding", aug)
    x = sample.flatten(0, 1).float()
    emb = emb.repeat_interleave(Fn, dim=0)
    if isinstance(encoder_hidden_states, tuple):
        ehs, ips = encoder_hidden_states
        if ehs.shape[0] == B:
            ehs = ehs.repeat_interleave(Fn, dim=0)
        ehs = (ehs.float(), [s.float() for s in ips])
    else:
        ehs = encoder_hidden_states.float()
        if ehs.shape[0] == B:
            ehs = ehs.repeat_interleave(Fn, dim=0)
    x = F.conv2d(x, sd["conv_in.weight"], sd["conv_in.bias"], padding=1)
    if spatial_condition is not None:
        x = x + spatial_condition.flatten(0, 1).float()
    cak = cross_attention_kwargs or {}

    skips = [x]
    # down: 0-2 CrossAttnDown (eps 1e-6, unet_3d_blocks.py:2278), 3 Down (eps 1e-5, :2178)
    for i in range(4):
        p = f"down_blocks.{i}"
        for j in range(cfg["layers_per_block"]):
            if i < 3:
                x = spatio_temporal_res_block(sd, f"{p}.resnets.{j}", x, emb, Fn, 1e-6)
                x = transformer_st(sd, f"{p}.attentions.{j}", x, ehs, cak, Fn, heads[i], ip_scale, mamba=True)
            else:
                x = spatio_temporal_res_block(sd, f"{p}.resnets.{j}", x, emb, Fn, 1e-5)
            skips.append(x)
        if i < 3:
            x = downsample_2d(sd, f"{p}.downsamplers.0", x)
            skips.append(x)
    # mid (eps 1e-5, :2072,2093; plain transformer)
    x = spatio_temporal_res_block(sd, "mid_block.resnets.0", x, emb, Fn, 1e-5)
    x = transformer_st(sd, "mid_block.attentions.0", x, ehs, cak, Fn, heads[-1], ip_scale, mamba=False)
    x = spatio_temporal_res_block(sd, "mid_block.resnets.1", x, emb, Fn, 1e-5)
    # up: 0 UpBlock, 1-3 CrossAttnUp; all eps 1e-6 (get_up_block does not forward resnet_eps)
    rev_heads = list(reversed(heads))
    for i in range(4):
        p = f"up_blocks.{i}"
        for j in range(cfg["layers_per_block"] + 1):
            x = torch.cat([x, skips.pop()], dim=1)
            x = spatio_temporal_res_block(sd, f"{p}.resnets.{j}", x, emb, Fn, 1e-6)
            if i > 0:
                x = transformer_st(sd, f"{p}.attentions.{j}", x, ehs, cak, Fn, rev_heads[i], ip_scale, mamba=True)
        if i < 3:
            x = upsample_2d(sd, f"{p}.upsamplers.0", x)
    x = F.silu(group_norm(sd, "conv_norm_out", x, 1e-5))
    x = F.conv2d(x, sd["conv_out.weight"], sd["conv_out.bias"], padding=1)
    return x.reshape(B, Fn, *x.shape[1:])


# ============================================================================ conditioning adapters
def _k(p: str, name: str) -> str:
    return name if not p else p + "." + name


def audio_proj_model(sd: SD, p: str, audio_embeds, context_tokens=32):
    """AudioProjModel.forward (src/models/audio_adapter/audio_proj.py:103-130)."""
    bz, f = audio_embeds.shape[:2]
    x = audio_embeds.reshape(bz * f, -1)
    x = F.relu(linear(sd, _k(p, "proj1"), x))
    x = F.relu(linear(sd, _k(p, "proj2"), x))
    x = linear(sd, _k(p, "proj3"), x).reshape(bz * f, context_tokens, -1)
    x = layer_norm(sd, _k(p, "norm"), x)
    return x.reshape(bz, f, context_tokens, -1)


def vasa_proj_model(sd: SD, p: str, x):
    """VasaProjModel.forward (audio_proj.py:147-150)."""
    return layer_norm(sd, _k(p, "norm"), linear(sd, _k(p, "proj1"), x))


def id_proj_model(sd: SD, p: str, x):
    """IDProjModel.forward (audio_proj.py:162-170); ExpProjModel (:181-189) is the same MLP."""
    x = F.relu(linear(sd, _k(p, "proj1"), x))
    x = F.relu(linear(sd, _k(p, "proj2"), x))
    return linear(sd, _k(p, "proj3"), x)


def pose_guider(sd: SD, p: str, cond, n_blocks: int = 6):
    """PoseGuider.forward (pose_guider.py:63-73): InflatedConv3d = Conv2d per frame (:17-25)."""
    b, c, f, h, w = cond.shape

    def conv(name, x, stride=1):
        y = F.conv2d(x, sd[_k(p, name + ".weight")], sd[_k(p, name + ".bias")], stride=stride, padding=1)
        return y

    x = cond.permute(0, 2, 1, 3, 4).reshape(b * f, c, h, w)
    x = F.silu(conv("conv_in", x))
    for i in range(n_blocks):
        x = F.silu(conv(f"blocks.{i}", x, stride=1 if i % 2 == 0 else 2))
    x = conv("conv_out", x)
    return x.reshape(b, f, *x.shape[1:]).permute(0, 2, 1, 3, 4)


# ============================================================================ VAE
# diffusers 0.29.2 AutoencoderKLTemporalDecoder (Inference.py:41-44; used at pipeline:235-290, :520-536,
# :766). diffusers is absent here: restated from the pinned version's published source.
def vae_resnet2d(sd: SD, p: str, x, eps=1e-6):
    """ResnetBlock2D with temb_channels=None (resnet.py)."""
    h = F.silu(group_norm(sd, p + ".norm1", x, eps))
    h = F.conv2d(h, sd[p + ".conv1.weight"], sd[p + ".conv1.bias"], padding=1)
    h = F.silu(group_norm(sd, p + ".norm2", h, eps))
    h = F.conv2d(h, sd[p + ".conv2.weight"], sd[p + ".conv2.bias"], padding=1)
    if p + ".conv_shortcut.weight" in sd:
        x = F.conv2d(x, sd[p + ".conv_shortcut.weight"], sd[p + ".conv_shortcut.bias"])
    return x + h


def vae_temporal_resnet(sd: SD, p: str, x, eps=1e-5):
    """TemporalResnetBlock with temb None on (B, C, F, H, W)."""
    h = F.silu(group_norm(sd, p + ".norm1", x, eps))
    h = F.conv3d(h, sd[p + ".conv1.weight"], sd[p + ".conv1.bias"], padding=(1, 0, 0))
    h = F.silu(group_norm(sd, p + ".norm2", h, eps))
    h = F.conv3d(h, sd[p + ".conv2.weight"], sd[p + ".conv2.bias"], padding=(1, 0, 0))
    return x + h


def vae_st_resblock(sd: SD, p: str, x, num_frames):
    """SpatioTemporalResBlock(temb None, eps 1e-6, temporal_eps 1e-5, merge 'learned',
    switch_spatial_to_temporal_mix=True): AlphaBlender alpha = 1 - sigmoid(mix_factor)."""
    h = vae_resnet2d(sd, p + ".spatial_res_block", x, 1e-6)
    bf, c, hh, ww = h.shape
    b = bf // num_frames
    h5 = h.reshape(b, num_frames, c, hh, ww).permute(0, 2, 1, 3, 4)
    t = vae_temporal_resnet(sd, p + ".temporal_res_block", h5, 1e-5)
    a = 1.0 - torch.sigmoid(sd[p + ".time_mixer.mix_factor"])
    out = a * h5 + (1.0 - a) * t
    return out.permute(0, 2, 1, 3, 4).reshape(bf, c, hh, ww)


def vae_attention(sd: SD, p: str, x, eps=1e-6):
    """Attention(heads=1, dim_head=C, norm_num_groups=32, residual_connection, bias) under AttnProcessor2_0
    on a 4-D input (attention_processor.py:1528-1605 semantics)."""
    B, C, H, W = x.shape
    h = x.view(B, C, H * W)
    h = group_norm(sd, p + ".group_norm", h, eps).transpose(1, 2)
    q, k, v = (linear(sd, p + n, h) for n in (".to_q", ".to_k", ".to_v"))
    o = F.scaled_dot_product_attention(q[:, None], k[:, None], v[:, None])[:, 0]
    o = linear(sd, p + ".to_out.0", o).transpose(1, 2).reshape(B, C, H, W)
    return o + x


def vae_decode(sd: SD, z, num_frames, p: str = "decoder", n_up: int = 4, layers_per_block: int = 2):
    """AutoencoderKLTemporalDecoder.decode -> TemporalDecoder.forward (image_only_indicator zeros)."""
    x = F.conv2d(z, sd[p + ".conv_in.weight"], sd[p + ".conv_in.bias"], padding=1)
    x = vae_st_resblock(sd, p + ".mid_block.resnets.0", x, num_frames)
    for i in range(1, layers_per_block):
        x = vae_attention(sd, p + f".mid_block.attentions.{i - 1}", x)
        x = vae_st_resblock(sd, p + f".mid_block.resnets.{i}", x, num_frames)
    for u in range(n_up):
        for r in range(layers_per_block + 1):
            x = vae_st_resblock(sd, p + f".up_blocks.{u}.resnets.{r}", x, num_frames)
        if p + f".up_blocks.{u}.upsamplers.0.conv.weight" in sd:
            x = upsample_2d(sd, p + f".up_blocks.{u}.upsamplers.0", x)
    x = F.silu(group_norm(sd, p + ".conv_norm_out", x, 1e-6))
    x = F.conv2d(x, sd[p + ".conv_out.weight"], sd[p + ".conv_out.bias"], padding=1)
    bf, c, hh, ww = x.shape
    x = x.reshape(bf // num_frames, num_frames, c, hh, ww).permute(0, 2, 1, 3, 4)
    x = F.conv3d(x, sd[p + ".time_conv_out.weight"], sd[p + ".time_conv_out.bias"], padding=(1, 0, 0))
    return x.permute(0, 2, 1, 3, 4).reshape(bf, c, hh, ww)


def vae_encode_moments(sd: SD, x, p: str = "encoder", n_down: int = 4, layers_per_block: int = 2):
    """Encoder.forward + quant_conv -> moments (B, 8, H/8, W/8); latent_dist.mean = moments[:, :4]."""
    x = F.conv2d(x, sd[p + ".conv_in.weight"], sd[p + ".conv_in.bias"], padding=1)
    for d in range(n_down):
        for r in range(layers_per_block):
            x = vae_resnet2d(sd, p + f".down_blocks.{d}.resnets.{r}", x, 1e-6)
        q = p + f".down_blocks.{d}.downsamplers.0.conv"
        if q + ".weight" in sd:   # Downsample2D(padding=0): pad right/bottom by one, conv stride 2
            x = F.conv2d(F.pad(x, (0, 1, 0, 1)), sd[q + ".weight"], sd[q + ".bias"], stride=2)
    x = vae_resnet2d(sd, p + ".mid_block.resnets.0", x, 1e-6)
    x = vae_attention(sd, p + ".mid_block.attentions.0", x)
    x = vae_resnet2d(sd, p + ".mid_block.resnets.1", x, 1e-6)
    x = F.silu(group_norm(sd, p + ".conv_norm_out", x, 1e-6))
    x = F.conv2d(x, sd[p + ".conv_out.weight"], sd[p + ".conv_out.bias"], padding=1)
    return F.conv2d(x, sd["quant_conv.weight"], sd["quant_conv.bias"])


# ============================================================================ Whisper-tiny encoder
def whisper_encoder_hidden_states(sd: SD, x, heads: int = 6, n_layers: int = 4):
    """transformers WhisperEncoder (4.40.2, requirements.txt:11; called at Inference.py:453) with
    output_hidden_states: (input of every layer, final LayerNorm output)."""
    h = F.gelu(F.conv1d(x, sd["conv1.weight"], sd["conv1.bias"], padding=1))
    h = F.gelu(F.conv1d(h, sd["conv2.weight"], sd["conv2.bias"], stride=2, padding=1)).permute(0, 2, 1)
    h = h + sd["embed_positions.weight"][:h.shape[1]]
    states = []
    for i in range(n_layers):
        p = f"layers.{i}"
        states.append(h)
        r = h
        n = layer_norm(sd, p + ".self_attn_layer_norm", h)
        B, S, C = n.shape
        hd = C // heads
        q = (linear(sd, p + ".self_attn.q_proj", n) * hd ** -0.5).view(B, S, heads, hd).transpose(1, 2)
        k = F.linear(n, sd[p + ".self_attn.k_proj.weight"]).view(B, S, heads, hd).transpose(1, 2)
        v = linear(sd, p + ".self_attn.v_proj", n).view(B, S, heads, hd).transpose(1, 2)
        a = torch.softmax(q @ k.transpose(-1, -2), -1) @ v
        h = r + linear(sd, p + ".self_attn.out_proj", a.transpose(1, 2).reshape(B, S, C))
        r = h
        f = F.gelu(linear(sd, p + ".fc1", layer_norm(sd, p + ".final_layer_norm", h)))
        h = r + linear(sd, p + ".fc2", f)
    states.append(layer_norm(sd, "layer_norm", h))
    return tuple(states)


# ============================================================================ scheduler + loop
def euler_karras_tables(num_inference_steps: int = 25, sigma_min: float = 0.002, sigma_max: float = 700.0,
                        rho: float = 7.0):
    """diffusers 0.29.2 EulerDiscreteScheduler.set_timesteps with use_karras_sigmas=True,
    timestep_type='continuous', prediction_type='v_prediction' (SVD-XT scheduler_config):
    sigmas (steps+1, last 0) and timesteps 0.25*ln(sigma)."""
    ramp = np.linspace(0, 1, num_inference_steps)
    min_inv_rho = sigma_min ** (1 / rho)
    max_inv_rho = sigma_max ** (1 / rho)
    sigmas = (max_inv_rho + ramp * (min_inv_rho - max_inv_rho)) ** rho
    sigmas = torch.from_numpy(sigmas).to(dtype=torch.float32)
    timesteps = torch.Tensor([0.25 * s.log() for s in sigmas])
    sigmas = torch.cat([sigmas, torch.zeros(1)])
    return sigmas, timesteps


def euler_step_v(model_output, sigma, sigma_next, sample):
    """EulerDiscreteScheduler.step, v-prediction, s_churn = 0 (mirror scheduling_euler_discrete.py:141-207)."""
    sample = sample.float()
    x0 = model_output * (-sigma / (sigma ** 2 + 1) ** 0.5) + (sample / (sigma ** 2 + 1))
    derivative = (sample - x0) / sigma
    return sample + derivative * (sigma_next - sigma)


def denoise_loop(unet_fn, latents_all, image_latents, image_embeddings, audio_prompts, vasa_prompts, pose_fea,
                 added_time_ids, masks: List[torch.Tensor], gate, num_frames: int, frames_per_batch: int,
                 overlap: int, shift_offset: int, guidance, num_inference_steps: int = 25,
                 sigma_min=0.002, sigma_max=700.0, resume=None, on_step=None):
    """Pose2VideoLongSVDPipeline.__call__ step x window loop (pipeline_svd_audio_adapter_motionexp_idembed_
    vasa_two_ip.py:670-756). Tensor shapes are the pipeline's after CFG stacking:
      latents_all (1, T, 4, h, w), image_latents (4, T, 4, h, w), image_embeddings (4, T, 1, 1024),
      audio_prompts (4, T, 32, 1024), vasa_prompts (4, T, 1, 1024), pose_fea (1, N or T, 320, h, w), T = N + fpb.
    unet_fn(sample, t, ehs, added_time_ids, spatial_condition, cak) -> (4, fpb, 4, h, w).
    guidance: (g1, g2, g3), or one such triple per step (the pipeline's linspace schedules, :640-657).
    resume=(i0, latents_all) restarts at step i0 (the shift is a function of the step index, :752-753);
    on_step(i, latents_all) is called after every step (long CPU runs checkpoint through it)."""
    sigmas, timesteps = euler_karras_tables(num_inference_steps, sigma_min, sigma_max)
    per_step = isinstance(guidance[0], (tuple, list))
    T = num_frames + frames_per_batch
    i0 = 0
    if resume is not None:
        i0, latents_all = resume
    shift = (i0 * shift_offset) % frames_per_batch
    for i, t in enumerate(timesteps):
        if i < i0:
            continue
        g1, g2, g3 = guidance[i] if per_step else guidance
        pred = torch.zeros_like(latents_all)
        counter = torch.zeros((latents_all.shape[0], T, 1, 1, 1))
        for index_start in range(0, T, frames_per_batch - overlap):
            index_start -= shift
            idx_list = [(j % T) for j in range(index_start, index_start + frames_per_batch)]
            lat = latents_all[:, idx_list]
            # indice_slice wraps every tensor by its OWN frame count (pipeline:687-693): pose_fea has the
            # N pose frames, everything else T = N + fpb
            pose = pose_fea[:, [j % pose_fea.shape[1] for j in range(index_start, index_start + frames_per_batch)]]
            pose = pose.repeat(4, 1, 1, 1, 1)
            img = image_latents[:, idx_list]
            ide = image_embeddings[:, idx_list]
            aud = audio_prompts[:, idx_list]
            vas = vasa_prompts[:, idx_list]
            face_mask, mouth_mask, exp_mask = masks          # pipeline:636-646, 702-711
            if gate[0] == 1 and gate[1] == 1:
                mask_list = [mouth_mask, exp_mask]
            elif gate[0] == 1 and gate[1] == 0:
                mask_list = [face_mask, torch.zeros_like(face_mask)]
            else:
                mask_list = [torch.zeros_like(face_mask), face_mask]
            sigma = sigmas[i]
            inp = torch.cat([lat] * 4) / ((sigma ** 2 + 1) ** 0.5)
            inp = torch.cat([inp, img], dim=2)
            ehs = (ide.flatten(0, 1), [aud.flatten(0, 1) * gate[0], vas.flatten(0, 1) * gate[1]])
            noise = unet_fn(inp, t, ehs, added_time_ids, pose, {"ip_adapter_masks": mask_list})
            u, dav, dv, c = noise.chunk(4)
            eps = u + g1 * (dav - u) + g2 * (dv - dav) + g3 * (c - dv)
            lat = euler_step_v(eps, sigma, sigmas[i + 1], lat)
            for j in range(frames_per_batch):
                pidx = (index_start + j) % T
                pred[:, pidx] += lat[:, j]
                counter[:, pidx] += 1
        shift = (shift + shift_offset) % frames_per_batch
        latents_all = pred / counter
        if on_step is not None:
            on_step(i, latents_all)
    return latents_all
