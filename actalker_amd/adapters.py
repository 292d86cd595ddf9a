"""Conditioning adapters on the step before the denoising loop.

Drop-in counterparts of the reference's adapter modules, with their constructor arguments,
parameter names (``state_dict`` loads with ``strict=True``) and forward signatures:

  AudioProjModel   src/models/audio_adapter/audio_proj.py:40-130   (Inference.py:76)
  VasaProjModel    audio_proj.py:132-151                           (Inference.py:78)
  IDProjModel      audio_proj.py:153-170                           (Inference.py:77)
  PoseGuider       src/models/audio_adapter/pose_guider.py:28-73   (Inference.py:72-75)

Compute runs in libactalker_hip.so: the projection MLPs are MFMA GEMMs with bias + ReLU fused in
the epilogue and the LayerNorm kernel after them; PoseGuider's narrow convolutions (Cin = 3, 16,
32, 96) run on the direct-conv kernel with SiLU fused, its 256 -> 320 conv_out on the MFMA implicit
GEMM. Activations are bf16, accumulation fp32. Outputs are bf16 tensors in the reference's shapes
(PoseGuider: fp32 (b, C, f, h, w) like the reference's InflatedConv3d layout); ``forward_tokens``
returns the token-major rows the UNet consumes without a layout change.
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.nn as nn

from . import ops
from .modules import Linear, LayerNorm, Packed, _f32


class _AdapterBase(nn.Module):
    """Packed kernel-layout weights are dropped whenever parameters move or are reloaded."""

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

    @property
    def dtype(self):
        return next(self.parameters()).dtype


class AudioProjModel(_AdapterBase):
    def __init__(self, seq_len=5, blocks=12, channels=768, intermediate_dim=512, output_dim=768, context_tokens=32):
        super().__init__()
        self.seq_len, self.blocks, self.channels = seq_len, blocks, channels
        self.input_dim = seq_len * blocks * channels
        self.intermediate_dim, self.context_tokens, self.output_dim = intermediate_dim, context_tokens, output_dim
        self.proj1 = Linear(self.input_dim, intermediate_dim)
        self.proj2 = Linear(intermediate_dim, intermediate_dim)
        self.proj3 = Linear(intermediate_dim, context_tokens * output_dim)
        self.norm = LayerNorm(output_dim)

    def forward(self, audio_embeds: torch.Tensor) -> torch.Tensor:
        """(bz, f, w, b, c) -> (bz, f, context_tokens, output_dim) (audio_proj.py:103-130)."""
        bz, f = audio_embeds.shape[:2]
        x = audio_embeds.reshape(bz * f, -1).to(torch.bfloat16).contiguous()
        if x.shape[1] != self.input_dim:
            raise ValueError(f"AudioProjModel: expected {self.input_dim} features per frame, got {x.shape[1]}")
        h = ops.gemm(x, self.proj1.w(), bias=self.proj1.b(), act=ops.ACT_RELU)
        h = ops.gemm(h, self.proj2.w(), bias=self.proj2.b(), act=ops.ACT_RELU)
        t = ops.gemm(h, self.proj3.w(), bias=self.proj3.b())
        g, b = self.norm.gb()
        t = ops.layernorm(t.view(bz * f * self.context_tokens, self.output_dim), g, b, self.norm.eps)
        return t.view(bz, f, self.context_tokens, self.output_dim)


class VasaProjModel(_AdapterBase):
    def __init__(self, input_dim=512, output_dim=768):
        super().__init__()
        self.input_dim, self.output_dim = input_dim, output_dim
        self.proj1 = Linear(input_dim, output_dim)
        self.norm = LayerNorm(output_dim)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """(..., input_dim) -> (..., output_dim): LayerNorm(proj1(x)) (audio_proj.py:147-150)."""
        lead = x.shape[:-1]
        h = ops.gemm(x.reshape(-1, self.input_dim).to(torch.bfloat16).contiguous(), self.proj1.w(),
                     bias=self.proj1.b())
        g, b = self.norm.gb()
        return ops.layernorm(h, g, b, self.norm.eps).view(*lead, self.output_dim)


class _MLP3(_AdapterBase):
    """relu(proj1) -> relu(proj2) -> proj3 (IDProjModel audio_proj.py:153-170, ExpProjModel :172-189)."""

    def __init__(self, input_dim, output_dim, intermediate_dim):
        super().__init__()
        self.proj1 = Linear(input_dim, intermediate_dim)
        self.proj2 = Linear(intermediate_dim, intermediate_dim)
        self.proj3 = Linear(intermediate_dim, output_dim)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        lead = x.shape[:-1]
        h = x.reshape(-1, x.shape[-1]).to(torch.bfloat16).contiguous()
        h = ops.gemm(h, self.proj1.w(), bias=self.proj1.b(), act=ops.ACT_RELU)
        h = ops.gemm(h, self.proj2.w(), bias=self.proj2.b(), act=ops.ACT_RELU)
        h = ops.gemm(h, self.proj3.w(), bias=self.proj3.b())
        return h.view(*lead, h.shape[-1])


class IDProjModel(_MLP3):
    def __init__(self, input_dim=512, output_dim=768, intermediate_dim=768):
        super().__init__(input_dim, output_dim, intermediate_dim)


class ExpProjModel(_MLP3):
    def __init__(self, input_dim=512 + 6, output_dim=768, intermediate_dim=768):
        super().__init__(input_dim, output_dim, intermediate_dim)


class InflatedConv3d(nn.Conv2d, Packed):
    """Conv2d applied per frame of a (b, c, f, h, w) volume (pose_guider.py:17-25)."""

    def wd(self):
        return self._pk("wd", lambda: ops.pack_conv_direct(self.weight))

    def w3(self):
        from .modules import pack_conv3x3
        return self._pk("w3", lambda: pack_conv3x3(self.weight))

    def b(self):
        return self._pk("b", lambda: _f32(self.bias))

    def run(self, x, nfr, H, W, act):
        """x: NHWC rows (nfr*H*W, Cin) bf16 -> rows (nfr*Ho*Wo, Cout)."""
        s = self.stride[0]
        if self.in_channels % 64 == 0 and act == ops.ACT_NONE:
            return ops.conv3x3(x, self.w3(), nfr, H, W, stride=s, bias=self.b())
        return ops.conv_direct(x, self.wd(), self.b(), B=nfr, H=H, W=W, stride=s, act=act)


class PoseGuider(_AdapterBase):
    def __init__(self, conditioning_embedding_channels: int, conditioning_channels: int = 3,
                 block_out_channels: Tuple[int, ...] = (16, 32, 64, 128)):
        super().__init__()
        self.conv_in = InflatedConv3d(conditioning_channels, block_out_channels[0], kernel_size=3, padding=1)
        self.blocks = nn.ModuleList([])
        for i in range(len(block_out_channels) - 1):
            cin, cout = block_out_channels[i], block_out_channels[i + 1]
            self.blocks.append(InflatedConv3d(cin, cin, kernel_size=3, padding=1))
            self.blocks.append(InflatedConv3d(cin, cout, kernel_size=3, padding=1, stride=2))
        self.conv_out = InflatedConv3d(block_out_channels[-1], conditioning_embedding_channels, kernel_size=3,
                                       padding=1)
        with torch.no_grad():                      # zero_module (pose_guider.py:10-14, :56-63)
            for p in self.conv_out.parameters():
                p.zero_()

    def forward_tokens(self, conditioning: torch.Tensor):
        """(b, c, f, H, W) -> (rows (b*f*h*w, C) bf16, (b, f, h, w)) with h, w the output grid."""
        b, c, f, H, W = conditioning.shape
        # (b, c, [f h w]) -> rows (b, f, h, w) x c: the flattened (f, h, w) axis is the "pixel" axis
        x = ops.nchw_to_tokens(conditioning.reshape(b, c, f * H, W))
        nfr = b * f
        x = self.conv_in.run(x, nfr, H, W, ops.ACT_SILU)
        for blk in self.blocks:
            s = blk.stride[0]
            x = blk.run(x, nfr, H, W, ops.ACT_SILU)
            H, W = (H - 1) // s + 1, (W - 1) // s + 1
        x = self.conv_out.run(x, nfr, H, W, ops.ACT_NONE)
        return x, (b, f, H, W)

    def forward(self, conditioning: torch.Tensor) -> torch.Tensor:
        """(b, c, f, H, W) -> (b, C, f, H/8, W/8) fp32 (pose_guider.py:63-73)."""
        x, (b, f, h, w) = self.forward_tokens(conditioning)
        C = x.shape[1]
        return ops.tokens_to_nchw(x, b, f * h, w).view(b, C, f, h, w)
