"""Whisper-tiny audio encoder and the reference's audio windowing on HIP.

Reference: Inference.py:179 (``WhisperModel.from_pretrained(whisper-tiny)``), :444-460 (30 s windows of
3000 mel frames -> ``wav_enc.encoder(..., output_hidden_states=True).hidden_states`` stacked on dim 2,
trimmed to 2 tokens per video frame, zero-padded 4 in front / 6 behind) and :523-524 (each output
frame i takes the 10-token clip ``[2*step*i, 2*step*i + 10)`` into AudioProjModel). The encoder is
transformers' WhisperEncoder (pinned 4.40.2, requirements.txt:11; installed here 5.15): conv1 (k3) ->
GELU -> conv2 (k3, stride 2) -> GELU -> + positions -> pre-LN blocks (6-head SDPA, q scaled by
head_dim^-0.5 before the product, k without bias; GELU MLP) -> final LayerNorm. hidden_states follows
4.40.2: (embeddings, layer 0..L-2 outputs, LayerNorm(layer L-1 output)).

MI355X mapping: conv1 / conv2 are the direct-conv kernel as H = 1 convolutions with GELU fused; the
position add is fused into the first LayerNorm (which also emits the sum); q/k/v is one GEMM;
attention is the flash kernel (head_dim 64, ragged 1500 keys, its 1/8 scale = Whisper's q scale);
out-proj / fc2 carry the residual in their epilogues, fc1 the GELU.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import torch
import torch.nn as nn

from . import ops
from .modules import LayerNorm, Linear, Packed, _bf, _f32


class _Conv1d(nn.Conv1d, Packed):
    def wd(self):
        def f():
            w = self.weight.detach().float()
            w4 = torch.zeros(w.shape[0], w.shape[1], 3, 3, device=w.device)
            w4[:, :, 1, :] = w                       # H = 1: only the middle kernel row sees data
            return ops.pack_conv_direct(w4)
        return self._pk("wd", f)

    def b(self):
        return self._pk("b", lambda: _f32(self.bias))


class WhisperAttention(Packed):
    def __init__(self, embed_dim, num_heads):
        super().__init__()
        self.embed_dim, self.num_heads = embed_dim, num_heads
        self.head_dim = embed_dim // num_heads
        self.scaling = self.head_dim ** -0.5
        self.k_proj = Linear(embed_dim, embed_dim, bias=False)
        self.v_proj = Linear(embed_dim, embed_dim, bias=True)
        self.q_proj = Linear(embed_dim, embed_dim, bias=True)
        self.out_proj = Linear(embed_dim, embed_dim, bias=True)

    def packs(self):
        def f():
            w = torch.cat([self.q_proj.weight, self.k_proj.weight, self.v_proj.weight], 0)
            b = torch.cat([self.q_proj.bias.detach(), torch.zeros_like(self.q_proj.bias.detach()),
                           self.v_proj.bias.detach()])
            return _bf(w), _f32(b)
        return self._pk("qkv", f)


class WhisperEncoderLayer(nn.Module):
    def __init__(self, d_model, heads, ffn_dim):
        super().__init__()
        self.self_attn = WhisperAttention(d_model, heads)
        self.self_attn_layer_norm = LayerNorm(d_model)
        self.fc1 = Linear(d_model, ffn_dim)
        self.fc2 = Linear(ffn_dim, d_model)
        self.final_layer_norm = LayerNorm(d_model)


@dataclass
class BaseModelOutput:
    last_hidden_state: torch.Tensor
    hidden_states: Optional[Tuple[torch.Tensor, ...]] = None


class WhisperEncoder(nn.Module):
    """transformers WhisperEncoder parameter names (``conv1``, ``conv2``, ``embed_positions``,
    ``layers.N.*``, ``layer_norm``); whisper-tiny defaults."""

    def __init__(self, num_mel_bins=80, d_model=384, encoder_layers=4, encoder_attention_heads=6,
                 encoder_ffn_dim=1536, max_source_positions=1500):
        super().__init__()
        if d_model // encoder_attention_heads != 64:
            raise ValueError("the HIP attention kernel needs head_dim 64")
        self.num_mel_bins, self.d_model, self.max_source_positions = num_mel_bins, d_model, max_source_positions
        self.heads = encoder_attention_heads
        self.conv1 = _Conv1d(num_mel_bins, d_model, kernel_size=3, padding=1)
        self.conv2 = _Conv1d(d_model, d_model, kernel_size=3, stride=2, padding=1)
        self.embed_positions = nn.Embedding(max_source_positions, d_model)
        self.layers = nn.ModuleList([WhisperEncoderLayer(d_model, encoder_attention_heads, encoder_ffn_dim)
                                     for _ in range(encoder_layers)])
        self.layer_norm = LayerNorm(d_model)

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

    def forward(self, input_features: torch.Tensor, output_hidden_states: bool = False, return_dict: bool = True):
        B, nmel, L = input_features.shape
        expected = self.max_source_positions * 2
        if L != expected:
            raise ValueError(f"Whisper expects the mel input features to be of length {expected}, but found {L}. "
                             f"Make sure to pad the input mel features to {expected}.")
        S, C = self.max_source_positions, self.d_model
        x = ops.nchw_to_tokens(input_features.float().reshape(B, nmel, 1, L))                 # (B*L, 80)
        x = ops.conv_direct(x, self.conv1.wd(), self.conv1.b(), B=B, H=1, W=L, act=ops.ACT_GELU)
        x = ops.conv_direct(x, self.conv2.wd(), self.conv2.b(), B=B, H=1, W=L, stride=2, act=ops.ACT_GELU)
        pos = self.embed_positions.weight.detach().to(torch.bfloat16).contiguous()
        states = []
        h = torch.empty_like(x)
        n = torch.empty_like(x)
        l0 = self.layers[0].self_attn_layer_norm
        g, b = l0.gb()
        for bi in range(B):                                   # h = emb + pos and n = LN(h) in one pass
            r = slice(bi * S, (bi + 1) * S)
            ops.layernorm(x[r], g, b, l0.eps, add=pos, add_div=1, sum_out=h[r], out=n[r])
        for li, layer in enumerate(self.layers):
            if output_hidden_states:
                states.append(h)
            if li > 0:
                g, b = layer.self_attn_layer_norm.gb()
                n = ops.layernorm(h, g, b, layer.self_attn_layer_norm.eps)
            at = layer.self_attn
            w_qkv, b_qkv = at.packs()
            qkv = ops.gemm(n, w_qkv, bias=b_qkv)
            a = ops.flash_attn(qkv, B, S, self.heads)
            h = ops.gemm(a, at.out_proj.w(), bias=at.out_proj.b(), residual=h)
            g, b = layer.final_layer_norm.gb()
            n2 = ops.layernorm(h, g, b, layer.final_layer_norm.eps)
            f = ops.gemm(n2, layer.fc1.w(), bias=layer.fc1.b(), act=ops.ACT_GELU)
            h = ops.gemm(f, layer.fc2.w(), bias=layer.fc2.b(), residual=h)
        g, b = self.layer_norm.gb()
        last = ops.layernorm(h, g, b, self.layer_norm.eps)
        view = lambda t: t.view(B, S, C)                      # noqa: E731
        hs = tuple(view(t) for t in states) + (view(last),) if output_hidden_states else None
        return BaseModelOutput(last_hidden_state=view(last), hidden_states=hs)


class WhisperModelEncoderOnly(nn.Module):
    """The part of transformers' WhisperModel the reference uses: ``.encoder``. Loads a WhisperModel
    state dict (``encoder.*`` keys; decoder keys are ignored)."""

    def __init__(self, **kw):
        super().__init__()
        self.encoder = WhisperEncoder(**kw)

    def load_whisper_state_dict(self, sd):
        enc = {k[len("encoder."):]: v for k, v in sd.items() if k.startswith("encoder.")}
        return self.encoder.load_state_dict(enc, strict=True)


def audio_prompts_from_features(encoder: WhisperEncoder, audio_feature: torch.Tensor, audio_len: int,
                                window: int = 3000) -> torch.Tensor:
    """Inference.py:449-460: (1, 80, n*3000) mel -> (1, 2*audio_len + 10, L+1, 384) fp32 hidden-state
    stacks (4 zero tokens in front, 6 behind)."""
    prompts = []
    for i in range(0, audio_feature.shape[-1], window):
        hs = encoder(audio_feature[:, :, i:i + window], output_hidden_states=True).hidden_states
        prompts.append(torch.stack([t.float() for t in hs], dim=2))
    p = torch.cat(prompts, dim=1)[:, :audio_len * 2]
    return torch.cat([torch.zeros_like(p[:, :4]), p, torch.zeros_like(p[:, :6])], 1)


def audio_clips(audio_prompts: torch.Tensor, n_frames: int, step: int = 2) -> torch.Tensor:
    """Per output frame i: the 10-token clip audio_prompts[:, 2*step*i : 2*step*i + 10]
    (Inference.py:523) -> (1, n_frames, 10, L+1, 384), AudioProjModel's input layout."""
    return torch.stack([audio_prompts[0, i * 2 * step:i * 2 * step + 10] for i in range(n_frames)], 0)[None]
