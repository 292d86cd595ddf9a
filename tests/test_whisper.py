"""Whisper-tiny audio encoder + audio windowing (Inference.py:179, 444-460, 523).

Pinning: tests/golden/whisper_tiny.safetensors comes from transformers' own WhisperEncoder
(tools/gen_golden_whisper.py; transformers 5.15 here, the reference pins 4.40.2 whose encoder math is
the same) with ``actalker_amd.synthetic`` weights. The fixture holds every 10th token row of the 5
hidden states plus full-tensor sums. The CPU oracle must match to fp32 rounding; the HIP path
(bf16 activations) within relative L2 3e-2 per hidden state.
"""
import os

import pytest
import torch
from safetensors.torch import load_file

from actalker_amd.synthetic import synthetic_state_dict
from oracle import reference_cpu as ref
from tests.whisper_case import SEED, WHISPER_TINY, mel_input

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "whisper_tiny.safetensors")


def _weights():
    from actalker_amd.whisper import WhisperEncoder
    m = WhisperEncoder(**WHISPER_TINY)
    sd = synthetic_state_dict(SEED, {k: tuple(v.shape) for k, v in m.state_dict().items()})
    m.load_state_dict(sd, strict=True)
    return m, sd


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


def test_oracle_matches_transformers_golden():
    g = load_file(GOLD)
    x = mel_input()
    assert torch.allclose(x.sum().reshape(1), g["x_sum"])
    _, sd = _weights()
    with torch.no_grad():
        hs = ref.whisper_encoder_hidden_states(sd, x)
    assert len(hs) == 5
    for i, h in enumerate(hs):
        assert _rel(h[0, ::10], g[f"h{i}_rows"]) < 1e-5, i
        assert abs(h.double().abs().sum().item() / g[f"h{i}_abs_sum"].item() - 1) < 1e-5


def test_audio_windowing_shapes():
    from actalker_amd.whisper import audio_clips
    p = torch.arange(2 * 7 + 10, dtype=torch.float32).view(1, -1, 1, 1).expand(1, 24, 5, 384)
    clips = audio_clips(p, n_frames=3, step=2)
    assert clips.shape == (1, 3, 10, 5, 384)
    assert clips[0, 1, 0, 0, 0].item() == 4.0 and clips[0, 2, 9, 0, 0].item() == 17.0


@pytest.mark.gpu
def test_whisper_encoder_gpu_matches_golden(dev):
    g = load_file(GOLD)
    m, _ = _weights()
    out = m.to(dev)(mel_input().to(dev), output_hidden_states=True)
    torch.cuda.synchronize()
    assert len(out.hidden_states) == 5
    for i, h in enumerate(out.hidden_states):
        assert h.shape == (1, 1500, 384)
        err = _rel(h[0, ::10].cpu(), g[f"h{i}_rows"])
        assert err < 3e-2, f"hidden state {i}: rel-L2 {err:.3e}"
    assert torch.equal(out.last_hidden_state, out.hidden_states[-1])


@pytest.mark.gpu
def test_audio_prompts_pipeline_gpu(dev):
    """Two 30 s windows -> stacked hidden states, trimmed to 2*audio_len, padded 4 / 6 (Inference.py:449-460),
    and the 10-token clips into AudioProjModel (Inference.py:523-524)."""
    from actalker_amd.adapters import AudioProjModel
    from actalker_amd.whisper import audio_clips, audio_prompts_from_features
    m, sd = _weights()
    m = m.to(dev)
    feats = torch.cat([mel_input(), torch.randn(1, 80, 3000, generator=torch.Generator().manual_seed(3))], -1)
    audio_len = 1200
    p = audio_prompts_from_features(m, feats.to(dev), audio_len)
    assert p.shape == (1, 2 * audio_len + 10, 5, 384)
    assert torch.count_nonzero(p[:, :4]) == 0 and torch.count_nonzero(p[:, -6:]) == 0
    with torch.no_grad():
        w2 = ref.whisper_encoder_hidden_states(sd, feats[:, :, 3000:])
    want = torch.stack(w2, dim=2)[:, :2 * audio_len - 1500]
    assert _rel(p[:, 4 + 1500:4 + 2 * audio_len].cpu(), want) < 3e-2
    ap = AudioProjModel(seq_len=10, blocks=5, channels=384, intermediate_dim=1024, output_dim=1024,
                        context_tokens=32)
    ap.load_state_dict(synthetic_state_dict(5, {k: tuple(v.shape) for k, v in ap.state_dict().items()}))
    clips = audio_clips(p, n_frames=4, step=2)
    tok = ap.to(dev)(clips)
    assert tok.shape == (1, 4, 32, 1024) and torch.isfinite(tok.float()).all()
