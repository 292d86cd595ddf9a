"""Golden vectors for the Whisper-tiny audio encoder from transformers' own WhisperEncoder.

The reference calls ``WhisperModel.from_pretrained(whisper-tiny).encoder(mel, output_hidden_states=True)
.hidden_states`` (Inference.py:179, :453) with transformers 4.40.2 (requirements.txt:11). transformers
5.15 is installed here; its WhisperEncoder math is the same (conv1/conv2 + GELU, positions, pre-LN
blocks, final LayerNorm). 5.x records hidden states through hooks, so the tuple is assembled here in
4.40.2's convention: the input of every layer, then the final LayerNorm output.

Weights: ``actalker_amd.synthetic.synthetic_state_dict(seed, shapes)`` over the encoder's state dict
(whisper-tiny shapes); input mel: seeded N(0, 1) (1, 80, 3000). The fixture keeps every 10th token
row of each hidden state plus per-state full sums (the full tensors are 11.5 MB).

Writes tests/golden/whisper_tiny.safetensors.   Usage:  python tools/gen_golden_whisper.py
"""
from __future__ import annotations

import os
import sys

import torch
from safetensors.torch import save_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from actalker_amd.synthetic import synthetic_state_dict  # noqa: E402
from tests.whisper_case import SEED, mel_input, WHISPER_TINY  # noqa: E402


def main():
    from transformers import WhisperConfig, WhisperModel
    cfg = WhisperConfig(**WHISPER_TINY, decoder_layers=1, decoder_attention_heads=6, decoder_ffn_dim=256)
    enc = WhisperModel(cfg).encoder.eval()
    sd = synthetic_state_dict(SEED, {k: tuple(v.shape) for k, v in enc.state_dict().items()})
    enc.load_state_dict(sd, strict=True)
    inputs = []
    hooks = [layer.register_forward_pre_hook(lambda m, a: inputs.append(a[0].detach().clone()))
             for layer in enc.layers]
    x = mel_input()
    with torch.no_grad():
        last = enc(x).last_hidden_state
    for h in hooks:
        h.remove()
    states = inputs + [last]
    out = {"x_sum": x.sum().reshape(1)}
    for i, s in enumerate(states):
        out[f"h{i}_rows"] = s[0, ::10].contiguous()
        out[f"h{i}_sum"] = s.double().sum().float().reshape(1)
        out[f"h{i}_abs_sum"] = s.double().abs().sum().float().reshape(1)
    save_file(out, os.path.join(ROOT, "tests", "golden", "whisper_tiny.safetensors"))
    print(len(states), "hidden states", [tuple(s.shape) for s in states][:1], float(last.abs().mean()))


if __name__ == "__main__":
    main()
