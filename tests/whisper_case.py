"""The Whisper-tiny golden case (shared by tools/gen_golden_whisper.py and tests/test_whisper.py)."""
import torch

SEED = 71
WHISPER_TINY = dict(d_model=384, encoder_layers=4, encoder_attention_heads=6, encoder_ffn_dim=1536, num_mel_bins=80,
                    max_source_positions=1500)


def mel_input() -> torch.Tensor:
    return torch.randn(1, 80, 3000, generator=torch.Generator().manual_seed(SEED + 1))
