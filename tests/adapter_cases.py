"""Golden cases for the conditioning adapters (shared by tools/gen_golden_adapters.py and the tests).

Configurations follow Inference.py:72-78; inputs are seeded N(0, 1) tensors of the shapes the
pipeline feeds (audio windows (bz, f, 10, 5, 384) from Inference.py:523-524; ID embedding
(1, 1, 512), pipeline:145; VASA expression (n, 512), Inference.py:500-503; pose images
(b, 3, f, H, W) in [0, 1], pipeline:617-636).
"""
from __future__ import annotations

import torch

ADAPTER_CASES = {
    "audio_proj": dict(cls="AudioProjModel", seed=31, in_shape=[1, 3, 10, 5, 384],
                       kwargs=dict(seq_len=10, blocks=5, channels=384, intermediate_dim=1024, output_dim=1024,
                                   context_tokens=32)),
    "id_proj": dict(cls="IDProjModel", seed=32, in_shape=[1, 1, 512],
                    kwargs=dict(input_dim=512, output_dim=1024, intermediate_dim=1024)),
    "vasa_proj": dict(cls="VasaProjModel", seed=33, in_shape=[4, 512], kwargs=dict(input_dim=512, output_dim=1024)),
    "pose_guider": dict(cls="PoseGuider", seed=34, in_shape=[1, 3, 2, 64, 96],
                        kwargs=dict(conditioning_embedding_channels=320, block_out_channels=[16, 32, 96, 256])),
    # odd spatial size: stride-2 layers with H, W not divisible by 8 (ragged borders)
    "pose_guider_odd": dict(cls="PoseGuider", seed=35, in_shape=[1, 3, 3, 37, 50],
                            kwargs=dict(conditioning_embedding_channels=320, block_out_channels=[16, 32, 96, 256])),
}


def adapter_input(case) -> torch.Tensor:
    g = torch.Generator().manual_seed(case["seed"] + 500)
    x = torch.randn(*case["in_shape"], generator=g)
    if case["cls"] == "PoseGuider":
        x = torch.rand(*case["in_shape"], generator=g)
    return x
