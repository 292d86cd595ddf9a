"""Inputs of the full-length (25 Karras steps, sigma 700 -> 0.002) sampler-loop parity cases, shared by
tools/gen_golden_loop.py (oracle fixtures) and tests/test_full_geometry_gpu.py.

The tiny full-topology UNet of __graft_entry__ (widths 64/128/128/128) keeps the oracle loop at
seconds; the conditioning is stacked exactly as the pipeline does (pipeline:162-200: ID [0,e,e,e],
image latents [0,l,l,l], audio [u,u,a,a], VASA [u,u,u,v], prompts gated at :724) so the HIP loop's
twin-branch elimination is active in modes 0 / 1, and the masks are partial so the masked IP /
Mamba paths run (face = centre box, mouth = lower half, expression = upper half)."""
import torch

N, FPB, H, W = 4, 2, 16, 32
SHIFT = 1
GATES = {"mode0": [1, 0], "mode1": [0, 1], "mode2": [1, 1]}
UNET_SEED = 9


def loop_inputs(seed: int = 31, pose_ch: int = 64):
    """pose_ch: the UNet's block_out_channels[0] (64 for the tiny UNet, 320 for the real-width one)."""
    g = torch.Generator().manual_seed(seed)
    T = N + FPB
    latents = 0.18215 * torch.randn(1, 1, 4, H, W, generator=g) + 700.0 * torch.randn(1, T, 4, H, W, generator=g)
    il = torch.randn(1, T, 4, H, W, generator=g)
    imgl = torch.cat([torch.zeros_like(il), il, il, il])
    e = torch.randn(1, T, 1, 1024, generator=g)
    ide = torch.cat([torch.zeros_like(e), e, e, e])
    a_u, a_c = torch.randn(1, T, 32, 1024, generator=g), torch.randn(1, T, 32, 1024, generator=g)
    aud = torch.cat([a_u, a_u, a_c, a_c])
    v_u, v_c = torch.randn(1, T, 1, 1024, generator=g), torch.randn(1, T, 1, 1024, generator=g)
    vas = torch.cat([v_u, v_u, v_u, v_c])
    pose = 0.1 * torch.randn(1, N, pose_ch, H, W, generator=g)     # N pose frames: indexed mod N
    added = torch.tensor([[12.5, 12.0, 20.0]] * 4)
    Hp, Wp = 8 * H, 8 * W
    face = torch.zeros(1, 1, Hp, Wp)
    face[..., Hp // 4: 3 * Hp // 4, Wp // 4: 3 * Wp // 4] = 1.0
    mouth = torch.zeros(1, 1, Hp, Wp)
    mouth[..., Hp // 2:, :] = 1.0
    masks = (face, mouth, 1.0 - mouth)
    return latents, imgl, ide, aud, vas, pose, added, masks


def oracle_loop(sd, cfg, gate, steps=25, pose_ch: int = 64, dtype=None):
    """dtype (torch.float16 / bfloat16): the oracle with every op's inputs and outputs rounded to it
    (oracle.precision.rounded; sd must already be rounded by precision.round_state_dict)."""
    import contextlib
    from oracle import reference_cpu as ref
    latents, imgl, ide, aud, vas, pose, added, masks = loop_inputs(pose_ch=pose_ch)
    if dtype is not None:
        from oracle import precision
        ctx = precision.rounded(dtype)
    else:
        ctx = contextlib.nullcontext()

    def unet_fn(sample, t, ehs, added_ids, sc, cak):
        return ref.unet_forward(sd, sample, t, ehs, added_ids, sc, cak, ip_scale=(1.25, 1.25),
                                cfg=dict(block_out_channels=cfg["block_out_channels"],
                                         num_attention_heads=cfg["num_attention_heads"]))

    with ctx:
        return ref.denoise_loop(unet_fn, latents, imgl, ide, aud, vas, pose, added, list(masks), gate, N, FPB,
                                overlap=0, shift_offset=SHIFT, guidance=(2.0, 7.5, 3.0), num_inference_steps=steps)


FULL_CFG = dict(block_out_channels=[320, 640, 1280, 1280], num_attention_heads=[5, 10, 20, 20])
