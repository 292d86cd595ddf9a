"""Seeded synthetic weights for the UNet (no checkpoints are available offline).

Weights depend only on (seed, parameter name, shape): one CPU ``torch.Generator`` per parameter,
seeded from the seed and a stable hash of the name, so any subset of the model (or the oracle's
state dict) can be regenerated identically on any host. Scales keep activations O(1) through the
~80 residual blocks: linear/conv weights ~ N(0, 1/fan_in), small biases, norms near identity, Mamba
parameters from the reference's own initialisers (S4D-real A, D = 1, dt in [1e-3, 1e-1]).
"""
from __future__ import annotations

import math
import zlib
from typing import Dict, Iterable, Tuple

import torch


def _gen(seed: int, name: str) -> torch.Generator:
    return torch.Generator().manual_seed((seed * 1000003 + zlib.crc32(name.encode())) & 0x7FFFFFFFFFFF)


def synthetic_tensor(seed: int, name: str, shape: Tuple[int, ...]) -> torch.Tensor:
    g = _gen(seed, name)
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "A_logs":
        t = torch.log(torch.arange(1, shape[-1] + 1, dtype=torch.float32)).expand(shape).clone()
        t += 0.1 * torch.randn(shape, generator=g)
    elif leaf == "Ds":
        t = 1.0 + 0.1 * torch.randn(shape, generator=g)
    elif leaf == "dt_projs_bias":
        dt = torch.exp(torch.rand(shape, generator=g) * (math.log(0.1) - math.log(0.001)) + math.log(0.001))
        t = dt + torch.log(-torch.expm1(-dt))
    elif leaf == "dt_projs_weight":
        t = (torch.rand(shape, generator=g) * 2 - 1) * shape[-1] ** -0.5
    elif leaf == "mix_factor":
        t = 0.5 * torch.randn(shape, generator=g)
    elif len(shape) == 1 and "norm" in name and leaf == "weight":
        t = 1.0 + 0.05 * torch.randn(shape, generator=g)
    elif len(shape) == 1:
        t = 0.05 * torch.randn(shape, generator=g)
    else:
        fan_in = int(math.prod(shape[1:]))
        t = torch.randn(shape, generator=g) / math.sqrt(fan_in)
    return t.float().contiguous()


def synthetic_state_dict(seed: int, shapes: Dict[str, Tuple[int, ...]]) -> Dict[str, torch.Tensor]:
    return {k: synthetic_tensor(seed, k, tuple(v)) for k, v in shapes.items()}


@torch.no_grad()
def init_synthetic_(module: torch.nn.Module, seed: int = 72589, names: Iterable[str] = None) -> torch.nn.Module:
    """Overwrite every parameter of ``module`` (reference names) with its synthetic value."""
    params = dict(module.named_parameters())
    for k in (names if names is not None else params):
        p = params[k]
        p.copy_(synthetic_tensor(seed, k, tuple(p.shape)).to(p.device, p.dtype))
    if hasattr(module, "invalidate_kernel_cache"):
        module.invalidate_kernel_cache()
    return module
