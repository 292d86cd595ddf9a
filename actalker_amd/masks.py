"""Host-side mask preprocessing (computed once per mask tensor and token count, then cached).

The reference recomputes these on every block call: IP-adapter region weights
(``IPAdapterMaskProcessor.downsample``, diffusers 0.29.2, called at attention_processor.py:2892)
and Mamba token selection ``downsample(...).view(-1).int().nonzero()`` (mamba_layer.py:1962-1981),
which forces a device->host sync each time. Masks are constant over a sampler run, so here they
are evaluated once on the host in fp32 and uploaded as small index / weight arrays.
"""
from __future__ import annotations

import math
import weakref
from typing import Dict, Tuple

import torch
import torch.nn.functional as F


def mask_downsample(mask: torch.Tensor, batch_size: int, num_queries: int, value_embed_dim: int) -> torch.Tensor:
    """Restatement of diffusers 0.29.2 ``IPAdapterMaskProcessor.downsample`` (mask: (1, H, W))."""
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


class MaskInfo:
    """Per (mask, token count) data: IP weights and Mamba selection."""

    def __init__(self, weights: torch.Tensor, sel: torch.Tensor, S: int, device):
        self.S = S
        w = weights.reshape(-1)[:S].float()
        self.all_one = bool(torch.all(w == 1.0))
        self.all_zero = bool(torch.all(w == 0.0))
        self.weights = w.to(device)
        self.n_sel = int(sel.numel())
        self.identity = self.n_sel == S and bool(torch.all(sel == torch.arange(S)))
        self.idx = sel.to(torch.int32).to(device)
        pos = torch.full((S,), -1, dtype=torch.int32)
        pos[sel] = torch.arange(self.n_sel, dtype=torch.int32)
        self.pos = pos.to(device)


# keyed by the mask tensor object itself (weakly): an entry dies with its tensor, so a new mask
# allocated at a recycled address can never hit a stale entry; in-place edits bump _version
_CACHE: Dict[int, Tuple["weakref.ref", int, Dict]] = {}


def mask_info(mask: torch.Tensor, S: int, device) -> MaskInfo:
    """mask: (1, 1, H, W) (the pipeline's ``ip_adapter_masks`` entries)."""
    version = getattr(mask, "_version", 0)
    ent = _CACHE.get(id(mask))
    if ent is None or ent[0]() is not mask or ent[1] != version:
        if len(_CACHE) > 64:
            for k in [k for k, e in _CACHE.items() if e[0]() is None]:
                del _CACHE[k]
        ent = (weakref.ref(mask), version, {})
        _CACHE[id(mask)] = ent
    key = (S, str(device))
    hit = ent[2].get(key)
    if hit is not None:
        return hit
    m = mask.detach().to("cpu", torch.float32)[:, 0]            # (1, H, W)
    weights = mask_downsample(m, 1, S, 1)                       # IP-adapter weights (float)
    sel = weights.view(-1).int().nonzero().view(-1)             # Mamba int() truncation
    info = MaskInfo(weights, sel, S, device)
    ent[2][key] = info
    return info
