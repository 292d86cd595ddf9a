"""Drop-in replacement for ``mamba_ssm.ops.selective_scan_interface.selective_scan_fn``.

The reference binds mamba-ssm 1.2.0's CUDA op as a module global (mamba_layer.py:21-34) and calls it
from SS2D_Unit.forward_core (mamba_layer.py:1532-1538) with u/delta (B, K*d, L), A (K*d, 16) fp32,
B/C (B, K, 16, L), D and delta_bias fp32, delta_softplus=True, z=None. Rebinding that global::

    import src.models.base.mamba_layer as ml
    from actalker_amd.selective_scan_interface import selective_scan_fn
    ml.selective_scan_fn = selective_scan_fn

runs the reference's own SS2D_Unit on the gfx950 scan kernel. Same argument
meaning, output dtype = u.dtype. Features the reference never uses (z gating, last state, complex
A) raise NotImplementedError instead of silently differing. A must be <= 0 (the reference's A = -exp(A_log)): the
kernel scans log(-A). A device-side A is not inspected on the host (no sync per call), so an A > 0 channel returns
NaN where mamba-ssm would return exp(delta A) > 1 growth -- a documented divergence, loud rather than silent;
ACTH_CHECK_ARGS=1 (or a CPU-side A) checks the sign on the host and raises ValueError.
"""
from __future__ import annotations

import os

import torch

from . import ops

# ACTH_CHECK_ARGS=1: validate A's sign on the host (a device -> host sync per call; off by default so the op keeps
# the boundary's no-sync contract, include/actalker_hip.h). The reference builds A = -exp(A_log) afresh on every
# call (mamba_layer.py:1530), so no per-tensor cache could skip the sync either.
_CHECK_A = os.environ.get("ACTH_CHECK_ARGS", "0") == "1"


def selective_scan_fn(u, delta, A, B, C, D=None, z=None, delta_bias=None, delta_softplus=False,
                      return_last_state=False):
    if z is not None:
        raise NotImplementedError("selective_scan_fn: z gating is not used by ACTalker and not implemented")
    if return_last_state:
        raise NotImplementedError("selective_scan_fn: return_last_state is not implemented")
    if A.is_complex():
        raise NotImplementedError("selective_scan_fn: complex A is not implemented")
    if not u.is_cuda:
        raise RuntimeError("selective_scan_fn (actalker_amd) runs on the MI355X kernel only")
    batch, dim, L = u.shape
    N = A.shape[1]
    if N != 16:
        raise NotImplementedError("selective_scan_fn: d_state must be 16")
    if B.dim() == 3:
        B = B.unsqueeze(1)
    if C.dim() == 3:
        C = C.unsqueeze(1)
    G = B.shape[1]
    if dim % G:
        raise ValueError("dim must be a multiple of the number of B/C groups")
    A = A.float()
    if _CHECK_A or not A.is_cuda:
        # a device-side A is not inspected on the host (30 syncs per UNet forward otherwise): there A > 0 turns that
        # channel's outputs into NaN (the kernel scans log(-A)) where mamba-ssm returns its exp(delta A) > 1 growth --
        # loud, never silently different; A = 0 is exact (log 0 = -inf, -exp(-inf) = 0)
        if bool((A > 0).any()):
            raise ValueError("selective_scan_fn (actalker_amd) expects A <= 0 (A = -exp(A_log))")
    u_t = u.transpose(1, 2).reshape(batch * L, dim).to(ops.act_dtype()).contiguous()
    d_t = delta.transpose(1, 2).reshape(batch * L, dim).float().contiguous()
    bc = torch.cat([B.float(), C.float()], dim=2)                    # (batch, G, 32, L)
    bc = bc.permute(0, 3, 1, 2).reshape(batch * L, G * 2 * N).contiguous()
    out = ops.selective_scan_op(u_t, d_t, bc, torch.log(-A).contiguous(),
                                None if D is None else D.float().contiguous(),
                                None if delta_bias is None else delta_bias.float().contiguous(),
                                nb=batch, L=L, G=G, softplus=bool(delta_softplus))
    return out.view(batch, L, dim).transpose(1, 2).to(u.dtype)


def selective_scan_ref(*args, **kwargs):
    raise NotImplementedError("the pure-torch reference scan lives in the test oracle, not in the product")
