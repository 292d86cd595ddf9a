"""ORACLE — test infrastructure only. Never imported by actalker_amd.

Reduced-precision emulation of the oracle ("a stated fp16 tolerance"). The reference
ships ``weight_dtype: 'fp16'`` (config/inference.yaml:66; Inference.py:168-177 casts the UNet, 430-433
re-casts A_logs / Ds / dt_projs_bias to fp32): on the GPU every torch op then reads fp16 tensors,
accumulates in fp32 (cuDNN conv, cuBLAS GEMM, flash SDPA, GroupNorm / LayerNorm statistics) and writes
fp16. ``rounded(torch.float16)`` models exactly that on the CPU: the oracle's weights are rounded to
fp16 (the SSM parameters stay fp32) and every torch.nn.functional op of the oracle rounds its tensor
inputs and its output to fp16 while computing in fp32. The selective scan keeps its fp32 state and
rounds its output (mamba-ssm returns u's dtype). ``rounded(torch.bfloat16)`` is the same model with
bf16 rounding -- the precision the HIP build computes in.

The deviation of the fp16-rounded oracle from the fp32 oracle is the numerical noise the reference's
own shipped fp16 path carries; the HIP bf16 result is reported beside it (tests/test_full_geometry_gpu.py,
DESIGN.md §4).
"""
from __future__ import annotations

import contextlib
import types

import torch
import torch.nn.functional as F

from oracle import reference_cpu as ref

_OPS = ("linear", "conv2d", "conv3d", "group_norm", "layer_norm", "scaled_dot_product_attention", "silu", "gelu",
        "interpolate", "softplus")
_FP32_PARAMS = ("A_logs", "Ds", "dt_projs_bias")


def round_state_dict(sd, dtype):
    """Weights as the reference holds them under weight_dtype: dtype, SSM parameters fp32 (Inference.py:430-433)."""
    out = {}
    for k, v in sd.items():
        if k.rsplit(".", 1)[-1] in _FP32_PARAMS or not v.is_floating_point():
            out[k] = v.float()
        else:
            out[k] = v.to(dtype).float()
    return out


def _rnd(x, dtype):
    return x.to(dtype).float() if torch.is_tensor(x) and x.is_floating_point() else x


@contextlib.contextmanager
def rounded(dtype=torch.float16):
    """Inside the context, oracle.reference_cpu's functional ops round inputs / outputs to ``dtype``."""
    shim = types.ModuleType("F_rounded")
    shim.__dict__.update(F.__dict__)

    def wrap(fn):
        def op(*a, **k):
            a = [_rnd(x, dtype) for x in a]
            k = {n: _rnd(x, dtype) for n, x in k.items()}
            return _rnd(fn(*a, **k), dtype)
        return op

    for name in _OPS:
        setattr(shim, name, wrap(getattr(F, name)))
    orig_F, orig_scan = ref.F, ref.selective_scan_ref

    def scan(u, delta, A, B, C, *a, **k):
        # mamba-ssm: fp16 u / delta / B / C in (x_proj / dt_proj outputs), fp32 state, output in u's dtype
        return _rnd(orig_scan(_rnd(u, dtype), _rnd(delta, dtype), A, _rnd(B, dtype), _rnd(C, dtype), *a, **k), dtype)

    ref.F, ref.selective_scan_ref = shim, scan
    try:
        yield
    finally:
        ref.F, ref.selective_scan_ref = orig_F, orig_scan
