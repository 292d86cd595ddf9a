"""Torch-tensor front end of the C ABI (libactalker_hip.so / libactalker_hip_f16.so).

Every function here validates shapes on the host, allocates its output with torch's caching
allocator (device memory is torch's; compute is ours) and launches on
``torch.cuda.current_stream()``. Activations are token-major 2-D tensors ``(rows, C)`` in the current
activation dtype: bf16 by default, fp16 inside ``compute_dtype(torch.float16)`` -- the same kernels built
with fp16 activations (the reference's shipped ``weight_dtype: 'fp16'``, config/inference.yaml:66).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import math
import threading
from typing import Optional, Sequence

import torch

from . import _lib

ACT_NONE, ACT_SILU, ACT_GEGLU, ACT_GELU, ACT_RELU = 0, 1, 2, 3, 4

_TLS = threading.local()        # per-thread stack: concurrent UNet calls (LoopConfig.concurrent_calls) nest safely


def act_dtype() -> torch.dtype:
    """The activation dtype the ops compute in (and the library they launch from)."""
    st = getattr(_TLS, "stack", None)
    return st[-1] if st else torch.bfloat16


@contextlib.contextmanager
def compute_dtype(dtype: torch.dtype):
    """Run the ops inside the block with ``dtype`` activations (torch.bfloat16 or torch.float16)."""
    if dtype not in (torch.bfloat16, torch.float16):
        raise _lib.ActhError(f"compute dtype must be bfloat16 or float16, got {dtype}")
    st = getattr(_TLS, "stack", None)
    if st is None:
        st = _TLS.stack = []
    st.append(dtype)
    try:
        yield
    finally:
        st.pop()


def _p(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _need(t: torch.Tensor, dtype, what: str):
    if not t.is_cuda:
        raise _lib.ActhError(f"{what}: expected a device tensor, got {t.device}")
    if t.dtype != dtype:
        raise _lib.ActhError(f"{what}: expected {dtype}, got {t.dtype}")


def _rows(t: torch.Tensor, what: str) -> int:
    """Row stride (elements) of a 2-D tensor whose rows are contiguous."""
    if t.dim() != 2 or t.stride(1) != 1:
        raise _lib.ActhError(f"{what}: expected a 2-D row-major tensor, got shape {tuple(t.shape)} "
                             f"strides {t.stride()}")
    return t.stride(0)


# ------------------------------------------------------------------------------------------
# ACTH_GEMM_TILE_FLAGS: main-loop flag bits OR-ed into every GEMM's tile word (0x1000 ring, 0x2000 4-phase loop):
# A/B of whole-step timings on one box (tools/ab_gemm.py does the same per shape)
_GEMM_TILE_FLAGS = int(os.environ.get("ACTH_GEMM_TILE_FLAGS", "0"), 0) & 0x3000
# ACTH_GEMM_RING_K: dense products with K >= this also take the ring main loop (0: the convs only, the default)
_GEMM_RING_K = int(os.environ.get("ACTH_GEMM_RING_K", "0"))


def gemm(a: torch.Tensor, w: torch.Tensor, *, M: Optional[int] = None, a2: Optional[torch.Tensor] = None,
         k1: Optional[int] = None, conv: Optional[dict] = None, temporal: Optional[dict] = None,
         bias: Optional[torch.Tensor] = None, rowbias: Optional[torch.Tensor] = None, rb_div: int = 1,
         residual: Optional[torch.Tensor] = None, rmap: Optional[torch.Tensor] = None, r_div: int = 1,
         r_mod: int = 1, mix: Optional[torch.Tensor] = None, mix_alpha: float = 0.0, alpha: float = 1.0,
         act: int = ACT_NONE, out: Optional[torch.Tensor] = None, out_f32: bool = False,
         orow: Optional[Sequence[int]] = None, tile: int = 0, rmap_max: Optional[int] = None) -> torch.Tensor:
    """out = epilogue(A . w^T).  ``tile``: 0 auto, 1 128x128, 2 256x256, 3 256x160, 4 256x256 8-phase,
    5 256x320 8-phase (tests force one).  ``w``: packed (N, K) bf16.

    Every operand the kernel reads or writes through a flat pointer is bounds-checked here on the
    host (the kernels do not check): residual / mix / row-bias rows against M, ``rmap`` entries
    against ``rmap_max`` (the caller's host-side bound on the map's values), the ``orow`` remap
    against ``out``.

    A modes: dense (a is (M, K1) [+ a2 (M, K-K1)]), ``conv=dict(H, W, Ho, Wo, stride, upsample, B)``
    (a is the NHWC image as (B*H*W, C1) [+ a2]), ``temporal=dict(F, S)`` (a is (M, C1) rows).
    """
    lib = _lib.load(act_dtype())
    _need(w, act_dtype(), "gemm weight")
    N, K = w.shape
    d = _lib.GemmDesc()
    d.A = a.data_ptr()
    d.lda = _rows(a, "gemm A")
    _need(a, act_dtype(), "gemm A")
    c1 = a.shape[1] if k1 is None else k1
    if a2 is not None:
        _need(a2, act_dtype(), "gemm A2")
        d.A2 = a2.data_ptr()
        d.lda2 = _rows(a2, "gemm A2")
    d.K1 = c1 if a2 is not None else (1 << 30)
    if conv is not None:
        cin = c1 + (a2.shape[1] if a2 is not None else 0)
        d.amode = 1
        d.H, d.W, d.Ho, d.Wo = conv["H"], conv["W"], conv["Ho"], conv["Wo"]
        d.conv_stride = conv.get("stride", 1)
        d.upsample = int(conv.get("upsample", False))
        d.Cin = cin
        if K != 9 * cin:
            raise _lib.ActhError(f"conv gemm: weight K={K} != 9*Cin={9 * cin}")
        M = conv["B"] * conv["Ho"] * conv["Wo"]
        if a.shape[0] < conv["B"] * conv["H"] * conv["W"]:
            raise _lib.ActhError(f"conv gemm: image has {a.shape[0]} rows < B*H*W")
        d.K1 = c1
    elif temporal is not None:
        cin = c1 + (a2.shape[1] if a2 is not None else 0)
        d.amode = 2
        d.F, d.S = temporal["F"], temporal["S"]
        d.Cin = cin
        if K != 3 * cin:
            raise _lib.ActhError(f"temporal gemm: weight K={K} != 3*Cin={3 * cin}")
        M = a.shape[0]
        d.K1 = c1
    else:
        d.amode = 0
        M = a.shape[0] if M is None else M
        if a.shape[0] < M or (a2 is not None and a2.shape[0] < M):
            raise _lib.ActhError(f"gemm: A has fewer than M={M} rows")
        if a2 is None and a.shape[1] < K:
            raise _lib.ActhError(f"gemm: A has {a.shape[1]} columns < K={K}")
    d.B = w.data_ptr()
    d.ldb = _rows(w, "gemm weight")
    d.M, d.N, d.K = M, N, K
    n_out = N // 2 if act == ACT_GEGLU else N
    if bias is not None:
        _need(bias, torch.float32, "gemm bias")
        if bias.numel() < N:
            raise _lib.ActhError(f"gemm: bias has {bias.numel()} entries < N={N}")
        d.bias = bias.data_ptr()
    if rowbias is not None:
        _need(rowbias, torch.float32, "gemm rowbias")
        if rb_div < 1 or rowbias.shape[0] < -(-M // rb_div) or rowbias.shape[1] < N:
            raise _lib.ActhError(f"gemm: rowbias {tuple(rowbias.shape)} too small for ceil(M/{rb_div}) x N={N}")
        d.rowbias = rowbias.data_ptr()
        d.rb_div = rb_div
        d.ldrb = _rows(rowbias, "gemm rowbias")
    if residual is not None:
        _need(residual, act_dtype(), "gemm residual")
        if residual.dim() != 2 or residual.shape[1] < n_out:
            raise _lib.ActhError(f"gemm: residual {tuple(residual.shape)} narrower than N={n_out}")
        d.R = residual.data_ptr()
        d.ldr = _rows(residual, "gemm residual")
        if rmap is not None:
            _need(rmap, torch.int32, "gemm rmap")
            if rmap_max is None:
                raise _lib.ActhError("gemm: rmap needs rmap_max, a host-side bound on its entries")
            if r_div < 1 or r_mod < 1 or rmap.numel() < min(r_mod, -(-M // r_div)):
                raise _lib.ActhError(f"gemm: rmap has {rmap.numel()} entries, r_div={r_div} r_mod={r_mod}, M={M}")
            if (int(rmap_max) + 1) * r_div > residual.shape[0]:
                raise _lib.ActhError(f"gemm: rmap entries up to {rmap_max} read residual rows beyond "
                                     f"{residual.shape[0]}")
            d.rmap = rmap.data_ptr()
            d.r_div, d.r_mod = r_div, r_mod
        elif residual.shape[0] < M:
            raise _lib.ActhError(f"gemm: residual has {residual.shape[0]} rows < M={M}")
    if mix is not None:
        _need(mix, act_dtype(), "gemm mix")
        if mix.dim() != 2 or mix.shape[0] < M or mix.shape[1] < n_out:
            raise _lib.ActhError(f"gemm: mix {tuple(mix.shape)} too small for ({M}, {n_out})")
        d.MIX = mix.data_ptr()
        d.ldmix = _rows(mix, "gemm mix")
        d.mix_alpha = float(mix_alpha)
    d.alpha = float(alpha)
    d.act = act
    if out is None:
        if orow is not None:
            raise _lib.ActhError("gemm: orow remap needs an explicit output tensor")
        out = torch.empty((M, n_out), device=a.device, dtype=torch.float32 if out_f32 else act_dtype())
    else:
        _need(out, torch.float32 if out_f32 else act_dtype(), "gemm out")
    d.out_f32 = int(out_f32)
    d.C = out.data_ptr()
    d.ldc = _rows(out, "gemm out")
    if orow is None:
        d.orow_div, d.orow_stride, d.orow_off = max(M, 1), max(M, 1), 0
        if out.shape[0] < M or out.shape[1] < n_out:
            raise _lib.ActhError(f"gemm: out {tuple(out.shape)} too small for ({M}, {n_out})")
    else:
        od, ost, oo = (int(v) for v in orow)
        if od < 1 or ost < 0 or oo < 0:
            raise _lib.ActhError(f"gemm: bad orow {tuple(orow)}")
        last = ((M - 1) // od) * ost + (M - 1) % od + oo if M > 0 else -1
        if out.shape[0] <= last or out.shape[1] < n_out:
            raise _lib.ActhError(f"gemm: out {tuple(out.shape)} too small for orow {tuple(orow)} at M={M}")
        d.orow_div, d.orow_stride, d.orow_off = od, ost, oo
    flags = _GEMM_TILE_FLAGS
    if _GEMM_RING_K and not flags and d.amode == 0 and K >= _GEMM_RING_K:
        flags = 0x1000
    d.tile = tile | flags
    _lib.check(lib.acth_gemm(ctypes.byref(d), _stream()), "acth_gemm")
    return out


def conv3x3(x: torch.Tensor, w: torch.Tensor, B: int, H: int, W: int, *, x2=None, stride: int = 1,
            upsample: bool = False, **kw) -> torch.Tensor:
    if upsample:
        Ho, Wo = 2 * H, 2 * W
    else:
        Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    return gemm(x, w, a2=x2, conv=dict(B=B, H=H, W=W, Ho=Ho, Wo=Wo, stride=stride, upsample=upsample), **kw)


# ------------------------------------------------------------------------------------------
def flash_attn(qkv: torch.Tensor, nbatch: int, S: int, heads: int, out: Optional[torch.Tensor] = None):
    """Self-attention over S tokens per batch on fused [q|k|v] rows (nbatch*S, 3C)."""
    lib = _lib.load(act_dtype())
    _need(qkv, act_dtype(), "flash_attn qkv")
    C = heads * 64
    ld = _rows(qkv, "flash_attn qkv")
    if out is None:
        out = torch.empty((nbatch * S, C), device=qkv.device, dtype=act_dtype())
    d = _lib.AttnDesc()
    base = qkv.data_ptr()
    d.q, d.k, d.v, d.o = base, base + 2 * C, base + 4 * C, out.data_ptr()
    d.ldq = d.ldk = d.ldv = ld
    d.ldo = _rows(out, "flash_attn out")
    d.bsq = d.bsk = d.bsv = S * ld
    d.bso = S * d.ldo
    d.nbatch, d.nheads, d.Sq, d.Skv = nbatch, heads, S, S
    d.scale = 1.0 / 8.0
    _lib.check(lib.acth_flash_attn(ctypes.byref(d), _stream()), "acth_flash_attn")
    return out


def temporal_attn(qkv: torch.Tensor, B: int, F: int, S: int, heads: int, out=None):
    lib = _lib.load(act_dtype())
    _need(qkv, act_dtype(), "temporal_attn qkv")
    if out is None:
        out = torch.empty((B * F * S, heads * 64), device=qkv.device, dtype=act_dtype())
    d = _lib.TemporalAttnDesc()
    d.qkv, d.ldqkv = qkv.data_ptr(), _rows(qkv, "temporal_attn qkv")
    d.o, d.ldo = out.data_ptr(), _rows(out, "temporal_attn out")
    d.B, d.F, d.S, d.H = B, F, S, heads
    d.scale = 1.0 / 8.0
    _lib.check(lib.acth_temporal_attn(ctypes.byref(d), _stream()), "acth_temporal_attn")
    return out


def ip_attn(vbase: torch.Tensor, M: int, heads: int, rows_per_ctx: int, S: int, *, q=None, kv=None, nkeys=32,
            vb=None, mask_a=None, mask_b=None, sa=1.0, sb=1.0, out=None):
    lib = _lib.load(act_dtype())
    if out is None:
        out = torch.empty((M, heads * 64), device=vbase.device, dtype=act_dtype())
    d = _lib.IpAttnDesc()
    if kv is not None:
        d.q, d.ldq = q.data_ptr(), _rows(q, "ip_attn q")
        d.kv, d.ldkv, d.nkeys = kv.data_ptr(), _rows(kv, "ip_attn kv"), nkeys
    d.vbase, d.ldvbase = vbase.data_ptr(), _rows(vbase, "ip_attn vbase")
    if vb is not None:
        d.vb, d.ldvb = vb.data_ptr(), _rows(vb, "ip_attn vb")
    if mask_a is not None:
        _need(mask_a, torch.float32, "ip_attn mask_a")
        d.mask_a = mask_a.data_ptr()
    if mask_b is not None:
        _need(mask_b, torch.float32, "ip_attn mask_b")
        d.mask_b = mask_b.data_ptr()
    d.sa, d.sb, d.scale = float(sa), float(sb), 1.0 / 8.0
    d.out, d.ldo = out.data_ptr(), _rows(out, "ip_attn out")
    d.M, d.H, d.rows_per_ctx, d.S = M, heads, rows_per_ctx, S
    _lib.check(lib.acth_ip_attn(ctypes.byref(d), _stream()), "acth_ip_attn")
    return out


XATTN_C = (320,)       # channel widths acth_xattn implements

XATTN_ROWS = 64        # rows per workgroup: a context (frame / window) must be a multiple


def ip_fold(wq: torch.Tensor, woT: torch.Tensor, bo: Optional[torch.Tensor], vid: torch.Tensor, *,
            kv: Optional[torch.Tensor] = None, vb: Optional[torch.Tensor] = None, heads: int,
            norm2=None, kscale: float = 1.4426950408889634 / 8.0):
    """Fold the to_q / to_out projections of an IP-adapter attn2 into its per-context audio keys / values
    (acth_ip_fold; ``woT`` = to_out[0].weight transposed, contiguous; ``norm2`` = (gamma, beta) of the LayerNorm
    in front, folded in): returns (kp, vp, gb, base, vbw) -- K'' / V' (nctx*H*32, C) bf16 and the per-key LN2
    constants gb (nctx*H*32, 2) fp32 (None without ``kv``), base = bo + Wo v_id and vbw = Wo v_vasa (nctx, C)
    fp32 (vbw None without ``vb``)."""
    lib = _lib.load(act_dtype())
    C = wq.shape[0]
    nctx = vid.shape[0]
    for t, nm in ((wq, "wq"), (woT, "woT"), (vid, "vid")):
        _need(t, act_dtype(), f"ip_fold {nm}")
    if tuple(wq.shape) != (C, C) or tuple(woT.shape) != (C, C) or vid.shape[1] != C or heads * 64 != C:
        raise _lib.ActhError(f"ip_fold: wq {tuple(wq.shape)} woT {tuple(woT.shape)} vid {tuple(vid.shape)} H={heads}")
    d = _lib.IpFoldDesc()
    d.wq, d.ldwq = wq.data_ptr(), _rows(wq, "ip_fold wq")
    d.wo, d.ldwo = woT.data_ptr(), _rows(woT, "ip_fold woT")
    if bo is not None:
        _need(bo, torch.float32, "ip_fold bo")
        d.bo = bo.data_ptr()
    d.vid, d.ldvid = vid.data_ptr(), _rows(vid, "ip_fold vid")
    base = torch.empty((nctx, C), device=vid.device, dtype=torch.float32)
    d.base = base.data_ptr()
    vbw = kp = vp = gb = None
    if norm2 is not None:
        d.g2, d.b2 = _p(norm2[0]), _p(norm2[1])
    if vb is not None:
        _need(vb, act_dtype(), "ip_fold vb")
        if tuple(vb.shape) != (nctx, C):
            raise _lib.ActhError(f"ip_fold: vb {tuple(vb.shape)} for {nctx} contexts")
        d.vb, d.ldvb = vb.data_ptr(), _rows(vb, "ip_fold vb")
        vbw = torch.empty((nctx, C), device=vid.device, dtype=torch.float32)
        d.vbw = vbw.data_ptr()
    if kv is not None:
        _need(kv, act_dtype(), "ip_fold kv")
        if kv.shape[0] != nctx * 32 or kv.shape[1] < 2 * C:
            raise _lib.ActhError(f"ip_fold: kv {tuple(kv.shape)} for {nctx} contexts x 32 keys, C={C}")
        d.kv, d.ldkv = kv.data_ptr(), _rows(kv, "ip_fold kv")
        kp = torch.empty((nctx * heads * 32, C), device=vid.device, dtype=act_dtype())
        vp = torch.empty_like(kp)
        gb = torch.empty((nctx * heads * 32, 2), device=vid.device, dtype=torch.float32)
        d.kp, d.vp, d.gb = kp.data_ptr(), vp.data_ptr(), gb.data_ptr()
    d.kscale = float(kscale)
    d.nctx, d.C, d.H = nctx, C, heads
    _lib.check(lib.acth_ip_fold(ctypes.byref(d), _stream()), "acth_ip_fold")
    return kp, vp, gb, base, vbw


def xattn(h: torch.Tensor, eps2: float, norm3, base: torch.Tensor, *, heads: int, rows_per_ctx: int, S: int,
          kp: Optional[torch.Tensor] = None, vp: Optional[torch.Tensor] = None, gb: Optional[torch.Tensor] = None,
          vbw: Optional[torch.Tensor] = None,
          mask_a: Optional[torch.Tensor] = None, mask_b: Optional[torch.Tensor] = None, sa: float = 1.0,
          sb: float = 1.0):
    """Fused IP-adapter attn2 block (acth_xattn): returns (h + attn2(norm2(h)), norm3(that)).
    ``eps2`` = norm2's eps (its weight / bias live in K'' / gb), ``norm3`` = (gamma fp32, beta fp32, eps), or
    None when the consumer (geglu_ffn's ``ln``) normalises itself -- then the second result is None;
    K'' / V' / gb / base / vbw from :func:`ip_fold`."""
    lib = _lib.load(act_dtype())
    _need(h, act_dtype(), "xattn h")
    M, C = h.shape
    if C not in XATTN_C or M % rows_per_ctx or rows_per_ctx % XATTN_ROWS:
        raise _lib.ActhError(f"xattn: M={M} C={C} rows_per_ctx={rows_per_ctx}")
    nctx = M // rows_per_ctx
    if tuple(base.shape) != (nctx, C) or (vbw is not None and tuple(vbw.shape) != (nctx, C)):
        raise _lib.ActhError(f"xattn: base / vbw rows != {nctx} contexts")
    if (kp is None) != (vp is None) or (kp is not None and (tuple(kp.shape) != (nctx * heads * 32, C) or gb is None
                                                             or tuple(gb.shape) != (nctx * heads * 32, 2))):
        raise _lib.ActhError("xattn: K'' / V' / gb missing or mis-shaped")
    for m, nm in ((mask_a, "mask_a"), (mask_b, "mask_b")):
        if m is not None:
            _need(m, torch.float32, f"xattn {nm}")
            if m.numel() < S:
                raise _lib.ActhError(f"xattn: {nm} has {m.numel()} < S={S} entries")
    out = torch.empty_like(h)
    n3 = None if norm3 is None else torch.empty_like(h)
    d = _lib.XattnDesc()
    d.h, d.ldh = h.data_ptr(), _rows(h, "xattn h")
    d.eps2 = float(eps2)
    if norm3 is not None:
        g3, b3, e3 = norm3
        d.g3, d.b3, d.eps3 = _p(g3), _p(b3), float(e3)
    if kp is not None:
        d.kp, d.vp, d.gb = kp.data_ptr(), vp.data_ptr(), gb.data_ptr()
    d.base, d.ldbase = base.data_ptr(), _rows(base, "xattn base")
    if vbw is not None:
        d.vbw, d.ldvbw = vbw.data_ptr(), _rows(vbw, "xattn vbw")
    d.mask_a, d.mask_b = _p(mask_a), _p(mask_b)
    d.sa, d.sb = float(sa), float(sb)
    d.out, d.ldo = out.data_ptr(), C
    if n3 is not None:
        d.n3, d.ldn3 = n3.data_ptr(), C
    d.M, d.C, d.H, d.rows_per_ctx, d.S = M, C, heads, rows_per_ctx, S
    _lib.check(lib.acth_xattn(ctypes.byref(d), _stream()), "acth_xattn")
    return out, n3


# ------------------------------------------------------------------------------------------
FFN_FUSED_C = (320,)   # channel widths acth_geglu_ffn implements


def geglu_ffn(x: torch.Tensor, w1: torch.Tensor, b1: Optional[torch.Tensor], w2p: torch.Tensor,
              b2: Optional[torch.Tensor], *, residual: Optional[torch.Tensor] = None,
              mix: Optional[torch.Tensor] = None, mix_alpha: float = 0.0,
              out: Optional[torch.Tensor] = None, ln=None, add: Optional[torch.Tensor] = None,
              add_div: int = 1) -> torch.Tensor:
    """Fused FeedForward(geglu): y = [a*mix + (1-a)*](W2 (h*gelu(g)) + b2 [+ residual]), [h | g] = W1 x' + b1.
    ``w1``/``b1`` from modules.pack_geglu, ``w2p`` from modules.pack_ffn_w2. ``ln`` = (gamma, beta, eps):
    x' = LayerNorm(x) computed in the kernel (else x' = x). ``add`` (rows, C) bf16: x and the residual each
    get bf16(. + add[row // add_div]) first (not with ``mix``)."""
    lib = _lib.load(act_dtype())
    _need(x, act_dtype(), "geglu_ffn x")
    M, C = x.shape
    if C not in FFN_FUSED_C:
        raise _lib.ActhError(f"geglu_ffn: C={C} not in {FFN_FUSED_C}")
    _need(w1, act_dtype(), "geglu_ffn w1")
    _need(w2p, act_dtype(), "geglu_ffn w2")
    if tuple(w1.shape) != (8 * C, C) or tuple(w2p.shape) != (C, 4 * C):
        raise _lib.ActhError(f"geglu_ffn: weights {tuple(w1.shape)} / {tuple(w2p.shape)} for C={C}")
    for t, nm in ((b1, "b1"), (b2, "b2")):
        if t is not None:
            _need(t, torch.float32, f"geglu_ffn {nm}")
            if not t.is_contiguous() or t.numel() != (8 * C if nm == "b1" else C):
                raise _lib.ActhError(f"geglu_ffn {nm}: {tuple(t.shape)}")
    for t, nm in ((residual, "residual"), (mix, "mix")):
        if t is not None:
            _need(t, act_dtype(), f"geglu_ffn {nm}")
            if t.dim() != 2 or t.shape[0] < M or t.shape[1] < C:
                raise _lib.ActhError(f"geglu_ffn {nm}: {tuple(t.shape)} for ({M}, {C})")
    if out is None:
        out = torch.empty((M, C), device=x.device, dtype=act_dtype())
    elif out.shape[0] < M or out.shape[1] < C:
        raise _lib.ActhError(f"geglu_ffn out: {tuple(out.shape)} for ({M}, {C})")
    d = _lib.FfnDesc()
    d.x, d.ldx = x.data_ptr(), _rows(x, "geglu_ffn x")
    d.w1, d.ldw1, d.b1 = w1.data_ptr(), _rows(w1, "geglu_ffn w1"), None if b1 is None else b1.data_ptr()
    d.w2, d.ldw2, d.b2 = w2p.data_ptr(), _rows(w2p, "geglu_ffn w2"), None if b2 is None else b2.data_ptr()
    if residual is not None:
        d.res, d.ldres = residual.data_ptr(), _rows(residual, "geglu_ffn residual")
    if mix is not None:
        d.mix, d.ldmix, d.mix_alpha = mix.data_ptr(), _rows(mix, "geglu_ffn mix"), float(mix_alpha)
    d.y, d.ldy = out.data_ptr(), _rows(out, "geglu_ffn out")
    d.M, d.C = M, C
    if ln is not None:
        g, b, eps = ln
        for t in (g, b):
            if t is not None and (t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != C):
                raise _lib.ActhError("geglu_ffn ln: gamma / beta must be contiguous fp32 of C entries")
        d.ln_g, d.ln_b, d.ln_eps, d.ln = _p(g), _p(b), float(eps), 1
    if add is not None:
        _need(add, act_dtype(), "geglu_ffn add")
        if mix is not None or add_div <= 0 or add_div % 64 or add.dim() != 2 or add.shape[1] < C or \
                add.shape[0] * add_div < M:
            raise _lib.ActhError(f"geglu_ffn add: {tuple(add.shape)} add_div={add_div} for M={M}")
        d.add, d.ldadd, d.add_div = add.data_ptr(), _rows(add, "geglu_ffn add"), int(add_div)
    _lib.check(lib.acth_geglu_ffn(ctypes.byref(d), _stream()), "acth_geglu_ffn")
    return out


# ------------------------------------------------------------------------------------------
def layernorm(x: torch.Tensor, gamma, beta, eps: float = 1e-5, *, add=None, add_div: int = 1,
              sum_out: Optional[torch.Tensor] = None, out=None):
    lib = _lib.load(act_dtype())
    _need(x, act_dtype(), "layernorm x")
    M, C = x.shape
    if out is None:
        out = torch.empty((M, C), device=x.device, dtype=act_dtype())
    d = _lib.LayerNormDesc()
    d.x, d.ldx = x.data_ptr(), _rows(x, "layernorm x")
    if add is not None:
        d.add, d.ldadd, d.add_div = add.data_ptr(), _rows(add, "layernorm add"), add_div
        if sum_out is not None:
            d.sum_out, d.ldsum = sum_out.data_ptr(), _rows(sum_out, "layernorm sum_out")
    d.gamma = gamma.data_ptr() if gamma is not None else None
    d.beta = beta.data_ptr() if beta is not None else None
    d.eps = float(eps)
    d.y, d.ldy = out.data_ptr(), _rows(out, "layernorm out")
    d.M, d.C = M, C
    _lib.check(lib.acth_layernorm(ctypes.byref(d), _stream()), "acth_layernorm")
    return out


def groupnorm(x: torch.Tensor, gamma, beta, eps: float, rows_per_stat: int, *, x2=None, silu=False, groups=32,
              out=None, relu=False, residual: Optional[torch.Tensor] = None):
    """y = act(GroupNorm(x) [+ residual]); act SiLU (``silu``) or ReLU (``relu``)."""
    lib = _lib.load(act_dtype())
    _need(x, act_dtype(), "groupnorm x")
    M = x.shape[0]
    C1 = x.shape[1]
    C = C1 + (x2.shape[1] if x2 is not None else 0)
    if out is None:
        out = torch.empty((M, C), device=x.device, dtype=act_dtype())
    ws_bytes = lib.acth_groupnorm_workspace_size(M, C, groups, rows_per_stat)
    ws = torch.empty((ws_bytes + 7) // 8, device=x.device, dtype=torch.float64)
    d = _lib.GroupNormDesc()
    d.x, d.ldx = x.data_ptr(), _rows(x, "groupnorm x")
    if x2 is not None:
        d.x2, d.ldx2 = x2.data_ptr(), _rows(x2, "groupnorm x2")
    d.C1 = C1
    d.M, d.C, d.G, d.rows_per_stat = M, C, groups, rows_per_stat
    d.gamma, d.beta, d.eps = gamma.data_ptr(), beta.data_ptr(), float(eps)
    if silu and relu:
        raise _lib.ActhError("groupnorm: silu and relu are exclusive")
    d.silu = 2 if relu else int(silu)
    if residual is not None:
        _need(residual, act_dtype(), "groupnorm residual")
        if residual.shape[0] < M or residual.shape[1] < C:
            raise _lib.ActhError(f"groupnorm: residual {tuple(residual.shape)} too small for ({M}, {C})")
        d.res, d.ldres = residual.data_ptr(), _rows(residual, "groupnorm residual")
    d.y, d.ldy = out.data_ptr(), _rows(out, "groupnorm out")
    d.ws = ws.data_ptr()
    _lib.check(lib.acth_groupnorm(ctypes.byref(d), _stream()), "acth_groupnorm")
    return out


def mamba_combine_ln(branch_a: dict, branch_e: dict, gamma, beta, eps: float, M: int, S: int, C: int, out=None):
    """Each branch dict: mode (0 none / 1 identity / 2 pos map), x, y0, y1, L, pos."""
    lib = _lib.load(act_dtype())
    if out is None:
        out = torch.empty((M, C), device=gamma.device, dtype=act_dtype())
    d = _lib.MambaCombineDesc()

    def fill(pre, br):
        mode = br["mode"]
        setattr(d, "mode_" + pre, mode)
        if br.get("x") is not None:
            setattr(d, "x" + pre, br["x"].data_ptr())
            setattr(d, "ldx" + pre, _rows(br["x"], "mamba x"))
        if mode != 0:
            setattr(d, "y" + pre + "0", br["y0"].data_ptr())
            setattr(d, "y" + pre + "1", br["y1"].data_ptr())
            setattr(d, "ldy" + pre, _rows(br["y0"], "mamba y"))
            setattr(d, "L" + pre, br["L"])
        if mode == 2:
            setattr(d, "pos_" + pre, br["pos"].data_ptr())

    fill("a", branch_a)
    fill("e", branch_e)
    d.gamma, d.beta, d.eps = gamma.data_ptr(), beta.data_ptr(), float(eps)
    d.y, d.ldy = out.data_ptr(), _rows(out, "mamba out")
    d.M, d.S, d.C = M, S, C
    _lib.check(lib.acth_mamba_combine_ln(ctypes.byref(d), _stream()), "acth_mamba_combine_ln")
    return out


# bf16 x_proj rows: 0 = paired-lane kernel, 1 = scan_quad_kernel (MFMA input term; ACTH_SCAN_QUAD=1)
SCAN_ALGO = int(os.environ.get("ACTH_SCAN_QUAD", "0"))


def _fused_scan_desc(u, xdbl, dt_w, dt_b, A_log, Dskip, nb, L, R, n_keep, y0, y1, nchunks):
    """Checks and ScanDesc of one fused bidirectional scan; (None, y0, y1, None) when n_keep is 0."""
    _need(u, act_dtype(), "scan u")
    if xdbl.dtype not in (torch.float32, act_dtype()):
        raise _lib.ActhError(f"scan xdbl must be float32 or {act_dtype()}, got {xdbl.dtype}")
    D = u.shape[1]
    for t, nm in ((dt_w, "dt_w"), (dt_b, "dt_b"), (A_log, "A_log"), (Dskip, "D")):
        _need(t, torch.float32, "scan " + nm)
        if not t.is_contiguous():
            raise _lib.ActhError(f"scan {nm} must be contiguous")
    if y0 is None:
        y0 = torch.empty((nb * n_keep, D), device=u.device, dtype=act_dtype())
    if y1 is None:
        y1 = torch.empty((nb * n_keep, D), device=u.device, dtype=act_dtype())
    if n_keep == 0:
        return None, y0, y1, None
    d = _lib.ScanDesc()
    d.u, d.ldu = u.data_ptr(), _rows(u, "scan u")
    d.xdbl, d.ldx = xdbl.data_ptr(), _rows(xdbl, "scan xdbl")
    d.dt_w, d.dt_b, d.A_log, d.Dskip = dt_w.data_ptr(), dt_b.data_ptr(), A_log.data_ptr(), Dskip.data_ptr()
    d.y0, d.y1, d.ldy = y0.data_ptr(), y1.data_ptr(), _rows(y0, "scan y0")
    d.nb, d.L, d.D, d.R, d.N, d.n_keep = nb, L, D, R, 16, n_keep
    d.softplus, d.G, d.u_gstride, d.y_gstride, d.flip1 = 1, 2, 0, 0, 1
    d.xdbl_bf16 = int(xdbl.dtype == act_dtype())
    d.scan_algo = SCAN_ALGO
    if d.xdbl_bf16:
        d.nchunks = 1          # the bf16-xdbl kernel is single-pass
        return d, y0, y1, None
    ws = _scan_chunking(d, nb, 2, D, L, nchunks, u.device)
    return d, y0, y1, ws


def selective_scan(u: torch.Tensor, xdbl: torch.Tensor, dt_w, dt_b, A_log, Dskip, *, nb: int, L: int, R: int,
                   n_keep: int, y0=None, y1=None, nchunks: Optional[int] = None):
    """Fused bidirectional scan. u: (nb*L, D) bf16; xdbl: (nb*L, 2*(R+32)) fp32 rows [dt | B | C] per
    direction, or bf16 rows (the reference's x_dbl dtype) of 2*(R4+32) with R4 = R rounded up to 4
    (dt padding columns ignored; ``SS2D_Unit.packed()['xproj_pad']`` holds the x_proj weights in that layout)."""
    lib = _lib.load(act_dtype())
    d, y0, y1, ws = _fused_scan_desc(u, xdbl, dt_w, dt_b, A_log, Dskip, nb, L, R, n_keep, y0, y1, nchunks)
    if d is not None:
        _lib.check(lib.acth_selective_scan(ctypes.byref(d), _stream()), "acth_selective_scan")
    del ws
    return y0, y1


def selective_scan2(a: dict, b: dict):
    """Two fused bidirectional scans (selective_scan's keyword arguments each: u, xdbl, dt_w, dt_b,
    A_log, Dskip, nb, L, R, n_keep) in one launch -- SS2D_cond_v10's audio and expression branches.
    Returns ((y0, y1) of a, (y0, y1) of b)."""
    lib = _lib.load(act_dtype())
    da, ya0, ya1, wsa = _fused_scan_desc(nchunks=1, y0=None, y1=None, **a)
    db, yb0, yb1, wsb = _fused_scan_desc(nchunks=1, y0=None, y1=None, **b)
    if da is not None and db is not None:
        _lib.check(lib.acth_selective_scan2(ctypes.byref(da), ctypes.byref(db), _stream()),
                   "acth_selective_scan2")
    else:
        for d in (da, db):
            if d is not None:
                _lib.check(lib.acth_selective_scan(ctypes.byref(d), _stream()), "acth_selective_scan")
    del wsa, wsb
    return (ya0, ya1), (yb0, yb1)


def scan_auto_chunks(nb: int, G: int, D: int, L: int) -> int:
    """Single pass (the paired-lane kernel, 2 lanes per channel) at every ACTalker shape: it beats
    the two-pass chunked kernel by 4 % / 19 % / 35 % at levels 0 / 1 / 2 (tools/bench_scan.py);
    the chunked kernel stays available through an explicit ``nchunks`` > 1."""
    return 1


def _scan_chunking(d, nb, G, D, L, nchunks, device):
    lib = _lib.load(act_dtype())
    nc = scan_auto_chunks(nb, G, D, L) if nchunks is None else int(nchunks)
    d.nchunks = nc
    ws = None
    if nc > 1:
        nbytes = lib.acth_selective_scan_workspace_size(nb, G, D, nc)
        ws = torch.empty((nbytes + 3) // 4, device=device, dtype=torch.float32)
        d.ws = ws.data_ptr()
    return ws


def selective_scan_op(u_t: torch.Tensor, delta_t: torch.Tensor, bc: torch.Tensor, A_log: torch.Tensor,
                      Dskip: Optional[torch.Tensor], delta_bias: Optional[torch.Tensor], *, nb: int, L: int,
                      G: int, softplus: bool, out: Optional[torch.Tensor] = None, nchunks: Optional[int] = None):
    """Generic op mode: u_t (nb*L, G*D) bf16, delta_t (nb*L, G*D) fp32/bf16, bc (nb*L, G*32) fp32
    [B(16) | C(16)] per group, forward traversal, all L outputs -> (nb*L, G*D) bf16."""
    lib = _lib.load(act_dtype())
    _need(u_t, act_dtype(), "scan u")
    _need(bc, torch.float32, "scan B/C")
    GD = u_t.shape[1]
    D = GD // G
    if out is None:
        out = torch.empty((nb * L, GD), device=u_t.device, dtype=act_dtype())
    d = _lib.ScanDesc()
    d.u, d.ldu = u_t.data_ptr(), _rows(u_t, "scan u")
    d.xdbl, d.ldx = bc.data_ptr(), _rows(bc, "scan B/C")
    d.dt_b = None if delta_bias is None else delta_bias.data_ptr()
    d.A_log = A_log.data_ptr()
    d.Dskip = None if Dskip is None else Dskip.data_ptr()
    d.y0, d.ldy = out.data_ptr(), _rows(out, "scan out")
    d.nb, d.L, d.D, d.R, d.N, d.n_keep = nb, L, D, 0, 16, L
    d.delta, d.ld_delta = delta_t.data_ptr(), _rows(delta_t, "scan delta")
    d.delta_f32 = int(delta_t.dtype == torch.float32)
    d.softplus, d.G, d.u_gstride, d.y_gstride, d.flip1 = int(softplus), G, D, D, 0
    ws = _scan_chunking(d, nb, G, D, L, nchunks, u_t.device)
    _lib.check(lib.acth_selective_scan(ctypes.byref(d), _stream()), "acth_selective_scan")
    del ws
    return out


# ------------------------------------------------------------------------------------------
def timestep_embedding(t: torch.Tensor, dim: int, flip_sin_to_cos: bool = True, shift: float = 0.0,
                       scale: float = 1.0, max_period: float = 10000.0) -> torch.Tensor:
    lib = _lib.load(act_dtype())
    t = t.to(torch.float32).contiguous()
    out = torch.empty((t.numel(), dim), device=t.device, dtype=act_dtype())
    _lib.check(lib.acth_timestep_embedding(_p(t), t.numel(), dim, int(flip_sin_to_cos), shift, scale,
                                           max_period, _p(out), _stream()), "acth_timestep_embedding")
    return out


def nchw_to_tokens(x: torch.Tensor, out_dtype=None) -> torch.Tensor:
    """(B, C, H, W) or (B, F, C, H, W) -> (B*[F*]H*W, C)."""
    lib = _lib.load(act_dtype())
    x = x.contiguous()
    C, H, W = x.shape[-3:]
    B = x.numel() // (C * H * W)
    if x.dtype not in (torch.float32, act_dtype()):
        x = x.float()
    out_dtype = act_dtype() if out_dtype is None else out_dtype
    out = torch.empty((B * H * W, C), device=x.device, dtype=out_dtype)
    _lib.check(lib.acth_nchw_to_tokens(_p(x), int(x.dtype == torch.float32), _p(out),
                                       int(out_dtype == torch.float32), C, B, C, H * W, _stream()),
               "acth_nchw_to_tokens")
    return out


def tokens_to_nchw(x: torch.Tensor, B: int, H: int, W: int, out_dtype=torch.float32) -> torch.Tensor:
    lib = _lib.load(act_dtype())
    C = x.shape[1]
    out = torch.empty((B, C, H, W), device=x.device, dtype=out_dtype)
    _lib.check(lib.acth_tokens_to_nchw(_p(x), int(x.dtype == torch.float32), _rows(x, "tokens"), _p(out),
                                       int(out_dtype == torch.float32), B, C, H * W, _stream()),
               "acth_tokens_to_nchw")
    return out


def im2col3x3(x: torch.Tensor, B: int, H: int, W: int) -> torch.Tensor:
    lib = _lib.load(act_dtype())
    C = x.shape[1]
    K = 9 * C
    out = torch.empty((B * H * W, K), device=x.device, dtype=act_dtype())
    _lib.check(lib.acth_im2col3x3(_p(x.contiguous()), B, H, W, C, _p(out), K, _stream()), "acth_im2col3x3")
    return out


def im2col(x: torch.Tensor, B: int, H: int, W: int, kh: int, kw: int, stride: int, pad: int,
           kpad: Optional[int] = None) -> torch.Tensor:
    """NHWC rows (B*H*W, C) -> (B*Ho*Wo, Kpad) patches, column (ky*kw + kx)*C + c, zero-padded to Kpad
    (default: kh*kw*C rounded up to a multiple of 8)."""
    lib = _lib.load(act_dtype())
    _need(x, act_dtype(), "im2col x")
    C = x.shape[1]
    if x.shape[0] != B * H * W:
        raise _lib.ActhError(f"im2col: x has {x.shape[0]} rows, expected {B * H * W}")
    Ho, Wo = (H + 2 * pad - kh) // stride + 1, (W + 2 * pad - kw) // stride + 1
    K = kh * kw * C
    kp = (K + 7) // 8 * 8 if kpad is None else kpad
    out = torch.empty((B * Ho * Wo, kp), device=x.device, dtype=act_dtype())
    _lib.check(lib.acth_im2col(_p(x), _rows(x, "im2col x"), B, H, W, C, kh, kw, stride, pad, Ho, Wo, _p(out), kp,
                               _stream()), "acth_im2col")
    return out


def maxpool2d(x: torch.Tensor, B: int, H: int, W: int, k: int, stride: int, pad: int) -> torch.Tensor:
    lib = _lib.load(act_dtype())
    _need(x, act_dtype(), "maxpool x")
    C = x.shape[1]
    if x.shape[0] != B * H * W:
        raise _lib.ActhError(f"maxpool: x has {x.shape[0]} rows, expected {B * H * W}")
    Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    out = torch.empty((B * Ho * Wo, C), device=x.device, dtype=act_dtype())
    _lib.check(lib.acth_maxpool2d(_p(x), _rows(x, "maxpool x"), B, H, W, C, k, stride, pad, Ho, Wo, _p(out),
                                  _rows(out, "maxpool out"), _stream()), "acth_maxpool2d")
    return out


def gather_rows(src: torch.Tensor, idx: torch.Tensor, nb: int, Ls: int, dst: torch.Tensor, Ld: int):
    lib = _lib.load(act_dtype())
    _need(idx, torch.int32, "gather idx")
    C = src.shape[1]
    _lib.check(lib.acth_gather_rows(_p(src), _rows(src, "gather src"), Ls, _p(idx), idx.numel(), _p(dst),
                                    _rows(dst, "gather dst"), Ld, nb, C, _stream()), "acth_gather_rows")
    return dst


def gather_blocks(src: torch.Tensor, n_src: int, idx: torch.Tensor, idx_max: int) -> torch.Tensor:
    """``src`` viewed as ``n_src`` equal row blocks; returns the blocks ``idx`` names, in order
    (out block i = src block idx[i]). ``idx``: device int32; ``idx_max``: the caller's host-side bound on its
    entries (the kernel does not check them)."""
    lib = _lib.load(act_dtype())
    _need(idx, torch.int32, "gather_blocks idx")
    if not src.is_contiguous() or n_src < 1 or src.shape[0] % n_src:
        raise _lib.ActhError(f"gather_blocks: src {tuple(src.shape)} is not {n_src} contiguous row blocks")
    if not 0 <= int(idx_max) < n_src:
        raise _lib.ActhError(f"gather_blocks: index bound {idx_max} outside [0, {n_src})")
    n = idx.numel()
    per = src.shape[0] // n_src
    out = torch.empty((n * per, *src.shape[1:]), device=src.device, dtype=src.dtype)
    block_bytes = src.numel() // n_src * src.element_size()
    _lib.check(lib.acth_gather_blocks(_p(src), n_src, _p(idx), n, block_bytes, _p(out), _stream()),
               "acth_gather_blocks")
    return out


def frame_mean(x: torch.Tensor, B: int, F: int, T: int) -> torch.Tensor:
    """x rows ((b*F + f)*T + t) -> rows (b*T + t), mean over f."""
    lib = _lib.load(act_dtype())
    C = x.shape[1]
    out = torch.empty((B * T, C), device=x.device, dtype=act_dtype())
    _lib.check(lib.acth_frame_mean(_p(x), _rows(x, "frame_mean x"), B, F, T, C, _p(out), C, _stream()),
               "acth_frame_mean")
    return out


def window_input(lat: torch.Tensor, frame_idx: torch.Tensor, img: torch.Tensor, branch: torch.Tensor,
                 in_scale: float, U: int, F: int, S: int, T: int) -> torch.Tensor:
    """lat (T*S, 4) fp32, img (nbranch*T*S, 4) fp32 -> (U*F*S, 8) bf16 UNet input."""
    lib = _lib.load(act_dtype())
    out = torch.empty((U * F * S, 8), device=lat.device, dtype=act_dtype())
    _lib.check(lib.acth_window_input(_p(lat), _p(frame_idx), _p(img), _p(branch), float(in_scale), _p(out),
                                     U, F, S, T, _stream()), "acth_window_input")
    return out


def cfg_euler_accum(noise, unit_off, lat, frame_idx, g1, g2, g3, sigma, sigma_next, acc, cnt, F, S):
    lib = _lib.load(act_dtype())
    _lib.check(lib.acth_cfg_euler_accum(_p(noise), _p(unit_off), _p(lat), _p(frame_idx), float(g1), float(g2),
                                        float(g3), float(sigma), float(sigma_next), _p(acc), _p(cnt), F, S,
                                        _stream()), "acth_cfg_euler_accum")


def div_counter(acc, cnt, out, T, S):
    lib = _lib.load(act_dtype())
    _lib.check(lib.acth_div_counter(_p(acc), _p(cnt), _p(out), T, S, _stream()), "acth_div_counter")
    return out


# ------------------------------------------------------------------------------------------
def pack_conv_direct(w: torch.Tensor) -> torch.Tensor:
    """Conv weight (Cout, Cin, 3, 3) or (Cout, Cin, 3, 1, 1) -> fp32 (taps*Cin, Cout), k = tap*Cin + c."""
    w = w.detach().float()
    if w.dim() == 5:
        w = w[:, :, :, 0, 0]                                  # (Cout, Cin, 3)
        return w.permute(2, 1, 0).reshape(-1, w.shape[0]).contiguous()
    return w.permute(2, 3, 1, 0).reshape(-1, w.shape[0]).contiguous()


def conv_direct(x: torch.Tensor, wp: torch.Tensor, bias: Optional[torch.Tensor], *, B: int, H: int = 0, W: int = 0,
                stride: int = 1, pad0: bool = False, temporal: Optional[dict] = None, act: int = ACT_NONE, out_f32: bool = False,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Direct 3x3 (pad 1, stride 1/2) or (3,1,1) temporal conv on NHWC rows for narrow channels.
    ``wp`` from :func:`pack_conv_direct`; ``temporal=dict(F, S)`` selects the frame-axis form; ``pad0``
    pads only bottom/right (diffusers Downsample2D with padding=0: F.pad(x, (0, 1, 0, 1)), conv pad 0)."""
    lib = _lib.load(act_dtype())
    _need(x, act_dtype(), "conv_direct x")
    _need(wp, torch.float32, "conv_direct w")
    Cin = x.shape[1] if x.dim() == 2 else None
    taps = 3 if temporal is not None else 9
    if Cin is None or wp.shape[0] != taps * Cin:
        raise _lib.ActhError(f"conv_direct: weight rows {wp.shape[0]} != {taps}*Cin ({Cin})")
    Cout = wp.shape[1]
    d = _lib.ConvDirectDesc()
    if temporal is None:
        ps = 1 if pad0 else 2
        Ho, Wo = (H + ps - 3) // stride + 1, (W + ps - 3) // stride + 1
        if x.shape[0] != B * H * W:
            raise _lib.ActhError(f"conv_direct: x has {x.shape[0]} rows, expected {B * H * W}")
        d.mode, d.H, d.W, d.Ho, d.Wo, d.stride, d.pad0 = 0, H, W, Ho, Wo, stride, int(pad0)
        M = B * Ho * Wo
    else:
        Fr, S = temporal["F"], temporal["S"]
        if x.shape[0] != B * Fr * S:
            raise _lib.ActhError(f"conv_direct: x has {x.shape[0]} rows, expected {B * Fr * S}")
        d.mode, d.F, d.S = 1, Fr, S
        M = B * Fr * S
    if out is None:
        out = torch.empty((M, Cout), device=x.device, dtype=torch.float32 if out_f32 else act_dtype())
    d.x, d.ldx = x.data_ptr(), _rows(x, "conv_direct x")
    d.w = wp.data_ptr()
    if bias is not None:
        _need(bias, torch.float32, "conv_direct bias")
        d.bias = bias.data_ptr()
    d.y, d.ldy = out.data_ptr(), _rows(out, "conv_direct out")
    d.B, d.Cin, d.Cout, d.act, d.out_f32 = B, Cin, Cout, act, int(out_f32)
    _lib.check(lib.acth_conv_direct(ctypes.byref(d), _stream()), "acth_conv_direct")
    return out


def softmax_rows(x: torch.Tensor, scale: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bf16 softmax(scale * x) over the last dim of an fp32 (rows, cols) matrix."""
    lib = _lib.load(act_dtype())
    _need(x, torch.float32, "softmax x")
    rows, cols = x.shape
    if out is None:
        out = torch.empty((rows, cols), device=x.device, dtype=act_dtype())
    _lib.check(lib.acth_softmax_rows(_p(x), _rows(x, "softmax x"), _p(out), _rows(out, "softmax out"), rows, cols,
                                     float(scale), _stream()), "acth_softmax_rows")
    return out
