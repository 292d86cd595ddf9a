"""GPU: each kernel against a plain torch fp32 computation of the same op, in both builds: bf16 activations
(libactalker_hip.so) and fp16 activations (libactalker_hip_f16.so, ops.compute_dtype) -- every test runs once
per build (the ``act`` fixture).

Inputs are rounded to the activation dtype first so the comparison measures only the kernel's accumulation and
output rounding. Tolerance: relative L2 error <= 1e-2 (16-bit output, fp32 accumulation) unless
noted; the scan uses the oracle's restated mamba-ssm selective_scan_ref."""
import math

import pytest
import torch
import torch.nn.functional as F

from actalker_amd import ops
from oracle import reference_cpu as ref

pytestmark = pytest.mark.gpu


def bf(x):
    """Round to the activation dtype of the build under test (bf16 or fp16)."""
    return x.to(ops.act_dtype())


def rel(a, b):
    a = a.float().cpu()
    b = b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def rnd(*shape, scale=1.0, g=None):
    return (torch.randn(*shape, generator=g) * scale)


@pytest.fixture(autouse=True)
def _seed():
    torch.manual_seed(1234)


@pytest.fixture(autouse=True, params=["bf16", "fp16"])
def act(request):
    with ops.compute_dtype(torch.float16 if request.param == "fp16" else torch.bfloat16):
        yield request.param


# ------------------------------------------------------------------------------------------ GEMM
@pytest.mark.parametrize("M,N,K", [(1, 4, 64), (77, 130, 72), (300, 320, 320), (1024, 1280, 2560), (4, 1280, 768)])
def test_gemm_dense(dev, M, N, K):
    a = bf(rnd(M, K))
    w = bf(rnd(N, K, scale=K ** -0.5))
    b = rnd(N)
    out = ops.gemm(a.to(dev), w.to(dev), bias=b.to(dev))
    refo = a.float() @ w.float().t() + b
    assert rel(out, refo) < 1e-2


def test_gemm_epilogues(dev):
    M, N, K = 513, 256, 192
    a, w = bf(rnd(M, K)), bf(rnd(N, K, scale=K ** -0.5))
    bias = rnd(N)
    rowb = rnd(3, N)
    res = bf(rnd(M, N))
    mix = bf(rnd(M, N))
    base = a.float() @ w.float().t() + bias + rowb.repeat_interleave(171, 0) + res.float()
    out = ops.gemm(a.to(dev), w.to(dev), bias=bias.to(dev), rowbias=rowb.to(dev), rb_div=171,
                   residual=res.to(dev), mix=mix.to(dev), mix_alpha=0.3)
    assert rel(out, 0.3 * mix.float() + 0.7 * base) < 1e-2
    out = ops.gemm(a.to(dev), w.to(dev), bias=bias.to(dev), act=ops.ACT_SILU, out_f32=True)
    assert out.dtype == torch.float32
    assert rel(out, F.silu(a.float() @ w.float().t() + bias)) < 1e-2
    # two-source K split (skip-connection concat) + residual row remap
    a2 = bf(rnd(M, 64))
    w2 = bf(rnd(N, K + 64, scale=(K + 64) ** -0.5))
    rmap = torch.tensor([2, 0, 1], dtype=torch.int32)
    res3 = bf(rnd(3 * 57, N))
    out = ops.gemm(a.to(dev), w2.to(dev), a2=a2.to(dev), residual=res3.to(dev), rmap=rmap.to(dev), r_div=57,
                   r_mod=3, M=M, rmap_max=2)
    rows = torch.arange(M)
    rr = rmap[(rows // 57) % 3].long() * 57 + rows % 57
    refo = torch.cat([a, a2], 1).float() @ w2.float().t() + res3.float()[rr]
    assert rel(out, refo) < 1e-2


def test_gemm_geglu_and_orow(dev):
    from actalker_amd.modules import pack_geglu
    M, C, inner = 200, 128, 512
    x = bf(rnd(M, C))
    w = rnd(2 * inner, C, scale=C ** -0.5)
    b = rnd(2 * inner, scale=0.1)
    wp, bp = pack_geglu(w, b)
    out = ops.gemm(x.to(dev), wp.to(dev), bias=bp.to(dev), act=ops.ACT_GEGLU)
    h, g = (x.float() @ bf(w).float().t() + b).chunk(2, -1)
    assert out.shape == (M, inner)
    assert rel(out, h * F.gelu(g)) < 1e-2
    # orow: rows (m / 50) * 64 + m % 50 + 3 of a bigger buffer
    buf = torch.zeros(4 * 64 + 8, 96, device=dev, dtype=ops.act_dtype())
    w3 = bf(rnd(96, C, scale=C ** -0.5))
    ops.gemm(x.to(dev), w3.to(dev), out=buf, orow=(50, 64, 3))
    refo = x.float() @ w3.float().t()
    got = buf.cpu().float().view(-1, 96)
    for blk in range(4):
        assert rel(got[blk * 64 + 3: blk * 64 + 53], refo[blk * 50:(blk + 1) * 50]) < 1e-2
    assert float(got[0:3].abs().sum()) == 0.0


@pytest.mark.parametrize("M,case", [(1, "res"), (127, "plain"), (300, "res_mix"), (4133, "res"),
                                    (2 * 128 * 7 + 5, "res_mix"), (640, "nobias")])
def test_geglu_ffn_fused(dev, M, case):
    """acth_geglu_ffn (C = 320) against torch fp32 (hidden rounded to bf16 like the kernel) and
    against the two-GEMM path it replaces."""
    from actalker_amd.modules import pack_geglu, pack_ffn_w2
    C, inner = 320, 1280
    x = bf(rnd(M, C))
    w1 = rnd(2 * inner, C, scale=C ** -0.5)
    b1 = rnd(2 * inner, scale=0.1) if case != "nobias" else torch.zeros(2 * inner)
    w2 = rnd(C, inner, scale=inner ** -0.5)
    b2 = rnd(C, scale=0.1) if case != "nobias" else None
    res = bf(rnd(M, C)) if case in ("res", "res_mix") else None
    mix = bf(rnd(M, C)) if case == "res_mix" else None
    wp, bp = pack_geglu(w1, b1)
    w2p = pack_ffn_w2(w2)
    dv = lambda t: None if t is None else t.to(dev)
    out = ops.geglu_ffn(x.to(dev), wp.to(dev), None if case == "nobias" else bp.to(dev), w2p.to(dev), dv(b2),
                        residual=dv(res), mix=dv(mix), mix_alpha=0.3)
    h, g = (x.float() @ bf(w1).float().t() + b1).chunk(2, -1)
    hid = bf(h * F.gelu(g)).float()
    refo = hid @ bf(w2).float().t() + (b2 if b2 is not None else 0.0)
    if res is not None:
        refo = refo + res.float()
    if mix is not None:
        refo = 0.3 * mix.float() + 0.7 * refo
    assert out.shape == (M, C)
    assert rel(out, refo) < 1e-2
    # the two-kernel path (GEGLU GEMM + output GEMM) on the same packed operands
    gg = ops.gemm(x.to(dev), wp.to(dev), bias=bp.to(dev), act=ops.ACT_GEGLU)
    two = ops.gemm(gg, bf(w2).to(dev), bias=dv(b2), residual=dv(res), mix=dv(mix), mix_alpha=0.3)
    assert rel(out, two) < 4e-3


@pytest.mark.parametrize("M,case", [(1, "ln"), (300, "ln_mix"), (4133, "ln_add"), (2 * 128 * 7 + 5, "ln"),
                                    (14 * 64, "ln_add")])
def test_geglu_ffn_fused_layernorm(dev, M, case):
    """acth_geglu_ffn with its prologue LayerNorm (norm3 -> ff, norm_in (+ pos_emb) -> ff_in): y = FFN(LN(x')) +
    x' [mix], x' = bf16(x + add[row // div]); against torch fp32 and against layernorm + geglu_ffn. The rows carry
    a common offset (the statistics must remove it); the residual is subtracted before the comparison so the
    FFN term is what the tolerance measures."""
    from actalker_amd.modules import pack_geglu, pack_ffn_w2
    C, inner, div = 320, 1280, 64
    x = bf(rnd(M, C) + 3.0)
    g3, b3 = 1.0 + 0.2 * rnd(C), 0.1 * rnd(C)
    w1 = rnd(2 * inner, C, scale=C ** -0.5)
    b1 = rnd(2 * inner, scale=0.1)
    w2 = rnd(C, inner, scale=inner ** -0.5)
    b2 = rnd(C, scale=0.1)
    add = bf(rnd((M + div - 1) // div, C)) if case == "ln_add" else None
    mix = bf(rnd(M, C)) if case == "ln_mix" else None
    wp, bp = pack_geglu(w1, b1)
    w2p = pack_ffn_w2(w2)
    dv = lambda t: None if t is None else t.to(dev)
    xd = x.to(dev)
    out = ops.geglu_ffn(xd, wp.to(dev), bp.to(dev), w2p.to(dev), b2.to(dev), residual=xd, mix=dv(mix),
                        mix_alpha=0.3, ln=(g3.to(dev), b3.to(dev), 1e-5), add=dv(add), add_div=div)
    xs = x.float() if add is None else bf(x.float() + add.float().repeat_interleave(div, 0)[:M]).float()
    n = bf(F.layer_norm(xs, (C,), g3, b3, 1e-5)).float()
    h, g = (n @ bf(w1).float().t() + b1).chunk(2, -1)
    refo = bf(h * F.gelu(g)).float() @ bf(w2).float().t() + b2 + xs
    base = xs if mix is None else 0.3 * mix.float() + 0.7 * xs
    if mix is not None:
        refo = 0.3 * mix.float() + 0.7 * refo
    assert rel(out.float().cpu() - base, refo - base) < 1e-2
    # the unfused pair: acth_layernorm (+ row add, sum out) then acth_geglu_ffn
    xs_d = torch.empty_like(xd)
    nd = ops.layernorm(xd, g3.to(dev), b3.to(dev), 1e-5, add=dv(add), add_div=div,
                       sum_out=xs_d if add is not None else None)
    two = ops.geglu_ffn(nd, wp.to(dev), bp.to(dev), w2p.to(dev), b2.to(dev),
                        residual=xs_d if add is not None else xd, mix=dv(mix), mix_alpha=0.3)
    assert rel(out.float().cpu() - base, two.float().cpu() - base) < 4e-3


def test_geglu_ffn_rejects_bad_shapes(dev):
    from actalker_amd import _lib
    x = torch.zeros(8, 640, device=dev, dtype=ops.act_dtype())
    w1 = torch.zeros(8 * 640, 640, device=dev, dtype=ops.act_dtype())
    w2 = torch.zeros(640, 4 * 640, device=dev, dtype=ops.act_dtype())
    with pytest.raises(_lib.ActhError):
        ops.geglu_ffn(x, w1, None, w2, None)
    x = torch.zeros(8, 320, device=dev, dtype=ops.act_dtype())
    w1 = torch.zeros(8 * 320, 320, device=dev, dtype=ops.act_dtype())
    w2 = torch.zeros(320, 4 * 320, device=dev, dtype=ops.act_dtype())
    with pytest.raises(_lib.ActhError):
        ops.geglu_ffn(x, w1, None, w2, None, residual=torch.zeros(4, 320, device=dev, dtype=ops.act_dtype()))


@pytest.mark.parametrize("tile", [4, 5])
@pytest.mark.parametrize("gm", [1, 3, 8])
def test_gemm_grouped_raster(dev, tile, gm):
    """M-grouped tile order of the phased kernels (tile bits 16-23): every (m, n) tile written once,
    including the partial last group (11 row blocks over groups of 3 / 8) and a ragged N."""
    from actalker_amd.modules import pack_geglu
    M, N, K = 11 * 256 - 40, 1280 + 64, 192
    a, w = bf(rnd(M, K)), bf(rnd(N, K, scale=K ** -0.5))
    bias = rnd(N)
    if tile == 4:
        wp, bp = pack_geglu(rnd(2 * 640, K, scale=K ** -0.5), rnd(2 * 640, scale=0.1))
        out = ops.gemm(a.to(dev), wp.to(dev), bias=bp.to(dev), act=ops.ACT_GEGLU, tile=tile | (gm << 16))
        ref0 = ops.gemm(a.to(dev), wp.to(dev), bias=bp.to(dev), act=ops.ACT_GEGLU, tile=tile)
        assert torch.equal(out, ref0)
    else:
        out = ops.gemm(a.to(dev), w.to(dev), bias=bias.to(dev), tile=tile | (gm << 16))
        assert rel(out, a.float() @ w.float().t() + bias) < 1e-2
        assert torch.equal(out, ops.gemm(a.to(dev), w.to(dev), bias=bias.to(dev), tile=tile))


@pytest.mark.parametrize("tile", [4, 5])
@pytest.mark.parametrize("case", ["plain", "rmap_mix_silu", "ragged_n", "res_mix", "bias_only", "rowbias", "rb_res"])
def test_gemm_phased_vector_residual(dev, tile, case):
    """The phased kernels' vector residual path (16-byte-aligned residual rows, the residual chunk
    loaded one iteration ahead, invalid rows / columns clamped to row 0): N a multiple of 8, a
    ragged last row tile, residual through a row map, AlphaBlender mix and SiLU; "ragged_n" adds a
    partial last 8-column chunk (scalar fallback beside the vector chunks of the same rows)."""
    M, K = 11 * 256 - 40, 192
    N = 640 if case != "ragged_n" else 644
    a, w = bf(rnd(M, K)), bf(rnd(N, K, scale=K ** -0.5))
    bias = rnd(N)
    if case == "rmap_mix_silu":
        r_div = 97
        nq = -(-M // r_div)
        rmap = torch.randperm(nq).to(torch.int32)
        res = bf(rnd(nq * r_div, N))
        mix = bf(rnd(M, N))
        out = ops.gemm(a.to(dev), w.to(dev), bias=bias.to(dev), residual=res.to(dev), rmap=rmap.to(dev), r_div=r_div,
                       r_mod=nq, rmap_max=nq - 1, act=ops.ACT_SILU, mix=mix.to(dev), mix_alpha=0.3, tile=tile)
        rows = torch.arange(M)
        rr = rmap[rows // r_div].long() * r_div + rows % r_div
        refo = 0.3 * mix.float() + 0.7 * F.silu(a.float() @ w.float().t() + bias + res.float()[rr])
    elif case in ("res_mix", "bias_only", "rowbias", "rb_res"):
        # the fast-path epilogue combinations (compile-time bias / row bias / residual / mix choice)
        res, mix, rowb = bf(rnd(M, N)), bf(rnd(M, N)), rnd(-(-M // 700), N)
        kw = dict(bias=bias.to(dev))
        refo = a.float() @ w.float().t() + bias
        if case in ("res_mix", "rb_res"):
            kw["residual"] = res.to(dev)
            refo = refo + res.float()
        if case in ("rowbias", "rb_res"):
            kw.update(rowbias=rowb.to(dev), rb_div=700)
            refo = refo + rowb.repeat_interleave(700, 0)[:M]
        if case == "res_mix":
            kw.update(mix=mix.to(dev), mix_alpha=0.3)
            refo = 0.3 * mix.float() + 0.7 * refo
        out = ops.gemm(a.to(dev), w.to(dev), tile=tile, **kw)
    else:
        res = bf(rnd(M, N))
        out = ops.gemm(a.to(dev), w.to(dev), bias=bias.to(dev), residual=res.to(dev), tile=tile)
        refo = a.float() @ w.float().t() + bias + res.float()
    assert out.shape == (M, N)
    assert rel(out, refo) < 1e-2
    # every row, including the ragged last tile, individually
    err_rows = ((out.float().cpu() - refo).norm(dim=1) / refo.norm(dim=1)).max().item()
    assert err_rows < 2e-2, err_rows


def test_gemm_host_bounds_checks(dev):
    """ops.gemm refuses operands the kernel would read or write out of bounds."""
    from actalker_amd._lib import ActhError
    a, w = bf(rnd(300, 64)).to(dev), bf(rnd(128, 64)).to(dev)
    with pytest.raises(ActhError):
        ops.gemm(a, w, residual=bf(rnd(299, 128)).to(dev))
    with pytest.raises(ActhError):
        ops.gemm(a, w, mix=bf(rnd(300, 64)).to(dev), mix_alpha=0.5)
    with pytest.raises(ActhError):
        ops.gemm(a, w, rowbias=rnd(2, 128).to(dev), rb_div=100)
    with pytest.raises(ActhError):
        ops.gemm(a, w, residual=bf(rnd(200, 128)).to(dev), rmap=torch.tensor([0, 1, 2], dtype=torch.int32, device=dev),
                 r_div=100, r_mod=3, rmap_max=2)
    with pytest.raises(ActhError):
        ops.gemm(a, w, out=torch.empty(300, 128, device=dev, dtype=ops.act_dtype()), orow=(100, 110, 0))


@pytest.mark.parametrize("tile", [1, 2, 3, 4, 5, 6, 7])
def test_gemm_tile_variants(dev, tile):
    """Every tile kernel (128x128; 256x256 / 256x160 8-wave; phased 256x256 / 256x320 / 256x128 / 256x64)
    on all A loaders, tails and epilogues."""
    from actalker_amd.modules import pack_conv3x3, pack_conv3d_t, pack_geglu
    # dense, ragged M/N/K + bias + residual + silu, fp32 out
    M, N, K = 700, 330, 200
    a, w = bf(rnd(M, K)), bf(rnd(N, K, scale=K ** -0.5))
    bias, res = rnd(N), bf(rnd(M, N))
    out = ops.gemm(a.to(dev), w.to(dev), bias=bias.to(dev), residual=res.to(dev), act=ops.ACT_SILU,
                   out_f32=True, tile=tile)
    assert rel(out, F.silu(a.float() @ w.float().t() + bias + res.float())) < 1e-2
    # two-source concat + mix + rowbias
    a2 = bf(rnd(M, 128))
    w2 = bf(rnd(N, 192 + 128, scale=320 ** -0.5))
    a1 = bf(rnd(M, 192))
    rowb = rnd(2, N)
    mix = bf(rnd(M, N))
    out = ops.gemm(a1.to(dev), w2.to(dev), a2=a2.to(dev), rowbias=rowb.to(dev), rb_div=350, mix=mix.to(dev),
                   mix_alpha=0.25, tile=tile)
    base = torch.cat([a1, a2], 1).float() @ w2.float().t() + rowb.repeat_interleave(350, 0)
    assert rel(out, 0.25 * mix.float() + 0.75 * base) < 1e-2
    # row bias changing every 100 rows (more images per row tile than the LDS-staged kernels hold)
    rowb7 = rnd(7, N)
    out = ops.gemm(a.to(dev), w.to(dev), rowbias=rowb7.to(dev), rb_div=100, tile=tile)
    assert rel(out, a.float() @ w.float().t() + rowb7.repeat_interleave(100, 0)) < 1e-2
    # conv3x3 with skip concat, stride 1 / 2 / upsample
    B, H, W, C1, C2, Co = 2, 12, 20, 128, 64, 320
    x1, x2 = bf(rnd(B, C1, H, W)), bf(rnd(B, C2, H, W))
    wc = bf(rnd(Co, C1 + C2, 3, 3, scale=(9 * (C1 + C2)) ** -0.5))
    tok = lambda t_: t_.permute(0, 2, 3, 1).reshape(-1, t_.shape[1]).contiguous().to(dev)
    for mode in ("s1", "s2", "up"):
        st = 2 if mode == "s2" else 1
        Ho, Wo = (H * 2, W * 2) if mode == "up" else ((H - 1) // st + 1, (W - 1) // st + 1)
        out = ops.gemm(tok(x1), pack_conv3x3(wc).to(dev), a2=tok(x2),
                       conv=dict(H=H, W=W, Ho=Ho, Wo=Wo, stride=st, upsample=mode == "up", B=B), tile=tile)
        xr = torch.cat([x1, x2], 1).float()
        if mode == "up":
            xr = F.interpolate(xr, scale_factor=2.0, mode="nearest")
        refo = F.conv2d(xr, wc.float(), None, stride=st, padding=1)
        assert rel(out, refo.permute(0, 2, 3, 1).reshape(-1, Co)) < 1e-2, mode
    # temporal (3,1,1)
    Bt, Ft, S, C, Co = 2, 7, 40, 128, 160
    x = bf(rnd(Bt, C, Ft, 5, 8))
    wt = bf(rnd(Co, C, 3, 1, 1, scale=(3 * C) ** -0.5))
    tk = x.permute(0, 2, 3, 4, 1).reshape(-1, C).contiguous()
    out = ops.gemm(tk.to(dev), pack_conv3d_t(wt).to(dev), temporal=dict(F=Ft, S=S), tile=tile)
    refo = F.conv3d(x.float(), wt.float(), None, padding=(1, 0, 0)).permute(0, 2, 3, 4, 1).reshape(-1, Co)
    assert rel(out, refo) < 1e-2
    # GEGLU (the 256x160 tile rejects it: its wave tiles do not hold whole hidden|gate granule pairs)
    Mg, Cg, inner = 600, 192, 640
    xg = bf(rnd(Mg, Cg))
    wg, bg = rnd(2 * inner, Cg, scale=Cg ** -0.5), rnd(2 * inner, scale=0.1)
    wp, bp = pack_geglu(wg, bg)
    if tile in (3, 5, 6, 7):
        with pytest.raises(Exception):
            ops.gemm(xg.to(dev), wp.to(dev), bias=bp.to(dev), act=ops.ACT_GEGLU, tile=tile)
    else:
        out = ops.gemm(xg.to(dev), wp.to(dev), bias=bp.to(dev), act=ops.ACT_GEGLU, tile=tile)
        h, g = (xg.float() @ bf(wg).float().t() + bg).chunk(2, -1)
        assert rel(out, h * F.gelu(g)) < 1e-2


@pytest.mark.parametrize("tile", [4, 5, 6, 7])
def test_gemm_ring_matches_phased(dev, tile):
    """The phased kernels' ring main loop (tile bit 0x1000) against their 4-phase loop (0x2000): both add the
    K chunks to every accumulator in the same order, so the outputs are bitwise equal -- dense with a ragged K
    tail (K % 32 = 8), two-source concat, conv3x3 stride 1 / 2 / upsample with a skip concat, temporal (3,1,1)
    and GEGLU."""
    from actalker_amd.modules import pack_conv3x3, pack_conv3d_t, pack_geglu

    def both(*args, **kw):
        return ops.gemm(*args, tile=tile | 0x1000, **kw), ops.gemm(*args, tile=tile | 0x2000, **kw)

    M, N, K = 1100, 330, 200
    a, w = bf(rnd(M, K)), bf(rnd(N, K, scale=K ** -0.5))
    r, o = both(a.to(dev), w.to(dev), bias=rnd(N).to(dev), residual=bf(rnd(M, N)).to(dev))
    assert torch.equal(r, o)
    a1, a2, w2 = bf(rnd(M, 192)), bf(rnd(M, 128)), bf(rnd(N, 320, scale=320 ** -0.5))
    r, o = both(a1.to(dev), w2.to(dev), a2=a2.to(dev), rowbias=rnd(4, N).to(dev), rb_div=300)
    assert torch.equal(r, o)
    B, H, W, C1, C2, Co = 2, 12, 20, 128, 64, 320
    tok = lambda t_: t_.permute(0, 2, 3, 1).reshape(-1, t_.shape[1]).contiguous().to(dev)
    x1, x2 = tok(bf(rnd(B, C1, H, W))), tok(bf(rnd(B, C2, H, W)))
    wc = pack_conv3x3(bf(rnd(Co, C1 + C2, 3, 3, scale=(9 * (C1 + C2)) ** -0.5))).to(dev)
    for st, up in ((1, False), (2, False), (1, True)):
        Ho, Wo = (2 * H, 2 * W) if up else ((H - 1) // st + 1, (W - 1) // st + 1)
        cv = dict(H=H, W=W, Ho=Ho, Wo=Wo, stride=st, upsample=up, B=B)
        r, o = both(x1, wc, a2=x2, conv=cv)
        assert torch.equal(r, o), (st, up)
    x = bf(rnd(2 * 7 * 40, 128))
    wt = pack_conv3d_t(bf(rnd(160, 128, 3, 1, 1, scale=384 ** -0.5))).to(dev)
    r, o = both(x.to(dev), wt, temporal=dict(F=7, S=40))
    assert torch.equal(r, o)
    if tile == 4:
        wp, bp = pack_geglu(rnd(1280, 192, scale=192 ** -0.5), rnd(1280, scale=0.1))
        r, o = both(bf(rnd(600, 192)).to(dev), wp.to(dev), bias=bp.to(dev), act=ops.ACT_GEGLU)
        assert torch.equal(r, o)


def test_gemm_tall_skinny_auto_tile(dev):
    """The Mamba x_proj shape class (N = 2 (R + 32) <= 128 over >= 65536 rows, fp32 out) auto-selects
    the phased 256x128 kernel; ragged last row tile, N not a multiple of 16."""
    M, N, K = 256 * 260 - 37, 104, 640
    a, w = bf(rnd(M, K)), bf(rnd(N, K, scale=K ** -0.5))
    out = ops.gemm(a.to(dev), w.to(dev), out_f32=True)
    assert out.dtype == torch.float32
    assert rel(out, a.float() @ w.float().t()) < 1e-2
    # conv_out class: 3x3 conv to 4 channels over >= 32768 output rows (256x64 tile), fp32 out + bias
    from actalker_amd.modules import pack_conv3x3
    B, H, W, C = 4, 72, 128, 320
    x = bf(rnd(B, C, H, W))
    wc = bf(rnd(4, C, 3, 3, scale=(9 * C) ** -0.5))
    bias = rnd(4)
    tok = x.permute(0, 2, 3, 1).reshape(-1, C).contiguous().to(dev)
    out = ops.conv3x3(tok, pack_conv3x3(wc).to(dev), B, H, W, bias=bias.to(dev), out_f32=True)
    refo = F.conv2d(x.float(), wc.float(), bias, padding=1).permute(0, 2, 3, 1).reshape(-1, 4)
    assert rel(out, refo) < 1e-2


@pytest.mark.parametrize("B,H,W,C1,C2,Cout,mode", [
    (2, 9, 16, 64, 0, 128, "s1"), (3, 18, 32, 128, 64, 192, "s1"), (2, 9, 16, 128, 0, 128, "s2"),
    (2, 9, 16, 64, 0, 64, "up"), (1, 36, 64, 320, 320, 320, "s1")])
def test_conv3x3(dev, B, H, W, C1, C2, Cout, mode):
    from actalker_amd.modules import pack_conv3x3
    x1 = bf(rnd(B, C1, H, W))
    x2 = bf(rnd(B, C2, H, W)) if C2 else None
    xin = torch.cat([x1, x2], 1) if C2 else x1
    Cin = C1 + C2
    w = bf(rnd(Cout, Cin, 3, 3, scale=(9 * Cin) ** -0.5))
    bias = rnd(Cout)
    tok = lambda t: t.permute(0, 2, 3, 1).reshape(-1, t.shape[1]).contiguous().to(dev)
    kw = dict(stride=2) if mode == "s2" else dict(upsample=True) if mode == "up" else {}
    out = ops.conv3x3(tok(x1), pack_conv3x3(w).to(dev), B, H, W, x2=tok(x2) if C2 else None,
                      bias=bias.to(dev), **kw)
    xr = xin.float()
    if mode == "up":
        xr = F.interpolate(xr, scale_factor=2.0, mode="nearest")
    refo = F.conv2d(xr, w.float(), bias, stride=2 if mode == "s2" else 1, padding=1)
    assert rel(out, refo.permute(0, 2, 3, 1).reshape(-1, Cout)) < 1e-2


@pytest.mark.parametrize("tile,N", [(5, 320), (4, 256), (5, 640)])
@pytest.mark.parametrize("OD", [576, 144])
def test_gemm_orow_remap_fast_epilogue(dev, tile, N, OD):
    """Output-row remap (row m -> (m / OD) * OS + m % OD: the Mamba in_proj writing S-token images into
    L-row scan sequences) through the phased kernels' fast epilogue -- taken when every wave's rows lie in one
    remap group (OD % 32 == 0 at 256x320, % 64 at 256x256: 576) -- and the generic one (OD = 144), with bias
    and residual; the slots between groups stay untouched."""
    g = torch.Generator().manual_seed(OD + N)
    K, OS = 320, OD + 33
    M = 5 * OD + OD // 2
    a = bf(rnd(M, K, g=g))
    w = bf(rnd(N, K, scale=K ** -0.5, g=g))
    b = rnd(N, g=g)
    r = bf(rnd(M, N, g=g))
    ngrp = -(-M // OD)
    out = torch.zeros(ngrp * OS, N, device=dev, dtype=ops.act_dtype())
    ops.gemm(a.to(dev), w.to(dev), bias=b.to(dev), residual=r.to(dev), out=out, orow=(OD, OS, 0), tile=tile)
    src = torch.arange(M)
    dst = (src // OD) * OS + src % OD
    want = a.float() @ w.float().t() + b + r.float()
    got = out.cpu()
    assert rel(got[dst], want) < 1e-2
    keep = torch.ones(ngrp * OS, dtype=torch.bool)
    keep[dst] = False
    assert got[keep].abs().max().item() == 0.0


def test_gemm_over_2gib(dev):
    """A operands past the 2 GiB buffer extent run as row chunks (acth_gemm's descriptor rebasing):
    a strided dense A inside 4.5 GB rows (the mode-2 x_proj read of Mamba xz) with row-bias images and
    residual, and a 3x3 conv over a 2.2 GB image batch; checked on rows / images at the chunk seams
    against torch fp32 (rows are computed independently, so any row is as good as any other)."""
    from actalker_amd.modules import pack_conv3x3
    g = torch.Generator(device=dev).manual_seed(7)
    M, K, LDA, N, RB = 1_100_000, 1024, 2048, 128, 9216
    big = torch.randn(M, LDA, device=dev, generator=g, dtype=torch.float32).to(ops.act_dtype())
    a = big[:, :K]                                   # 4.5 GB rows, 2.25 GB operand extent
    w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(ops.act_dtype())
    rowb = torch.randn(-(-M // RB), N, device=dev, generator=g)
    res = torch.randn(M, N, device=dev, generator=g).to(ops.act_dtype())
    out = ops.gemm(a, w, rowbias=rowb, rb_div=RB, residual=res)
    chunk = ((1 << 30) - 65536) // (RB * LDA) * RB   # first chunk's rows (whole row-bias images)
    for r0 in (0, chunk - 700, chunk, M - 1000):
        rows = slice(r0, r0 + 1000)
        ref_rows = (a[rows].float() @ w.float().t() + rowb[torch.arange(r0, r0 + 1000, device=dev) // RB]
                    + res[rows].float())
        assert rel(out[rows], ref_rows) < 1e-2, r0
    # output-row remap across the chunks (Mamba in_proj writing S-token images into L = S + 33 row
    # slots, modules.SS2D_cond_v10): chunks are whole remap groups, C rebased by group
    OD, OS = 9216, 9249
    ngrp = -(-M // OD)
    outr = torch.zeros(ngrp * OS, N, device=dev, dtype=ops.act_dtype())
    ops.gemm(a, w, out=outr, orow=(OD, OS, 0))
    chunk = ((1 << 30) - 65536) // (OD * LDA) * OD
    for r0 in (0, chunk - 700, chunk, M - 1000):
        src = torch.arange(r0, r0 + 1000, device=dev)
        dst = (src // OD) * OS + src % OD
        assert rel(outr[dst], a[r0:r0 + 1000].float() @ w.float().t()) < 1e-2, r0
    pad = torch.arange(OD, OS, device=dev)                       # the slots between groups stay untouched
    assert outr[pad].abs().max().item() == 0.0 and outr[pad + (ngrp - 1) * OS].abs().max().item() == 0.0
    del big, a, res, out, outr
    torch.cuda.empty_cache()
    # conv: 190 images of 72 x 128 x 640 -> 2.24 GB of A
    B, H, W, Cin, Cout = 190, 72, 128, 640, 320
    x = torch.randn(B * H * W, Cin, device=dev, generator=g).to(ops.act_dtype())
    wc = (torch.randn(Cout, Cin, 3, 3, device=dev, generator=g) * (9 * Cin) ** -0.5).to(ops.act_dtype())
    out = ops.conv3x3(x, pack_conv3x3(wc), B, H, W)
    per = (1 << 30) // (H * W * Cin)                 # images per chunk
    for b in (0, per - 1, per, B - 1):
        img = x[b * H * W:(b + 1) * H * W].float().cpu().view(1, H, W, Cin).permute(0, 3, 1, 2)
        refo = F.conv2d(img, wc.float().cpu(), padding=1).permute(0, 2, 3, 1).reshape(-1, Cout)
        assert rel(out[b * H * W:(b + 1) * H * W], refo) < 1e-2, b


def test_conv_temporal(dev):
    from actalker_amd.modules import pack_conv3d_t
    B, F_, H, W, C, Co = 2, 5, 6, 8, 128, 64
    x = bf(rnd(B, C, F_, H, W))
    w = bf(rnd(Co, C, 3, 1, 1, scale=(3 * C) ** -0.5))
    bias = rnd(Co)
    tok = x.permute(0, 2, 3, 4, 1).reshape(-1, C).contiguous()
    out = ops.gemm(tok.to(dev), pack_conv3d_t(w).to(dev), temporal=dict(F=F_, S=H * W), bias=bias.to(dev))
    refo = F.conv3d(x.float(), w.float(), bias, padding=(1, 0, 0)).permute(0, 2, 3, 4, 1).reshape(-1, Co)
    assert rel(out, refo) < 1e-2


# ------------------------------------------------------------------------------------------ attention
@pytest.mark.parametrize("nb,S,heads", [(2, 64, 1), (3, 200, 2), (1, 1024, 5), (1, 144, 20), (1, 2304, 2), (2, 2100, 1)])
def test_flash_attn(dev, nb, S, heads):
    C = heads * 64
    qkv = bf(rnd(nb * S, 3 * C))
    out = ops.flash_attn(qkv.to(dev), nb, S, heads)
    q, k, v = qkv.float().view(nb, S, 3, heads, 64).permute(2, 0, 3, 1, 4)
    refo = F.scaled_dot_product_attention(q, k, v).permute(0, 2, 1, 3).reshape(nb * S, C)
    assert rel(out, refo) < 1e-2


def test_flash_attn_peaked_scores(dev):
    """Large logits force many online-softmax rescales across key blocks."""
    nb, S, heads = 1, 512, 2
    C = heads * 64
    qkv = rnd(nb * S, 3 * C)
    qkv[:, :C] *= 6.0
    qkv = bf(qkv)
    out = ops.flash_attn(qkv.to(dev), nb, S, heads)
    q, k, v = qkv.float().view(nb, S, 3, heads, 64).permute(2, 0, 3, 1, 4)
    refo = F.scaled_dot_product_attention(q, k, v).permute(0, 2, 1, 3).reshape(nb * S, C)
    assert rel(out, refo) < 2e-2


@pytest.mark.parametrize("sign", [1.0, -1.0])
def test_flash_attn_drifting_scores(dev, sign):
    """Scores that grow (sign +1) or fall (-1) steadily across key blocks, far past the deferred-max
    threshold: the kernel's running max must be raised tile after tile (or never)."""
    nb, S, heads = 2, 1000, 1
    C = heads * 64
    g = torch.Generator().manual_seed(3)
    d = torch.randn(64, generator=g)
    d = d / d.norm()
    q = d.expand(nb * S, 64) * 8.0 + 0.1 * torch.randn(nb * S, 64, generator=g)
    ramp = torch.linspace(-1.0, 1.0, S).repeat(nb)[:, None] * sign
    k = d.expand(nb * S, 64) * 12.0 * ramp + 0.5 * torch.randn(nb * S, 64, generator=g)
    v = torch.randn(nb * S, 64, generator=g)
    qkv = bf(torch.cat([q, k, v], 1))
    out = ops.flash_attn(qkv.to(dev), nb, S, heads)
    qf, kf, vf = qkv.float().view(nb, S, 3, heads, 64).permute(2, 0, 3, 1, 4)
    refo = F.scaled_dot_product_attention(qf, kf, vf).permute(0, 2, 1, 3).reshape(nb * S, C)
    assert torch.isfinite(out.float()).all()
    assert rel(out, refo) < 2e-2


@pytest.mark.parametrize("B,F_,S,heads", [(2, 14, 37, 5), (1, 3, 16, 2), (4, 16, 9, 1), (2, 25, 37, 5), (3, 17, 9, 2),
                                          (1, 32, 16, 1)])
def test_temporal_attn(dev, B, F_, S, heads):
    C = heads * 64
    qkv = bf(rnd(B * F_ * S, 3 * C))
    out = ops.temporal_attn(qkv.to(dev), B, F_, S, heads)
    t = qkv.float().view(B, F_, S, 3, heads, 64).permute(3, 0, 2, 4, 1, 5)   # (3, B, S, H, F, 64)
    o = F.scaled_dot_product_attention(t[0], t[1], t[2])                     # (B, S, H, F, 64)
    refo = o.permute(0, 3, 1, 2, 4).reshape(B * F_ * S, C)
    assert rel(out, refo) < 1e-2


@pytest.mark.parametrize("masked,fps,nk,use_vb", [(False, 1, 32, True), (True, 1, 32, True), (False, 3, 7, False),
                                                   (False, 48, 32, True)])
def test_ip_attn(dev, masked, fps, nk, use_vb):
    """fps = frames per context (1: spatial attn2, context = frame; >1: temporal attn2, context =
    window, rows_per_ctx = fps * S; 48 x 50 rows exercises the 8-wave path)."""
    nctx, S, heads = 3, 50, 2
    C = heads * 64
    rpc = fps * S
    M = nctx * rpc
    q = bf(rnd(M, C))
    kv = bf(rnd(nctx * nk, 2 * C))
    vbase = bf(rnd(nctx, C))
    vb = bf(rnd(nctx, C)) if use_vb else None
    ma = torch.rand(S) if masked else None
    mb = torch.rand(S) if masked else None
    out = ops.ip_attn(vbase.to(dev), M, heads, rpc, S, q=q.to(dev), kv=kv.to(dev), nkeys=nk,
                      vb=None if vb is None else vb.to(dev), mask_a=None if ma is None else ma.to(dev),
                      mask_b=None if mb is None else mb.to(dev), sa=1.25, sb=0.75)
    qh = q.float().view(nctx, rpc, heads, 64).transpose(1, 2)
    kh = kv.float()[:, :C].view(nctx, nk, heads, 64).transpose(1, 2)
    vh = kv.float()[:, C:].view(nctx, nk, heads, 64).transpose(1, 2)
    o = F.scaled_dot_product_attention(qh, kh, vh).transpose(1, 2).reshape(nctx, rpc, C)
    wa = (ma if masked else torch.ones(S)).repeat(fps)[None, :, None]
    refo = vbase.float()[:, None] + 1.25 * wa * o
    if use_vb:
        wb = (mb if masked else torch.ones(S)).repeat(fps)[None, :, None]
        refo = refo + 0.75 * wb * vb.float()[:, None]
    assert rel(out, refo.reshape(M, C)) < 1e-2
    # 1-key-only path (no audio attention): pure broadcast
    out2 = ops.ip_attn(vbase.to(dev), M, heads, rpc, S)
    assert rel(out2, vbase.float().repeat_interleave(rpc, 0)) < 5e-3


@pytest.mark.parametrize("fps,masked,use_a,use_b", [(1, True, True, True), (1, False, True, False),
                                                   (3, False, True, True), (1, True, False, True),
                                                   (1, False, False, False)])
def test_xattn_fused_block(dev, fps, masked, use_a, use_b):
    """acth_ip_fold + acth_xattn: norm2 -> IP-adapter cross attention (ID + 32-key audio + VASA, per-token
    masks) -> to_out + residual -> norm3 in one kernel, against torch fp32 of the unfused ops
    (attention_processor.py:2747-2934 + attention.py:223-343). fps = frames per context (1: spatial attn2,
    context = frame; 3: temporal attn2, context = window). C = 320, 5 heads; S = 256 tokens per frame."""
    nctx, S, heads = 3, 256, 5
    C = heads * 64
    rpc = fps * S
    M = nctx * rpc
    h = bf(rnd(M, C, scale=2.0) + 0.5)
    g2, b2, g3, b3 = 1 + 0.1 * rnd(C), 0.1 * rnd(C), 1 + 0.1 * rnd(C), 0.1 * rnd(C)
    wq, wo = bf(rnd(C, C, scale=C ** -0.5)), bf(rnd(C, C, scale=C ** -0.5))
    bo = 0.1 * rnd(C)
    kv = bf(rnd(nctx * 32, 2 * C)) if use_a else None
    vid = bf(rnd(nctx, C))
    vb = bf(rnd(nctx, C)) if use_b else None
    ma = torch.rand(S) if masked else None
    mb = torch.rand(S) if masked else None
    tod = lambda t: None if t is None else t.to(dev)   # noqa: E731
    kp, vp, gb, base, vbw = ops.ip_fold(wq.to(dev), wo.t().contiguous().to(dev), bo.to(dev), vid.to(dev),
                                        kv=tod(kv), vb=tod(vb), heads=heads, norm2=(g2.to(dev), b2.to(dev)))
    out, n3 = ops.xattn(h.to(dev), 1e-5, (g3.to(dev), b3.to(dev), 1e-5), base, heads=heads, rows_per_ctx=rpc, S=S,
                        kp=kp, vp=vp, gb=gb, vbw=vbw, mask_a=tod(ma), mask_b=tod(mb), sa=1.25, sb=0.75)
    n = F.layer_norm(h.float(), (C,), g2, b2, 1e-5)
    a = vid.float().repeat_interleave(rpc, 0)
    if use_a:
        q = (n @ wq.float().t()).view(nctx, rpc, heads, 64).transpose(1, 2)
        kh = kv.float()[:, :C].view(nctx, 32, heads, 64).transpose(1, 2)
        vh = kv.float()[:, C:].view(nctx, 32, heads, 64).transpose(1, 2)
        o = F.scaled_dot_product_attention(q, kh, vh).transpose(1, 2).reshape(M, C)
        wa = (ma if masked else torch.ones(S)).repeat(fps).repeat(nctx)[:, None]
        a = a + 1.25 * wa * o
    if use_b:
        wb = (mb if masked else torch.ones(S)).repeat(fps).repeat(nctx)[:, None]
        a = a + 0.75 * wb * vb.float().repeat_interleave(rpc, 0)
    ref_out = h.float() + a @ wo.float().t() + bo
    ref_n3 = F.layer_norm(ref_out, (C,), g3, b3, 1e-5)
    assert rel(out, ref_out) < 1e-2, rel(out, ref_out)
    assert rel(n3, ref_n3) < 1e-2, rel(n3, ref_n3)
    # the attention increment h' - h on its own (the residual h dominates the norm of h'): within the bf16
    # rounding of the output at |h| plus 1e-2
    hf = h.float()
    inc, inc_ref = out.float().cpu() - hf, ref_out - hf
    floor = rel(bf(ref_out).float() - hf, inc_ref)
    assert rel(inc, inc_ref) < floor + 1e-2, (rel(inc, inc_ref), floor)
    # norm3 left to the feed-forward kernel: the same h', no n3
    out2, none = ops.xattn(h.to(dev), 1e-5, None, base, heads=heads, rows_per_ctx=rpc, S=S,
                           kp=kp, vp=vp, gb=gb, vbw=vbw, mask_a=tod(ma), mask_b=tod(mb), sa=1.25, sb=0.75)
    assert none is None and torch.equal(out2, out)


# ------------------------------------------------------------------------------------------ norms
def test_layernorm_and_add(dev):
    M, C = 300, 640
    x = bf(rnd(M, C, scale=3.0) + 1.0)
    g, b = rnd(C), rnd(C)
    out = ops.layernorm(x.to(dev), g.to(dev), b.to(dev), 1e-5)
    assert rel(out, F.layer_norm(x.float(), (C,), g, b, 1e-5)) < 1e-2
    add = bf(rnd(3, C))
    s = torch.empty(M, C, device=dev, dtype=ops.act_dtype())
    out = ops.layernorm(x.to(dev), g.to(dev), b.to(dev), 1e-5, add=add.to(dev), add_div=100, sum_out=s)
    xs = bf(x.float() + add.float().repeat_interleave(100, 0)).float()
    assert rel(s, xs) < 5e-3
    assert rel(out, F.layer_norm(xs, (C,), g, b, 1e-5)) < 1e-2


@pytest.mark.parametrize("C1,C2,silu,temporal", [(320, 0, True, False), (640, 320, True, False),
                                                  (1280, 1280, False, False), (320, 0, True, True)])
def test_groupnorm(dev, C1, C2, silu, temporal):
    B, F_, S = 2, 3, 48
    C = C1 + C2
    x1 = bf(rnd(B * F_ * S, C1, scale=2.0) + 0.5)
    x2 = bf(rnd(B * F_ * S, C2)) if C2 else None
    g, b = rnd(C), rnd(C)
    rps = F_ * S if temporal else S
    out = ops.groupnorm(x1.to(dev), g.to(dev), b.to(dev), 1e-6, rps, x2=None if x2 is None else x2.to(dev),
                        silu=silu)
    xf = torch.cat([x1, x2], 1).float() if C2 else x1.float()
    nst = xf.shape[0] // rps
    xr = xf.view(nst, rps, C).permute(0, 2, 1)                     # (nstat, C, rows)
    yr = F.group_norm(xr, 32, g, b, 1e-6)
    if silu:
        yr = F.silu(yr)
    assert rel(out, yr.permute(0, 2, 1).reshape(-1, C)) < 1e-2
    # bit-reproducible (fixed-order block reductions; fp64 cross-block sums)
    for _ in range(3):
        again = ops.groupnorm(x1.to(dev), g.to(dev), b.to(dev), 1e-6, rps, x2=None if x2 is None else x2.to(dev),
                              silu=silu)
        assert torch.equal(again, out)


def test_groupnorm_large_rows_reproducible(dev):
    """Level-0 sized statistics batches (many stats blocks per batch, 320 channels)."""
    M, C, rps = 2 * 9216, 320, 9216
    x = bf(rnd(M, C, scale=3.0) + 1.0).to(dev)
    g, b = rnd(C).to(dev), rnd(C).to(dev)
    out = ops.groupnorm(x, g, b, 1e-6, rps, silu=True)
    xr = x.float().cpu().view(2, rps, C).permute(0, 2, 1)
    ref_y = F.silu(F.group_norm(xr, 32, g.cpu(), b.cpu(), 1e-6)).permute(0, 2, 1).reshape(M, C)
    assert rel(out, ref_y) < 1e-2
    for _ in range(3):
        assert torch.equal(ops.groupnorm(x, g, b, 1e-6, rps, silu=True), out)


# ------------------------------------------------------------------------------------------ scan
def _scan_case(nb, L, D, R, n_keep, g):
    u = bf(rnd(nb * L, D, g=g))
    xproj = rnd(2 * (R + 32), D, scale=D ** -0.5, g=g)
    dtw = (torch.rand(2, D, R, generator=g) * 2 - 1) * R ** -0.5
    dtb = torch.log(torch.expm1(torch.rand(2, D, generator=g) * 0.099 + 0.001))
    alog = torch.log(torch.arange(1, 17).float()).repeat(2 * D, 1) + 0.1 * rnd(2 * D, 16, g=g)
    Dp = 1 + 0.1 * rnd(2 * D, g=g)
    return u, xproj, dtw, dtb, alog, Dp


@pytest.mark.parametrize("nb,L,D,R,n_keep,nchunks", [
    (2, 40, 64, 4, 30, 1), (2, 40, 64, 4, 30, 3), (1, 300, 640, 20, 267, 1), (1, 300, 640, 20, 267, 5),
    (2, 97, 1280, 40, 64, 2), (1, 33, 2560, 80, 0, None), (3, 17, 128, 80, 17, 2), (1, 1000, 128, 20, 968, None),
    (2, 50, 72, 5, 40, 1), (3, 61, 200, 8, 61, 1)])
def test_selective_scan_fused(dev, nb, L, D, R, n_keep, nchunks):
    """nchunks: 1/None paired-lane single pass, > 1 two-pass chunked."""
    g = torch.Generator().manual_seed(nb * 1000 + L)
    u, xproj, dtw, dtb, alog, Dp = _scan_case(nb, L, D, R, n_keep, g)
    xdbl = u.float() @ bf(xproj).float().t()                        # (nb*L, 2*(R+32))
    y0, y1 = ops.selective_scan(u.to(dev), xdbl.to(dev), dtw.to(dev), dtb.to(dev), alog.to(dev), Dp.to(dev),
                                nb=nb, L=L, R=R, n_keep=n_keep, nchunks=nchunks)
    if n_keep == 0:
        return
    # oracle: reference layout (SS2D_Unit.forward_core + selective_scan_ref)
    W = R + 32
    x = u.float().view(nb, L, D).permute(0, 2, 1)                  # (nb, D, L)
    xs = torch.stack([x, torch.flip(x, dims=[-1])], 1)              # (nb, 2, D, L)
    x_dbl = torch.einsum("b k d l, k c d -> b k c l", xs, bf(xproj).float().view(2, W, D))
    dts, Bs, Cs = torch.split(x_dbl, [R, 16, 16], dim=2)
    dts = torch.einsum("b k r l, k d r -> b k d l", dts, dtw)
    out = ref.selective_scan_ref(xs.reshape(nb, 2 * D, L), dts.reshape(nb, 2 * D, L), -torch.exp(alog), Bs, Cs,
                                 Dp, delta_bias=dtb.reshape(-1), delta_softplus=True).view(nb, 2, D, L)
    r0 = out[:, 0, :, :n_keep].permute(0, 2, 1).reshape(-1, D)
    r1 = torch.flip(out[:, 1], dims=[-1])[:, :, :n_keep].permute(0, 2, 1).reshape(-1, D)
    assert rel(y0, r0) < 1e-2
    assert rel(y1, r1) < 1e-2


def _pad_xproj(xproj, R):
    """x_proj rows [dt (R) | B | C] per direction -> [dt (R) | 0 (R4 - R) | B | C] (SS2D_Unit.packed)."""
    W, D = R + 32, xproj.shape[1]
    R4 = (R + 3) // 4 * 4
    x = xproj.view(2, W, D)
    return torch.cat([x[:, :R], torch.zeros(2, R4 - R, D), x[:, R:]], 1).reshape(-1, D)


@pytest.mark.parametrize("nb,L,D,R,n_keep", [
    (2, 40, 64, 4, 30), (1, 300, 640, 20, 267), (2, 97, 1280, 40, 64), (1, 33, 2560, 80, 0), (3, 17, 128, 80, 17),
    (1, 1000, 128, 20, 968), (2, 50, 72, 5, 40), (3, 61, 200, 8, 61), (2, 23, 48, 1, 20), (1, 64, 256, 3, 5)])
@pytest.mark.parametrize("algo", [0, 1])
def test_selective_scan_quad(dev, nb, L, D, R, n_keep, algo, monkeypatch):
    """bf16 x_proj rows (algo 0: paired-lane kernel, 1: scan_quad_kernel): the reference's data flow with a
    half-precision x_dbl (mamba_layer.py:1521) -- the oracle scans the same bf16-rounded rows; dt padding
    columns (R % 4) must be ignored (filled with garbage here). Also == the paired-lane kernel fed those rows
    in fp32."""
    monkeypatch.setattr(ops, "SCAN_ALGO", algo)
    g = torch.Generator().manual_seed(nb * 1000 + L + R)
    u, xproj, dtw, dtb, alog, Dp = _scan_case(nb, L, D, R, n_keep, g)
    R4 = (R + 3) // 4 * 4
    xpad = _pad_xproj(bf(xproj).float(), R)
    xdbl = bf(u.float() @ xpad.t())                                 # (nb*L, 2*(R4+32)) bf16
    if R4 != R:                                                     # padding columns are ignored
        xv = xdbl.view(nb * L, 2, R4 + 32)
        xv[:, :, R:R4] = bf(torch.full((nb * L, 2, R4 - R), 7.0))
    args = dict(dt_w=dtw.to(dev), dt_b=dtb.to(dev), A_log=alog.to(dev), Dskip=Dp.to(dev), nb=nb, L=L, R=R,
                n_keep=n_keep)
    y0, y1 = ops.selective_scan(u.to(dev), xdbl.to(dev), **args)
    if n_keep == 0:
        return
    W = R + 32
    x = u.float().view(nb, L, D).permute(0, 2, 1)
    xs = torch.stack([x, torch.flip(x, dims=[-1])], 1)
    x_dbl = bf(torch.einsum("b k d l, k c d -> b k c l", xs, bf(xproj).float().view(2, W, D))).float()
    dts, Bs, Cs = torch.split(x_dbl, [R, 16, 16], dim=2)
    dts = torch.einsum("b k r l, k d r -> b k d l", dts, dtw)
    out = ref.selective_scan_ref(xs.reshape(nb, 2 * D, L), dts.reshape(nb, 2 * D, L), -torch.exp(alog), Bs, Cs,
                                 Dp, delta_bias=dtb.reshape(-1), delta_softplus=True).view(nb, 2, D, L)
    r0 = out[:, 0, :, :n_keep].permute(0, 2, 1).reshape(-1, D)
    r1 = torch.flip(out[:, 1], dims=[-1])[:, :, :n_keep].permute(0, 2, 1).reshape(-1, D)
    assert rel(y0, r0) < 1e-2
    assert rel(y1, r1) < 1e-2
    # the same rows in fp32 through the paired-lane kernel (unpadded layout)
    xf = xdbl.float().view(nb * L, 2, R4 + 32)
    xf = torch.cat([xf[:, :, :R], xf[:, :, R4:]], 2).reshape(nb * L, 2 * W).contiguous()
    p0, p1 = ops.selective_scan(u.to(dev), xf.to(dev), nchunks=1, **args)
    assert rel(y0, p0) < 4e-3 and rel(y1, p1) < 4e-3


@pytest.mark.parametrize("ca,cb", [
    ((2, 300, 640, 20, 267), (2, 45, 640, 20, 40)),        # same kernel config, different L / n_keep
    ((3, 97, 1280, 40, 64), (1, 33, 1280, 40, 33)),        # different nb
    ((2, 40, 64, 4, 30), (2, 40, 64, 8, 30)),              # different R: two launches
    ((2, 40, 64, 4, 0), (2, 50, 64, 4, 50))])              # one branch empty
@pytest.mark.parametrize("xdt", ["f32", "bf16", "bf16q"])
def test_selective_scan2_matches_single(dev, ca, cb, xdt, monkeypatch):
    """acth_selective_scan2 (both SS2D branches in one launch) == two acth_selective_scan calls, bit for bit."""
    monkeypatch.setattr(ops, "SCAN_ALGO", 1 if xdt == "bf16q" else 0)
    args, singles = [], []
    for i, (nb, L, D, R, n_keep) in enumerate((ca, cb)):
        g = torch.Generator().manual_seed(7 + i * 31 + L)
        u, xproj, dtw, dtb, alog, Dp = _scan_case(nb, L, D, R, n_keep, g)
        if xdt != "f32":
            xdbl = bf(u.float() @ _pad_xproj(bf(xproj).float(), R).t())
        else:
            xdbl = u.float() @ bf(xproj).float().t()
        a = dict(u=u.to(dev), xdbl=xdbl.to(dev), dt_w=dtw.to(dev), dt_b=dtb.to(dev), A_log=alog.to(dev),
                 Dskip=Dp.to(dev), nb=nb, L=L, R=R, n_keep=n_keep)
        args.append(a)
        singles.append(ops.selective_scan(**a))
    pair = ops.selective_scan2(args[0], args[1])
    for (p0, p1), (s0, s1) in zip(pair, singles):
        assert torch.equal(p0, s0) and torch.equal(p1, s1)


def test_selective_scan_fn_dropin(dev):
    """actalker_amd.selective_scan_interface.selective_scan_fn == mamba-ssm semantics (op mode)."""
    from actalker_amd.selective_scan_interface import selective_scan_fn
    g = torch.Generator().manual_seed(7)
    b, G, d, L, N = 2, 2, 64, 75, 16
    u = bf(rnd(b, G * d, L, g=g)).float()
    delta = rnd(b, G * d, L, scale=0.5, g=g)
    A = -torch.exp(0.3 * rnd(G * d, N, g=g))
    Bm, Cm = rnd(b, G, N, L, g=g), rnd(b, G, N, L, g=g)
    Dv, db = rnd(G * d, g=g), rnd(G * d, scale=0.1, g=g)
    out = selective_scan_fn(u.to(dev), delta.to(dev), A.to(dev), Bm.to(dev), Cm.to(dev), Dv.to(dev),
                            delta_bias=db.to(dev), delta_softplus=True)
    refo = ref.selective_scan_ref(u, delta, A, Bm, Cm, Dv, delta_bias=db, delta_softplus=True)
    assert out.shape == refo.shape
    assert rel(out, refo) < 1e-2
    # no host-side sign check (no sync per call): A = 0 is exact, A > 0 turns that channel's outputs to NaN
    A2 = A.clone()
    A2[3, :] = 0.0
    A2[5, 2] = 0.5
    out2 = selective_scan_fn(u.to(dev), delta.to(dev), A2.to(dev), Bm.to(dev), Cm.to(dev), Dv.to(dev),
                             delta_bias=db.to(dev), delta_softplus=True).cpu()
    ref2 = ref.selective_scan_ref(u, delta, A2, Bm, Cm, Dv, delta_bias=db, delta_softplus=True)
    assert torch.isnan(out2[:, 5]).all()
    keep = [c for c in range(G * d) if c != 5]
    assert rel(out2[:, keep], ref2[:, keep]) < 1e-2


# ------------------------------------------------------------------------------------------ misc
def test_timestep_embedding(dev):
    t = torch.tensor([0.25 * math.log(700.0), -1.3, 12.5, 20.0, 0.0, 7.0])
    for dim, flip in ((320, True), (256, True), (64, False)):
        out = ops.timestep_embedding(t.to(dev), dim, flip)
        assert rel(out, ref.timestep_embedding(t, dim, flip, 0)) < 5e-3


def test_layout_and_gather(dev):
    x = rnd(2, 3, 8, 5, 4)
    tok = ops.nchw_to_tokens(x.to(dev), out_dtype=torch.float32)
    torch.testing.assert_close(tok.cpu(), x.flatten(0, 1).permute(0, 2, 3, 1).reshape(-1, 8))
    back = ops.tokens_to_nchw(tok, 6, 5, 4)
    torch.testing.assert_close(back.cpu(), x.flatten(0, 1))
    src = bf(rnd(2 * 10, 16))
    idx = torch.tensor([9, 0, 4], dtype=torch.int32)
    dst = torch.zeros(2 * 6, 16, device=dev, dtype=ops.act_dtype())
    ops.gather_rows(src.to(dev), idx.to(dev), 2, 10, dst, 6)
    got = dst.cpu().view(2, 6, 16)
    assert torch.equal(got[:, :3], src.view(2, 10, 16)[:, idx.long()])
    fm = ops.frame_mean(src.to(dev), 2, 5, 2)
    refm = src.float().view(2, 5, 2, 16).mean(1).reshape(4, 16)
    assert rel(fm, refm) < 5e-3


@pytest.mark.parametrize("n_src,per,C,idx", [(2, 9216 * 3, 320, [0, 1, 1]), (4, 37, 8, [0, 1, 1, 3, 3, 1]),
                                             (3, 1, 8, [2, 0]), (1, 1033, 640, [0, 0, 0, 0]), (2, 5, 8, [])])
def test_gather_blocks_matches_index_select(dev, n_src, per, C, idx):
    """acth_gather_blocks (the UNet's CFG-prefix expand) is bitwise index_select over the batch blocks: repeated
    indices, one-row blocks, a block count that is not a multiple of the 1024-vector launch chunk, no indices."""
    src = bf(rnd(n_src * per, C)).to(dev)
    ix = torch.tensor(idx, dtype=torch.int32, device=dev)
    got = ops.gather_blocks(src, n_src, ix, max(idx) if idx else 0)
    want = src.view(n_src, per, C).index_select(0, ix.long()).reshape(-1, C)
    assert got.shape == want.shape and torch.equal(got, want)
    with pytest.raises(Exception):
        ops.gather_blocks(src, n_src, ix, n_src)             # host bound outside the source blocks
    with pytest.raises(Exception):
        ops.gather_blocks(src[:, :C - 1], n_src, ix, 0)      # rows not contiguous


def test_cfg_euler_accum(dev):
    F_, S, T = 3, 10, 6
    noise = rnd(4 * F_ * S, 4)
    lat = rnd(T * S, 4) * 5
    fidx = torch.tensor([4, 5, 0], dtype=torch.int32)
    offs = torch.tensor([0, F_ * S, 2 * F_ * S, 3 * F_ * S], dtype=torch.int64)
    acc = torch.zeros(T * S, 4, device=dev)
    cnt = torch.zeros(T, device=dev)
    ops.cfg_euler_accum(noise.to(dev), offs.to(dev), lat.to(dev), fidx.to(dev), 2.0, 7.5, 3.0, 3.7, 2.1, acc, cnt,
                        F_, S)
    u, dav, dv, c = noise.view(4, F_, S, 4)
    eps = u + 2.0 * (dav - u) + 7.5 * (dv - dav) + 3.0 * (c - dv)
    x = lat.view(T, S, 4)[fidx.long()]
    xn = ref.euler_step_v(eps, 3.7, 2.1, x)
    got = acc.cpu().view(T, S, 4)
    torch.testing.assert_close(got[fidx.long()], xn, rtol=1e-5, atol=1e-5)
    assert cnt.cpu().tolist() == [1, 0, 0, 0, 1, 1]


def test_cfg_euler_accum_matches_reference_scheduler_mirror(dev):
    """acth_cfg_euler_accum's Euler part at all 25 Karras steps against the REFERENCE scheduler mirror's
    ``step`` (scheduling_euler_discrete.py:80-207, tests/golden/euler_mirror.safetensors): with
    g1 = g2 = g3 = 0 the guided prediction is the uncond branch, so the kernel's output is exactly one
    v-prediction Euler step of it. fp32 state: rtol 1e-5."""
    import os
    from safetensors.torch import load_file
    g = load_file(os.path.join(os.path.dirname(__file__), "golden", "euler_mirror.safetensors"))
    _, F_, C, h, w = g["sample"].shape[1:]
    S = h * w
    sig = g["sigmas"].tolist()
    rows = lambda t: t.reshape(F_, C, S).permute(0, 2, 1).reshape(F_ * S, C).contiguous()   # noqa: E731
    for i in range(25):
        mo = rows(g["model_out"][i])
        noise = torch.cat([mo, torch.zeros(3 * F_ * S, C)]).to(dev)
        offs = torch.tensor([0, F_ * S, 2 * F_ * S, 3 * F_ * S], dtype=torch.int64, device=dev)
        lat = rows(g["sample"][i]).to(dev)
        fidx = torch.arange(F_, dtype=torch.int32, device=dev)
        acc = torch.zeros(F_ * S, C, device=dev)
        cnt = torch.zeros(F_, device=dev)
        ops.cfg_euler_accum(noise, offs, lat, fidx, 0.0, 0.0, 0.0, sig[i], sig[i + 1], acc, cnt, F_, S)
        want = rows(g["prev"][i])
        torch.testing.assert_close(acc.cpu(), want, rtol=1e-5, atol=1e-5 * (1 + sig[i]))


def test_empty_inputs_give_empty_outputs(dev):
    """Zero rows / an empty batch through the ops and the selective_scan_fn drop-in: empty outputs of the right shape,
    no launch (the C ABI's no-work rule, include/actalker_hip.h), as the torch ops they replace accept."""
    from actalker_amd.selective_scan_interface import selective_scan_fn
    dt = ops.act_dtype()
    x = torch.empty(0, 64, device=dev, dtype=dt)
    w = bf(rnd(32, 64)).to(dev)
    assert ops.gemm(x, w).shape == (0, 32)
    g, b = torch.ones(64, device=dev), torch.zeros(64, device=dev)
    assert ops.layernorm(x, g, b, 1e-5).shape == (0, 64)
    assert ops.groupnorm(x, g, b, 1e-6, 16, silu=True).shape == (0, 64)
    assert ops.flash_attn(torch.empty(0, 3 * 64, device=dev, dtype=dt), 0, 16, 1).shape[0] == 0
    u = torch.empty(0, 64, 12, device=dev, dtype=dt)
    A = -torch.rand(64, 16, device=dev)
    Bc = torch.empty(0, 2, 16, 12, device=dev, dtype=dt)
    y = selective_scan_fn(u, u, A, Bc, Bc, D=torch.ones(64, device=dev), delta_bias=torch.zeros(64, device=dev),
                          delta_softplus=True)
    assert y.shape == (0, 64, 12)
    torch.cuda.synchronize()
