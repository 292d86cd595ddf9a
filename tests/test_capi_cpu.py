"""CPU: the C-ABI library loads and exports every entry point include/actalker_hip.h declares;
argument validation rejects bad shapes before any launch (no GPU needed)."""
import ctypes
import os
import re

import pytest

from actalker_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "actalker_hip.h")


def header_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t)\s+(acth_\w+)\s*\(", src, flags=re.M)))


LIB_DTYPES = ["bf16", "fp16"]        # libactalker_hip.so and libactalker_hip_f16.so (ACTH_F16 build)


def load(which):
    import torch
    return _lib.load(torch.float16 if which == "fp16" else torch.bfloat16)


@pytest.mark.parametrize("which", LIB_DTYPES)
def test_library_exports_every_declared_symbol(which):
    lib = load(which)
    names = header_functions()
    assert len(names) >= 19
    for n in names:
        assert hasattr(lib, n), n
        assert n in _lib.SIGNATURES, f"{n} missing from the ctypes binding"
    assert set(_lib.SIGNATURES) == set(names)


@pytest.mark.parametrize("which", LIB_DTYPES)
def test_library_reports_its_activation_dtype(which):
    """Both builds export the same ABI; load() checks acth_act_dtype() so a bf16 build is never used for fp16."""
    assert load(which).acth_act_dtype() == (1 if which == "fp16" else 0)


@pytest.mark.parametrize("which", LIB_DTYPES)
def test_struct_layouts_match_header(which):
    lib = load(which)
    assert lib.acth_gemm_desc_size() == ctypes.sizeof(_lib.GemmDesc)
    src = open(HEADER).read()
    for cname, py in (("ActhGemmDesc", _lib.GemmDesc), ("ActhAttnDesc", _lib.AttnDesc),
                      ("ActhTemporalAttnDesc", _lib.TemporalAttnDesc), ("ActhIpAttnDesc", _lib.IpAttnDesc),
                      ("ActhLayerNormDesc", _lib.LayerNormDesc), ("ActhGroupNormDesc", _lib.GroupNormDesc),
                      ("ActhMambaCombineDesc", _lib.MambaCombineDesc), ("ActhScanDesc", _lib.ScanDesc),
                      ("ActhConvDirectDesc", _lib.ConvDirectDesc)):
        body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (cname, cname), src, flags=re.S).group(1)
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        fields = re.findall(r"(\w+)\s*(?:,|;)", body)
        assert fields == [f[0] for f in py._fields_], cname


@pytest.mark.parametrize("which", LIB_DTYPES)
def test_invalid_arguments_rejected_without_launch(which):
    lib = load(which)
    d = _lib.GemmDesc()
    d.M, d.N, d.K = 8, 8, 16
    assert lib.acth_gemm(ctypes.byref(d), None) == -1               # null operands
    d.A, d.B, d.C = 16, 16, 16
    d.M, d.N, d.K, d.lda, d.ldb, d.ldc = 8, 8, 12, 16, 16, 8           # K % 8 != 0
    assert lib.acth_gemm(ctypes.byref(d), None) == -1
    s = _lib.ScanDesc()
    s.u, s.xdbl, s.A_log, s.y0, s.dt_w = 16, 16, 16, 16, 16
    s.N, s.R, s.L, s.D, s.nb, s.G, s.ldx, s.ldu = 8, 4, 10, 64, 1, 2, 128, 64       # N != 16
    assert lib.acth_selective_scan(ctypes.byref(s), None) == -1
    a = _lib.TemporalAttnDesc()
    a.qkv, a.o, a.F, a.B, a.S, a.H = 16, 16, 33, 1, 1, 1                   # F > 32
    assert lib.acth_temporal_attn(ctypes.byref(a), None) == -1
    c = _lib.ConvDirectDesc()
    c.x, c.w, c.y, c.Cin, c.Cout, c.ldx, c.ldy, c.B, c.H, c.W, c.Ho, c.Wo = 16, 16, 16, 3, 16, 3, 16, 1, 8, 8, 8, 8
    c.stride = 3                                                            # stride must be 1 or 2
    assert lib.acth_conv_direct(ctypes.byref(c), None) == -1
    c.stride, c.Ho = 2, 8                                                   # Ho != (H-1)//2 + 1
    assert lib.acth_conv_direct(ctypes.byref(c), None) == -1
    assert lib.acth_softmax_rows(16, 4, 16, 8, 2, 8, 1.0, None) == -1        # ldx < cols


@pytest.mark.parametrize("which", LIB_DTYPES)
def test_zero_work_calls_are_noops(which):
    """A call with no rows / an empty batch returns ACTH_OK without reading its (here NULL) pointers, as the torch
    ops it replaces accept empty tensors; a negative size is still rejected."""
    lib = load(which)
    cases = [
        (lib.acth_gemm, _lib.GemmDesc, dict(N=8, K=16), "M"),
        (lib.acth_flash_attn, _lib.AttnDesc, dict(nheads=1, Sq=64, Skv=64), "nbatch"),
        (lib.acth_temporal_attn, _lib.TemporalAttnDesc, dict(F=14, S=4, H=1), "B"),
        (lib.acth_ip_attn, _lib.IpAttnDesc, dict(H=5, rows_per_ctx=64, S=64), "M"),
        (lib.acth_xattn, _lib.XattnDesc, dict(C=320, H=5, rows_per_ctx=64, S=64), "M"),
        (lib.acth_geglu_ffn, _lib.FfnDesc, dict(C=320), "M"),
        (lib.acth_layernorm, _lib.LayerNormDesc, dict(C=64), "M"),
        (lib.acth_groupnorm, _lib.GroupNormDesc, dict(C=64, C1=64, G=32, rows_per_stat=16), "M"),
        (lib.acth_mamba_combine_ln, _lib.MambaCombineDesc, dict(C=64, S=16), "M"),
        (lib.acth_selective_scan, _lib.ScanDesc, dict(N=16, R=4, L=64, D=64, G=2), "nb"),
        (lib.acth_conv_direct, _lib.ConvDirectDesc, dict(Cin=3, Cout=16, H=8, W=8), "B"),
    ]
    for fn, cls, fields, size in cases:
        d = cls()
        for k, v in fields.items():
            setattr(d, k, v)
        setattr(d, size, 0)
        assert fn(ctypes.byref(d), None) == 0, (fn.__name__, size)
        setattr(d, size, -1)
        assert fn(ctypes.byref(d), None) == -1, (fn.__name__, size)
    s0, s1 = _lib.ScanDesc(), _lib.ScanDesc()
    assert lib.acth_selective_scan2(ctypes.byref(s0), ctypes.byref(s1), None) == 0
    # block gather: no blocks (or empty blocks) is a no-op on NULL pointers; bad sizes are rejected first
    assert lib.acth_gather_blocks(None, 2, None, 0, 64, None, None) == 0
    assert lib.acth_gather_blocks(None, 2, None, 3, 0, None, None) == 0
    assert lib.acth_gather_blocks(None, 2, None, -1, 64, None, None) == -1
    assert lib.acth_gather_blocks(None, 2, None, 0, 24, None, None) == -1       # block_bytes % 16
    assert lib.acth_gather_blocks(None, 0, None, 0, 64, None, None) == -1       # no source blocks
    assert lib.acth_gather_blocks(None, 2, None, 3, 64, None, None) == -1       # work with NULL pointers


def test_no_cpu_fallback():
    import torch
    from actalker_amd import ops
    with pytest.raises(_lib.ActhError):
        ops.layernorm(torch.zeros(4, 8, dtype=torch.bfloat16), None, None)


def test_libraries_are_distinct_builds():
    import torch
    from actalker_amd import ops
    assert _lib.load(torch.float16) is not _lib.load(torch.bfloat16)
    assert ops.act_dtype() == torch.bfloat16
    with ops.compute_dtype(torch.float16):
        assert ops.act_dtype() == torch.float16
        with ops.compute_dtype(torch.bfloat16):
            assert ops.act_dtype() == torch.bfloat16
        assert ops.act_dtype() == torch.float16
    assert ops.act_dtype() == torch.bfloat16
    with pytest.raises(_lib.ActhError):
        with ops.compute_dtype(torch.float32):
            pass
