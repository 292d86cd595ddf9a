"""ctypes binding of libactalker_hip.so (the C ABI declared in include/actalker_hip.h).

The shared libraries are built in-tree by ``actalker_amd/csrc/Makefile`` (``__graft_entry__.build``): the
kernels with bf16 activations (libactalker_hip.so) and the same sources with fp16 activations
(libactalker_hip_f16.so, the reference's shipped weight_dtype). Both export the same C ABI.
There is deliberately no fallback: if a library cannot be loaded every op raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# ACTH_LIB overrides the in-tree library (A/B benchmarks of two builds in one GPU session)
LIB_PATH = os.environ.get("ACTH_LIB") or os.path.join(_HERE, "libactalker_hip.so")
LIB_PATH_F16 = os.environ.get("ACTH_LIB_F16") or os.path.join(_HERE, "libactalker_hip_f16.so")

def kernel_source_digest() -> str:
    """SHA-256 (16 hex digits) of the HIP kernel sources and the C ABI header: identifies the kernels a measured
    figure belongs to (PMC traffic files record it; bench.py drops figures recorded for other sources)."""
    import glob
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(_HERE, "csrc", "*.hip")) + glob.glob(os.path.join(_HERE, "csrc", "*.h")))
    files.append(os.path.join(os.path.dirname(_HERE), "include", "actalker_hip.h"))
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]



c_int = ctypes.c_int
c_float = ctypes.c_float
c_ll = ctypes.c_longlong
c_vp = ctypes.c_void_p
c_fp = ctypes.POINTER(ctypes.c_float)


class GemmDesc(ctypes.Structure):
    _fields_ = [
        ("A", c_vp), ("A2", c_vp), ("lda", c_int), ("lda2", c_int), ("K1", c_int),
        ("amode", c_int),
        ("H", c_int), ("W", c_int), ("Ho", c_int), ("Wo", c_int), ("conv_stride", c_int), ("upsample", c_int),
        ("Cin", c_int),
        ("F", c_int), ("S", c_int),
        ("B", c_vp), ("ldb", c_int),
        ("M", c_int), ("N", c_int), ("K", c_int),
        ("bias", c_vp),
        ("rowbias", c_vp), ("rb_div", c_int), ("ldrb", c_int),
        ("R", c_vp), ("ldr", c_int), ("rmap", c_vp), ("r_div", c_int), ("r_mod", c_int),
        ("MIX", c_vp), ("ldmix", c_int), ("mix_alpha", c_float),
        ("alpha", c_float),
        ("act", c_int),
        ("out_f32", c_int),
        ("C", c_vp), ("ldc", c_int),
        ("orow_div", c_int), ("orow_stride", c_int), ("orow_off", c_int),
        ("tile", c_int),
    ]


class AttnDesc(ctypes.Structure):
    _fields_ = [
        ("q", c_vp), ("k", c_vp), ("v", c_vp), ("o", c_vp),
        ("ldq", c_int), ("ldk", c_int), ("ldv", c_int), ("ldo", c_int),
        ("bsq", c_ll), ("bsk", c_ll), ("bsv", c_ll), ("bso", c_ll),
        ("nbatch", c_int), ("nheads", c_int), ("Sq", c_int), ("Skv", c_int),
        ("scale", c_float),
    ]


class TemporalAttnDesc(ctypes.Structure):
    _fields_ = [
        ("qkv", c_vp), ("ldqkv", c_int), ("o", c_vp), ("ldo", c_int),
        ("B", c_int), ("F", c_int), ("S", c_int), ("H", c_int),
        ("scale", c_float),
    ]


class IpAttnDesc(ctypes.Structure):
    _fields_ = [
        ("q", c_vp), ("ldq", c_int),
        ("kv", c_vp), ("ldkv", c_int), ("nkeys", c_int),
        ("vbase", c_vp), ("ldvbase", c_int),
        ("vb", c_vp), ("ldvb", c_int),
        ("mask_a", c_vp), ("mask_b", c_vp),
        ("sa", c_float), ("sb", c_float), ("scale", c_float),
        ("out", c_vp), ("ldo", c_int),
        ("M", c_int), ("H", c_int), ("rows_per_ctx", c_int), ("S", c_int),
    ]


class IpFoldDesc(ctypes.Structure):
    _fields_ = [
        ("kv", c_vp), ("ldkv", c_int),
        ("wq", c_vp), ("ldwq", c_int),
        ("wo", c_vp), ("ldwo", c_int),
        ("bo", c_vp),
        ("vid", c_vp), ("ldvid", c_int),
        ("vb", c_vp), ("ldvb", c_int),
        ("g2", c_vp), ("b2", c_vp),
        ("kscale", c_float),
        ("kp", c_vp), ("vp", c_vp),
        ("gb", c_vp),
        ("base", c_vp), ("vbw", c_vp),
        ("nctx", c_int), ("C", c_int), ("H", c_int),
    ]


class XattnDesc(ctypes.Structure):
    _fields_ = [
        ("h", c_vp), ("ldh", c_int),
        ("eps2", c_float),
        ("kp", c_vp), ("vp", c_vp),
        ("gb", c_vp),
        ("base", c_vp), ("ldbase", c_int),
        ("vbw", c_vp), ("ldvbw", c_int),
        ("mask_a", c_vp), ("mask_b", c_vp),
        ("sa", c_float), ("sb", c_float),
        ("g3", c_vp), ("b3", c_vp), ("eps3", c_float),
        ("out", c_vp), ("ldo", c_int),
        ("n3", c_vp), ("ldn3", c_int),
        ("M", c_int), ("C", c_int), ("H", c_int), ("rows_per_ctx", c_int), ("S", c_int),
    ]


class FfnDesc(ctypes.Structure):
    _fields_ = [
        ("x", c_vp), ("ldx", c_int),
        ("w1", c_vp), ("ldw1", c_int), ("b1", c_vp),
        ("w2", c_vp), ("ldw2", c_int), ("b2", c_vp),
        ("res", c_vp), ("ldres", c_int),
        ("mix", c_vp), ("ldmix", c_int), ("mix_alpha", c_float),
        ("y", c_vp), ("ldy", c_int),
        ("M", c_int), ("C", c_int),
        ("ln_g", c_vp), ("ln_b", c_vp), ("ln_eps", c_float), ("ln", c_int),
        ("add", c_vp), ("ldadd", c_int), ("add_div", c_int),
    ]


class LayerNormDesc(ctypes.Structure):
    _fields_ = [
        ("x", c_vp), ("ldx", c_int),
        ("add", c_vp), ("ldadd", c_int), ("add_div", c_int),
        ("sum_out", c_vp), ("ldsum", c_int),
        ("gamma", c_vp), ("beta", c_vp), ("eps", c_float),
        ("y", c_vp), ("ldy", c_int),
        ("M", c_int), ("C", c_int),
    ]


class GroupNormDesc(ctypes.Structure):
    _fields_ = [
        ("x", c_vp), ("ldx", c_int), ("x2", c_vp), ("ldx2", c_int), ("C1", c_int),
        ("M", c_int), ("C", c_int), ("G", c_int), ("rows_per_stat", c_int),
        ("gamma", c_vp), ("beta", c_vp), ("eps", c_float),
        ("silu", c_int),
        ("y", c_vp), ("ldy", c_int),
        ("ws", c_vp),
        ("res", c_vp), ("ldres", c_int),
    ]


class MambaCombineDesc(ctypes.Structure):
    _fields_ = [
        ("xa", c_vp), ("ldxa", c_int), ("ya0", c_vp), ("ya1", c_vp), ("ldya", c_int), ("La", c_int),
        ("pos_a", c_vp), ("mode_a", c_int),
        ("xe", c_vp), ("ldxe", c_int), ("ye0", c_vp), ("ye1", c_vp), ("ldye", c_int), ("Le", c_int),
        ("pos_e", c_vp), ("mode_e", c_int),
        ("gamma", c_vp), ("beta", c_vp), ("eps", c_float),
        ("y", c_vp), ("ldy", c_int),
        ("M", c_int), ("S", c_int), ("C", c_int),
    ]


class ScanDesc(ctypes.Structure):
    _fields_ = [
        ("u", c_vp), ("ldu", c_int),
        ("xdbl", c_vp), ("ldx", c_int),
        ("dt_w", c_vp), ("dt_b", c_vp), ("A_log", c_vp), ("Dskip", c_vp),
        ("y0", c_vp), ("y1", c_vp), ("ldy", c_int),
        ("nb", c_int), ("L", c_int), ("D", c_int), ("R", c_int), ("N", c_int), ("n_keep", c_int),
        ("delta", c_vp), ("ld_delta", c_int), ("delta_f32", c_int), ("softplus", c_int),
        ("G", c_int), ("u_gstride", c_int), ("y_gstride", c_int), ("flip1", c_int),
        ("nchunks", c_int), ("chunk_len", c_int), ("ws", c_vp),
        ("xdbl_bf16", c_int), ("scan_algo", c_int),
    ]


class ConvDirectDesc(ctypes.Structure):
    _fields_ = [
        ("x", c_vp), ("ldx", c_int),
        ("w", c_vp), ("bias", c_vp),
        ("y", c_vp), ("ldy", c_int),
        ("mode", c_int),
        ("B", c_int), ("H", c_int), ("W", c_int), ("Ho", c_int), ("Wo", c_int), ("stride", c_int),
        ("pad0", c_int),
        ("F", c_int), ("S", c_int),
        ("Cin", c_int), ("Cout", c_int), ("act", c_int), ("out_f32", c_int),
    ]


# Every symbol include/actalker_hip.h declares, with its ctypes signature.
_P = ctypes.POINTER
SIGNATURES = {
    "acth_gemm": ([_P(GemmDesc), c_vp], c_int),
    "acth_gemm_desc_size": ([], c_int),
    "acth_geglu_ffn": ([_P(FfnDesc), c_vp], c_int),
    "acth_debug_ffn_stamps": ([c_vp, c_int, c_int], c_int),
    "acth_flash_attn": ([_P(AttnDesc), c_vp], c_int),
    "acth_temporal_attn": ([_P(TemporalAttnDesc), c_vp], c_int),
    "acth_ip_attn": ([_P(IpAttnDesc), c_vp], c_int),
    "acth_ip_fold": ([_P(IpFoldDesc), c_vp], c_int),
    "acth_xattn": ([_P(XattnDesc), c_vp], c_int),
    "acth_debug_xattn_stamps": ([c_vp, c_int, c_int], c_int),
    "acth_layernorm": ([_P(LayerNormDesc), c_vp], c_int),
    "acth_im2col": ([c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_int,
                     c_vp], c_int),
    "acth_maxpool2d": ([c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_int,
                        c_vp], c_int),
    "acth_debug_gemm_stamps": ([c_vp, c_int], c_int),
    "acth_groupnorm": ([_P(GroupNormDesc), c_vp], c_int),
    "acth_groupnorm_workspace_size": ([c_int, c_int, c_int, c_int], ctypes.c_size_t),
    "acth_mamba_combine_ln": ([_P(MambaCombineDesc), c_vp], c_int),
    "acth_selective_scan": ([_P(ScanDesc), c_vp], c_int),
    "acth_selective_scan2": ([_P(ScanDesc), _P(ScanDesc), c_vp], c_int),
    "acth_selective_scan_workspace_size": ([c_int, c_int, c_int, c_int], ctypes.c_size_t),
    "acth_conv_direct": ([_P(ConvDirectDesc), c_vp], c_int),
    "acth_softmax_rows": ([c_vp, c_int, c_vp, c_int, c_int, c_int, c_float, c_vp], c_int),
    "acth_timestep_embedding": ([c_vp, c_int, c_int, c_int, c_float, c_float, c_float, c_vp, c_vp], c_int),
    "acth_nchw_to_tokens": ([c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_vp], c_int),
    "acth_tokens_to_nchw": ([c_vp, c_int, c_int, c_vp, c_int, c_int, c_int, c_int, c_vp], c_int),
    "acth_im2col3x3": ([c_vp, c_int, c_int, c_int, c_int, c_vp, c_int, c_vp], c_int),
    "acth_gather_rows": ([c_vp, c_int, c_int, c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_vp], c_int),
    "acth_frame_mean": ([c_vp, c_int, c_int, c_int, c_int, c_int, c_vp, c_int, c_vp], c_int),
    "acth_gather_blocks": ([c_vp, c_int, c_vp, c_int, ctypes.c_longlong, c_vp, c_vp], c_int),
    "acth_window_input": ([c_vp, c_vp, c_vp, c_vp, c_float, c_vp, c_int, c_int, c_int, c_int, c_vp], c_int),
    "acth_cfg_euler_accum": ([c_vp, c_vp, c_vp, c_vp, c_float, c_float, c_float, c_float, c_float, c_vp, c_vp,
                              c_int, c_int, c_vp], c_int),
    "acth_div_counter": ([c_vp, c_vp, c_vp, c_int, c_int, c_vp], c_int),
    "acth_version": ([], c_int),
    "acth_act_dtype": ([], c_int),
}

_libs = {}


class ActhError(RuntimeError):
    pass


def load(dtype=None):
    """Load the HIP library for the activation dtype (torch.bfloat16 -- the default -- or torch.float16), once.
    Raises if it is missing: there is no CPU fallback."""
    f16 = str(dtype) == "torch.float16"
    if f16 in _libs:
        return _libs[f16]
    path = LIB_PATH_F16 if f16 else LIB_PATH
    if not os.path.exists(path):
        raise ActhError(
            f"{path} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(or `make -C actalker_amd/csrc`). The ACTalker MI355X path has no fallback.")
    lib = ctypes.CDLL(path)
    for name, (argtypes, restype) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = restype
    if lib.acth_gemm_desc_size() != ctypes.sizeof(GemmDesc):
        raise ActhError("ActhGemmDesc layout mismatch between include/actalker_hip.h and _lib.py")
    if lib.acth_act_dtype() != int(f16):
        # both libraries export the same ABI: a bf16 build loaded for fp16 (or the reverse, e.g. a stale
        # ACTH_LIB_F16) would reinterpret every activation's bits
        raise ActhError(f"{path} was built for {'fp16' if lib.acth_act_dtype() else 'bf16'} activations, "
                        f"loaded for {'fp16' if f16 else 'bf16'}")
    _libs[f16] = lib
    return lib


_ERR = {-1: "invalid argument (shape/alignment rejected)", -2: "kernel launch failed"}


def check(rc: int, what: str):
    if rc != 0:
        raise ActhError(f"{what}: {_ERR.get(rc, rc)}")
