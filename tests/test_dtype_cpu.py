"""CPU: activation-dtype selection (round 4). An fp16 UNet -- the reference's ``unet.to(weight_dtype)`` with the
shipped ``weight_dtype: fp16`` (Inference.py:168-173, 202; config/inference.yaml:66) -- computes with fp16
activations (libactalker_hip_f16.so), any other weight dtype with bf16; ``acth_compute_dtype`` overrides. Weight
packs are cached per dtype, so one module tree can serve both. No kernel runs here (no GPU)."""
import threading

import pytest
import torch

from actalker_amd import _lib, modules, ops
from tests import golden_unet_ref as gu


@pytest.fixture(scope="module")
def tiny_unet():
    return gu.build_hip_unet("tiny_mode0")


def test_compute_dtype_follows_weight_dtype(tiny_unet):
    unet = tiny_unet
    assert unet.compute_dtype() == torch.bfloat16              # fp32 weights
    unet.half()
    try:
        assert unet.compute_dtype() == torch.float16           # the reference's shipped fp16 UNet
        unet.acth_compute_dtype = torch.bfloat16
        assert unet.compute_dtype() == torch.bfloat16
    finally:
        unet.acth_compute_dtype = None
        unet.float()
    unet.to(torch.bfloat16)
    try:
        assert unet.compute_dtype() == torch.bfloat16
    finally:
        unet.float()


def test_weight_packs_are_cached_per_dtype(tiny_unet):
    lin = next(m for m in tiny_unet.modules() if isinstance(m, modules.Linear))
    w16 = None
    wb = lin.w()
    assert wb.dtype == torch.bfloat16
    with ops.compute_dtype(torch.float16):
        w16 = lin.w()
        assert w16.dtype == torch.float16
        assert lin.w() is w16                                   # cached
    assert lin.w() is wb                                        # the bf16 pack is still the bf16 one
    torch.testing.assert_close(w16.float(), wb.float(), rtol=1e-2, atol=1e-3)


def test_compute_dtype_is_thread_local():
    seen = {}
    go = threading.Event()

    def worker():
        go.wait()
        seen["other"] = ops.act_dtype()

    t = threading.Thread(target=worker)
    t.start()
    with ops.compute_dtype(torch.float16):
        go.set()
        t.join()
        assert ops.act_dtype() == torch.float16
    assert seen["other"] == torch.bfloat16
    assert ops.act_dtype() == torch.bfloat16


def test_fp16_forward_needs_the_gpu(tiny_unet):
    tiny_unet.acth_compute_dtype = torch.float16
    try:
        x = torch.zeros(1, 2, 8, 8, 8)
        with pytest.raises(RuntimeError):
            tiny_unet(x, 1.0, torch.zeros(2, 1, 1024), torch.zeros(1, 3))
    finally:
        tiny_unet.acth_compute_dtype = None


def test_unknown_dtype_rejected():
    with pytest.raises(_lib.ActhError):
        with ops.compute_dtype(torch.float32):
            pass
