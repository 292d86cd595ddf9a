"""Time the fused level-0 GEGLU feed-forward (acth_geglu_ffn) against the two-GEMM path it replaces,
at the BASELINE geometry (M = 2 CFG x 14 frames x 72 x 128 tokens = 774144, C = 320)."""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from actalker_amd import ops  # noqa: E402
from actalker_amd.modules import pack_ffn_w2, pack_geglu  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=774144)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = "cuda"
    C, inner, M = 320, 1280, a.M
    g = torch.Generator().manual_seed(0)
    x = (torch.randn(M, C, generator=g)).to(torch.bfloat16).to(dev)
    res = (torch.randn(M, C, generator=g)).to(torch.bfloat16).to(dev)
    w1 = torch.randn(2 * inner, C, generator=g) * C ** -0.5
    b1 = torch.randn(2 * inner, generator=g) * 0.1
    w2 = torch.randn(C, inner, generator=g) * inner ** -0.5
    b2 = (torch.randn(C, generator=g) * 0.1).to(dev)
    wp, bp = (t.to(dev) for t in pack_geglu(w1, b1))
    w2p = pack_ffn_w2(w2).to(dev)
    w2b = w2.to(torch.bfloat16).to(dev)
    out = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
    hid = torch.empty(M, inner, device=dev, dtype=torch.bfloat16)

    def fused():
        ops.geglu_ffn(x, wp, bp, w2p, b2, residual=res, out=out)

    def two():
        ops.gemm(x, wp, bias=bp, act=ops.ACT_GEGLU, out=hid)
        ops.gemm(hid, w2b, bias=b2, residual=res, out=out)

    flops = 2.0 * M * C * (2 * inner) + 2.0 * M * inner * C
    tf = timeit(fused, a.reps)
    tt = timeit(two, a.reps)
    print(json.dumps({"M": M, "fused_ms": round(tf, 4), "two_gemm_ms": round(tt, 4),
                      "fused_tflops": round(flops / tf / 1e9, 1), "two_gemm_tflops": round(flops / tt / 1e9, 1)}))


if __name__ == "__main__":
    main()
