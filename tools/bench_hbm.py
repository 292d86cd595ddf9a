"""HBM bandwidth probes with torch ops (write-only fill, read-only sum, copy) at GEMM-output sizes."""
import torch


def t(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters / 1e3


def main():
    dev = torch.device("cuda:0")
    for nbytes in (330 << 20, 1320 << 20):
        n = nbytes // 2
        x = torch.empty(n, device=dev, dtype=torch.bfloat16).normal_()
        y = torch.empty_like(x)
        s = t(lambda: y.fill_(1.0))
        print(f"fill  {nbytes / 2**20:.0f} MiB: {nbytes / s / 1e12:.2f} TB/s", flush=True)
        s = t(lambda: y.copy_(x))
        print(f"copy  {nbytes / 2**20:.0f} MiB: {2 * nbytes / s / 1e12:.2f} TB/s (read+write)", flush=True)
        s = t(lambda: x.sum(dtype=torch.float32))
        print(f"sum   {nbytes / 2**20:.0f} MiB: {nbytes / s / 1e12:.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
