"""torch.matmul (hipBLASLt) on a few dense shapes, for a rocprofv3 kernel trace that names the library's kernels.

  rocprofv3 --kernel-trace --stats -d out -o run -- python3 tools/blas_names.py
"""
import torch

for M, N, K in [(8192, 8192, 8192), (48384, 10240, 1280), (193536, 5120, 640), (48384, 1280, 1280)]:
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    for _ in range(3):
        torch.matmul(x, w.t())
    torch.cuda.synchronize()
    print(M, N, K, flush=True)
