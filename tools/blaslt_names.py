"""Which hipBLASLt kernels torch picks for the training GEMM shapes (names encode macro tile,
MFMA shape and wave layout); run under rocprofv3 --kernel-trace."""
import torch
M = 14336
for (n, k) in ((2048, 2048), (2048, 8192), (8192, 2048), (6144, 2048)):
    a = torch.randn(M, k, device="cuda").bfloat16()
    w = torch.randn(n, k, device="cuda").bfloat16()
    for _ in range(5):
        torch.matmul(a, w.t())
    torch.cuda.synchronize()
