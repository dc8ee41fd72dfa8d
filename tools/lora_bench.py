"""LoRA skinny kernels at the LTX-2B shapes (M = 14336 image tokens / 2048 text tokens, 2048
features, r = 16): time per call and effective HBM rate of the big operand."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch
from ltx_amd import ops


def timeit(fn, iters=50):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


r, K, N = 16, 2048, 2048
for M in (14336, 2048):
    x = torch.randn(M, K, device="cuda").bfloat16()
    dy = torch.randn(M, N, device="cuda").bfloat16()
    A = torch.randn(r, K, device="cuda") / K ** 0.5
    Bm = torch.randn(N, r, device="cuda") * 0.05
    u = ops.lora_down(x, A)
    w = ops.lora_down(dy, Bm, alpha=0.5, transposed=True)
    gB = torch.zeros(N, r, device="cuda")
    gA = torch.zeros(r, K, device="cuda")
    gb = M * K * 2 / 1e9
    for name, fn in [("down A (split)", lambda: ops.lora_down(x, A, split=True)),
                     ("down B^T (split)", lambda: ops.lora_down(dy, Bm, alpha=0.5, transposed=True, split=True)),
                     ("wgrad dB", lambda: ops.lora_wgrad(dy, u, alpha=0.5, out=gB, accumulate=True)),
                     ("wgrad dA", lambda: ops.lora_wgrad(x, w, transpose_out=True, out=gA, accumulate=True))]:
        us = timeit(fn)
        print(f"M={M:6d} {name:18s} {us:7.1f} us  {gb / us * 1e6 / 1e3:6.2f} TB/s", flush=True)
