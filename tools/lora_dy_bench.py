"""ltx_lora_dy (one pass over dY) against the two kernels it replaces (ltx_lora_rows on dY +
ltx_lora_wgrad for lora_B) at config A's token-sized adapter shape (M = 14336, N = 2048, r = 16)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch
from ltx_amd import ops

M, N, r = 14336, 2048, 16
dy = torch.randn(M, N, device="cuda").bfloat16()
u = torch.randn(M, r, device="cuda")
Bm = torch.randn(N, r, device="cuda") * 0.05
pieces = ops.lora_pieces(Bm, transposed=True)
buf = torch.zeros(N, r, device="cuda")


def timeit(fn, iters=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def two():
    ops.lora_wgrad(dy, u, alpha=0.5, out=buf, accumulate=True)
    ops.lora_rows(dy, pieces, r, alpha=0.5, split=True)


for rnd in range(3):
    t1 = timeit(lambda: ops.lora_dy(dy, u, pieces, r, 0.5, buf))
    t2 = timeit(two)
    t3 = timeit(lambda: ops.lora_rows(dy, pieces, r, alpha=0.5, split=True))
    print(f"lora_dy {t1:6.1f} us   rows + wgrad {t2:6.1f} us   rows alone {t3:6.1f} us", flush=True)
