"""Row kernels at config A's size (M = 14336, D = 2048): RMSNorm + modulate fwd / bwd, HIP events."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch
from ltx_amd import ops

M, D, B = 14336, 2048, 8
x = torch.randn(M, D, device="cuda").bfloat16()
mods = torch.randn(B, 6, D, device="cuda").bfloat16()


def t(fn, it=50):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


y = ops.rmsnorm_modulate_fwd(x, mods[:, 0], mods[:, 1], mods.stride(0), M // B, 1e-6)
print(f"rmsnorm_mod_fwd {t(lambda: ops.rmsnorm_modulate_fwd(x, mods[:, 0], mods[:, 1], mods.stride(0), M // B, 1e-6)):.1f} us", flush=True)
dy = torch.randn(M, D, device="cuda").bfloat16()
rstd = torch.rand(M, device="cuda") + 0.5
dres = torch.randn(M, D, device="cuda").bfloat16()
print(f"rmsnorm_mod_bwd {t(lambda: ops.rmsnorm_modulate_bwd(dy, x, rstd, mods[:, 1], mods.stride(0), M // B, dres=dres)):.1f} us", flush=True)
