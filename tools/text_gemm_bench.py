"""Text-side GEMMs of one block at config A (shared prompt: M = 256 text rows): the merged K/V
projection with its LoRA K-extension (forward) and the encoder-gradient GEMM over [dK_raw | dV]
(backward). Run under rocprofv3 --kernel-trace --stats for per-kernel durations; the variant is
picked by the environment (an LTX_* switch under test)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch
from ltx_amd import ops

g = torch.Generator(device="cuda").manual_seed(0)
L, D, K2 = 256, 2048, 128
enc = torch.randn(L, D, device="cuda", generator=g).bfloat16()
wkv = (torch.randn(2 * D, D, device="cuda", generator=g) / 45).bfloat16()
a2 = torch.randn(L, K2, device="cuda", generator=g).bfloat16()
w2 = (torch.randn(2 * D, K2, device="cuda", generator=g) / 8).bfloat16()
dkv = torch.randn(L, 2 * D, device="cuda", generator=g).bfloat16()
wkvT = wkv.t().contiguous()
w2b = (torch.randn(D, K2, device="cuda", generator=g) / 8).bfloat16()
fw = lambda: ops.gemm(enc, wkv, ext=(a2, w2))
bw = lambda: ops.gemm(dkv, wkvT, ext=(a2, w2b))
ref_f = enc.float() @ wkv.float().t() + a2.float() @ w2.float().t()
ref_b = dkv.float() @ wkvT.float().t() + a2.float() @ w2b.float().t()
ef = float((fw().float() - ref_f).norm() / ref_f.norm())
eb = float((bw().float() - ref_b).norm() / ref_b.norm())
for _ in range(200):
    fw()
    bw()
torch.cuda.synchronize()
print(f"blocks={os.environ.get('LTX_GEMM_SMALL_BLOCKS', '256')} rel_fwd={ef:.2e} rel_bwd={eb:.2e}", flush=True)
