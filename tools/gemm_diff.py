"""Where does a GEMM variant differ from variant 0? (debug aid: per-row-in-tile / per-col-in-tile
/ per-tile counts of mismatching elements)
  python tools/gemm_diff.py VARIANT M N K [BMT]"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch
from ltx_amd import ops, _lib

v, M, N, K = (int(a) for a in sys.argv[1:5])
BMT = int(sys.argv[5]) if len(sys.argv) > 5 else 224
lib = _lib.load()
torch.manual_seed(0)
x = torch.randn(M, K, device="cuda").bfloat16()
w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
lib.ltx_gemm_set_variant(0)
c0 = ops.gemm(x, w)
lib.ltx_gemm_set_variant(v)
c1 = ops.gemm(x, w)
torch.cuda.synchronize()
bad = (c0 != c1)
print("mismatch fraction", float(bad.float().mean()))
r = bad.float().sum(1).view(-1, BMT).sum(0)
print("rows-in-tile with mismatches:", [i for i in range(BMT) if r[i] > 0][:64])
cc = bad.float().sum(0).view(-1, 256).sum(0)
print("cols-in-tile with mismatches:", [i for i in range(256) if cc[i] > 0][:64])
t = bad.float().view(M // BMT, BMT, N // 256, 256).sum((1, 3))
print("tiles with mismatches:", int((t > 0).sum()), "of", t.numel())
ref = x.float() @ w.float().t()
d0 = (c0.float() - ref).abs().max(); d1 = (c1.float() - ref).abs().max()
print("max abs err v0", float(d0), "v", float(d1))
# is the error a missing / doubled k-tile? compare against partial sums
for kt in range(K // 64):
    part = x[:, kt * 64:(kt + 1) * 64].float() @ w[:, kt * 64:(kt + 1) * 64].float().t()
    e = ((c1.float() - ref) - part).abs().mean() / (c1.float() - ref).abs().mean()
    e2 = ((c1.float() - ref) + part).abs().mean() / (c1.float() - ref).abs().mean()
    if e < 0.5 or e2 < 0.5:
        print("k-tile", kt, "explains the error: +part", float(e), "-part", float(e2))
