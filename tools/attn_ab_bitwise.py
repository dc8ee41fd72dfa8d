"""Bitwise A/B of the attention kernels of two library builds in one process (schedule-only changes
must not move a bit): self- and cross-attention forward + backward at the config-A shapes.
Usage: python tools/attn_ab_bitwise.py <libA.so> <libB.so>"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch  # noqa: E402
from ltx_amd import _lib, ops  # noqa: E402

B, N, L, H, d = 8, 1792, 256, 32, 64
D = H * d


def run(which):
    g = torch.Generator(device="cpu").manual_seed(5)
    Nk = N if which == "self" else L
    q = torch.randn(B * N, D, generator=g).bfloat16().cuda()
    k = torch.randn(B * Nk, D, generator=g).bfloat16().cuda()
    v = torch.randn(B * Nk, D, generator=g).bfloat16().cuda()
    do = torch.randn(B * N, D, generator=g).bfloat16().cuda()
    bias = None
    if which == "cross":
        bias = torch.zeros(B, Nk, device="cuda")
        bias[:, 16:] = -9984.0
    o, lse = ops.attn_fwd(q, k, v, B, H, d, d ** -0.5, key_bias=bias)
    dq, dk, dv = ops.attn_bwd(q, k, v, o, do, lse, B, H, d, d ** -0.5, key_bias=bias)
    torch.cuda.synchronize()
    return [t.clone() for t in (o, lse, dq, dk, dv)]


res = {}
for path in sys.argv[1:3]:
    _lib._lib = None
    _lib.load(path)
    res[path] = {w: run(w) for w in ("self", "cross")}
a, b = (res[p] for p in sys.argv[1:3])
ok = True
for w in ("self", "cross"):
    for name, x, y in zip(("O", "lse", "dQ", "dK", "dV"), a[w], b[w]):
        same = torch.equal(x, y)
        ok &= same
        print(f"{w} {name}: {'bitwise equal' if same else 'DIFFERS max %.3e' % (x.float() - y.float()).abs().max()}")
sys.exit(0 if ok else 1)
