"""q/k RMSNorm + RoPE kernels at config A's self-attention size (M = 8 x 1792, D = 2048, the
batch-shared RoPE table train_step builds), HIP events; writes the outputs to a .pt file so two
library builds can be compared bitwise (tools/qk_norm_bench.py OUT.pt [REF.pt]).
Usage: LTX_HIP_LIB=... python tools/qk_norm_bench.py out.pt [ref.pt]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch  # noqa: E402
from ltx_amd import ops  # noqa: E402

B, N, D = 8, 1792, 2048
M = B * N
g = torch.Generator(device="cuda").manual_seed(0)
qkv = torch.randn(M, 3 * D, device="cuda", generator=g).bfloat16()
qw = (1 + 0.1 * torch.randn(D, device="cuda", generator=g)).bfloat16()
kw = (1 + 0.1 * torch.randn(D, device="cuda", generator=g)).bfloat16()
coords = ops.latent_coords(1, 7, 16, 16, "cuda").expand(B, -1, -1)
rope = ops.RopeSpec(coords, D, 10000.0, [20, 2048, 2048])
assert rope.cs_batch_rows == 0
dq = torch.randn(M, D, device="cuda", generator=g).bfloat16()
dk = torch.randn(M, D, device="cuda", generator=g).bfloat16()


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


fwd = lambda: ops.qk_norm_rope_fwd(qkv[:, :D], qkv[:, D:2 * D], qw, kw, rope)  # noqa: E731
q, k, rq, rk = fwd()
bwd = lambda: ops.qk_norm_rope_bwd(dq, qkv[:, :D], qw, rq, dk, qkv[:, D:2 * D], kw, rk, rope)  # noqa: E731
gq, gk = bwd()
for r in range(3):
    print(f"round {r}: qk_norm_rope_fwd {t(fwd):.1f} us  qk_norm_rope_bwd {t(bwd):.1f} us", flush=True)
out = {"q": q.cpu(), "k": k.cpu(), "rq": rq.cpu(), "rk": rk.cpu(), "gq": gq.cpu(), "gk": gk.cpu()}
torch.save(out, sys.argv[1])
if len(sys.argv) > 2:
    ref = torch.load(sys.argv[2], weights_only=True)
    same = {n: torch.equal(out[n], ref[n]) for n in out}
    print("bitwise vs", os.path.basename(sys.argv[2]), same, flush=True)
    if not all(same.values()):
        sys.exit(1)
