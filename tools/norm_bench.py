"""Times the row-normalisation kernels at config A's token shape (M = 14336 rows of D = 2048, 8
batches): rmsnorm_modulate fwd / bwd and the self-attention q/k RMSNorm + RoPE forward, HIP events,
rotating operands (no cache reuse between calls)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch  # noqa: E402
from ltx_amd import _lib, ops  # noqa: E402

B, N, D = 8, 1792, 2048
M = B * N
_lib.ensure_device("cuda")
gen = torch.Generator(device="cpu").manual_seed(0)


def g(*shape, scale=1.0):
    return (torch.randn(*shape, generator=gen) * scale).to("cuda", torch.bfloat16)


def timeit(fn, iters=50):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


xs = [g(M, D) for _ in range(4)]  # rotating operands: no L2 / Infinity-Cache reuse between calls
mod = g(B, 6 * D, scale=0.1)
shift, one = mod[:, :D], mod[:, D:2 * D]
it = iter(range(1 << 30))
res = {}
res["rmsnorm_fwd_us"] = timeit(lambda: ops.rmsnorm_modulate_fwd(xs[next(it) % 4], shift, one, mod.stride(0), N, 1e-6))
y, rstd = ops.rmsnorm_modulate_fwd(xs[0], shift, one, mod.stride(0), N, 1e-6)
res["rmsnorm_bwd_us"] = timeit(lambda: ops.rmsnorm_modulate_bwd(xs[next(it) % 4], xs[0], rstd, one, mod.stride(0), N,
                                                               dres=xs[1]))
coords = ops.latent_coords(1, 7, 16, 16, "cuda")
rope = ops.RopeSpec(coords.expand(B, -1, -1), D, 10000.0, [20, 2048, 2048])
qkvs = [g(M, 3 * D) for _ in range(2)]
qw, kw = g(D, scale=0.1) + 1, g(D, scale=0.1) + 1
res["qk_rope_fwd_us"] = timeit(lambda: ops.qk_norm_rope_fwd((q := qkvs[next(it) % 2])[:, :D], q[:, D:2 * D], qw, kw,
                                                             rope))
_, _, rq, rk = ops.qk_norm_rope_fwd(qkvs[0][:, :D], qkvs[0][:, D:2 * D], qw, kw, rope)


def qk_bwd():
    q = qkvs[next(it) % 2]
    return ops.qk_norm_rope_bwd(xs[next(it) % 4], q[:, :D], qw, rq, xs[1], q[:, D:2 * D], kw, rk, rope)


res["qk_rope_bwd_us"] = timeit(qk_bwd)
print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)
