"""Attention kernels at the LTX-2B config-A shapes (self: B=8, N=1792, 32x64 heads, q/k/v in the
fused [M, 6144] layout; cross: Nk=256 with the key-padding bias), timed with HIP events; the PMC
target for rocprofv3 (--iters small)."""
import argparse, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch
from ltx_amd import ops

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--which", default="self,cross")
ap.add_argument("--env-ab", default=None, help="NAME: time each kernel with NAME=0 and NAME=1, interleaved")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--env-vals", default="0,1", help="the values --env-ab cycles through")
args = ap.parse_args()
B, N, L, H, d = 8, 1792, 256, 32, 64
D = H * d
dev = "cuda"
torch.manual_seed(0)


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


for which in args.which.split(","):
    Nk = N if which == "self" else L
    qkv = torch.randn(B * N, 3 * D, device=dev).bfloat16()
    kv = qkv if which == "self" else torch.randn(B * Nk, 2 * D, device=dev).bfloat16()
    q = qkv[:, :D]
    k = kv[:, D:2 * D] if which == "self" else kv[:, :D]
    v = kv[:, 2 * D:] if which == "self" else kv[:, D:]
    bias = None
    if which == "cross":
        bias = torch.zeros(B, Nk, device=dev)
        bias[:, 16:] = -9984.0
    scale = d ** -0.5
    o, lse = ops.attn_fwd(q, k, v, B, H, d, scale, key_bias=bias)
    do = torch.randn(B * N, D, device=dev).bfloat16()
    fwd = lambda: ops.attn_fwd(q, k, v, B, H, d, scale, key_bias=bias)
    bwd = lambda: ops.attn_bwd(q, k, v, o, do, lse, B, H, d, scale, key_bias=bias)
    prod = 2.0 * B * H * N * Nk * d
    if args.env_ab:
        for rd in range(args.rounds):
            for val in args.env_vals.split(","):
                os.environ[args.env_ab] = val
                tf, tb = timeit(fwd, args.iters), timeit(bwd, args.iters)
                print(f"{which} {args.env_ab}={val} round {rd}: fwd {tf * 1e3:.1f} us  bwd {tb * 1e3:.1f} us", flush=True)
        continue
    tf = timeit(fwd, args.iters)
    tb = timeit(bwd, args.iters)
    print(f"{which}: fwd {tf * 1e3:.1f} us ({2 * prod / tf / 1e9:.0f} TF)  bwd {tb * 1e3:.1f} us "
          f"(alg {4 * prod / tb / 1e9:.0f} TF, executed {7 * prod / tb / 1e9:.0f} TF)", flush=True)
