"""The attn2 cross-attention kernels exactly as a config-A training step calls them (B = 8,
N = 1792 queries, one shared 256-token prompt with 16 valid tokens: kv_shared, key bias -10000 on the
padding keys, delta precomputed by the dO GEMM), timed with HIP events; the rocprofv3 target for
their per-kernel traces and PMC passes (--iters small).
  --env-ab NAME: time with NAME cycling through --env-vals, interleaved rounds (A/B in one process).
  LTX_CROSS_ROTATE=1: rotate four q / dO sets (operands HBM-resident, as in the training step; the same
  operands every call stay in the Infinity Cache and hide the store pattern)."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch  # noqa: E402
from ltx_amd import _lib, ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=50)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--env-ab", default=None)
ap.add_argument("--env-vals", default="0,1")
ap.add_argument("--valid", type=int, default=16, help="valid caption tokens")
ap.add_argument("--check", action="store_true", help="compare the --env-vals settings' outputs")
args = ap.parse_args()
B, N, L, H, d = 8, 1792, 256, 32, 64
D = H * d
dev = "cuda"
_lib.ensure_device(dev)
g = torch.Generator(device="cpu").manual_seed(0)
rotate = os.environ.get("LTX_CROSS_ROTATE", "0") == "1"  # 4 operand sets: HBM-resident, as in the step
qs = [torch.randn(B * N, D, generator=g).to(dev, torch.bfloat16) for _ in range(4 if rotate else 1)]
q = qs[0]
kv = torch.randn(L, 2 * D, generator=g).to(dev, torch.bfloat16)
k, v = kv[:, :D], kv[:, D:]
bias = torch.zeros(1, L)
bias[:, args.valid:] = -10000.0
bias = bias.to(dev)
dos = [torch.randn(B * N, D, generator=g).to(dev, torch.bfloat16) for _ in range(4 if rotate else 1)]
do = dos[0]
scale = d ** -0.5


rot = iter(range(1 << 30))


def run_fwd():
    qq = qs[next(rot) % len(qs)]
    return ops.attn_fwd(qq, k, v, B, H, d, scale, key_bias=bias, kv_shared=True)


o, lse = run_fwd()
delta = (do.float() * o.float()).view(B, N, H, d).sum(-1).transpose(1, 2).contiguous()


def run_bwd():
    i = next(rot) % len(qs)
    return ops.attn_bwd(qs[i], k, v, o, dos[i], lse, B, H, d, scale, key_bias=bias, kv_shared=True, delta=delta)


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


# HBM bytes a launch must move: q (+ o written) forward; q, do read, dq written backward (+ the
# per-batch dK / dV rows of the shared keys); K / V / lse / delta are small
fwd_bytes = 2 * B * N * D * 2 + B * H * N * 4
bwd_bytes = 3 * B * N * D * 2 + 2 * B * L * D * 2 + 2 * B * H * N * 4
vals = args.env_vals.split(",") if args.env_ab else [None]
outs = {}
for rd in range(args.rounds):
    for val in vals:
        if val is not None:
            os.environ[args.env_ab] = val
        tf, tb = timeit(run_fwd, args.iters), timeit(run_bwd, args.iters)
        tag = f"{args.env_ab}={val}" if val is not None else "default"
        print(f"{tag} round {rd}: fwd {tf:.1f} us ({fwd_bytes / tf / 1e6:.2f} TB/s)  "
              f"bwd {tb:.1f} us ({bwd_bytes / tb / 1e6:.2f} TB/s)", flush=True)
        if args.check and rd == 0:
            outs[val] = (run_fwd(), run_bwd())
if args.check and len(outs) > 1:
    ref_key = vals[0]
    (o0, l0), (dq0, dk0, dv0) = outs[ref_key]
    for val in vals[1:]:
        (o1, l1), (dq1, dk1, dv1) = outs[val]
        for name, a_, b_ in (("O", o0, o1), ("lse", l0, l1), ("dQ", dq0, dq1), ("dK", dk0, dk1), ("dV", dv0, dv1)):
            same = torch.equal(a_, b_)
            err = float((a_.float() - b_.float()).abs().max())
            print(f"{args.env_ab}={val} vs {ref_key}: {name} bitwise {same} max abs diff {err:.3e}", flush=True)
