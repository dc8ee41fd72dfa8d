"""A/B of the large-tile GEMM variants (ltx_gemm_set_variant) on the training shapes, interleaved
rounds in one process; also a PMC target: `--only V --shape NAME --iters I` runs one config."""
import argparse, os, sys, json
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch
from ltx_amd import ops, _lib

M = 14336
SHAPES = {"ff_up_gelu": (M, 8192, 2048, "gelu"), "n8192_k8192": (M, 8192, 8192, "store"),
          "qkv": (M, 6144, 2048, "store"), "n2048_k2048": (M, 2048, 2048, "store"),
          "n2048_k8192": (M, 2048, 8192, "store"),
          "out1_gres": (M, 2048, 2048, "gated_residual"), "ffdown_gres": (M, 2048, 8192, "gated_residual"),
          "o2_accum": (M, 2048, 2048, "accum"), "ffdgrad_gelubwd": (M, 8192, 2048, "gelu_bwd")}
ROWS = 1792  # rows per batch (gated residual gates)


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


ap = argparse.ArgumentParser()
ap.add_argument("--variants", default="0,1,2")
ap.add_argument("--only", type=int, default=None)
ap.add_argument("--shape", default=None)
ap.add_argument("--shapes", default=None)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--torch", action="store_true")
ap.add_argument("--check", action="store_true")
args = ap.parse_args()
lib = _lib.load()
names = [args.shape] if args.shape else (args.shapes.split(",") if args.shapes else list(SHAPES))
res = {}
for name in names:
    m, n, k, epi = SHAPES[name]
    x = torch.randn(m, k, device="cuda").bfloat16()
    w = (torch.randn(n, k, device="cuda") / k ** 0.5).bfloat16()
    bias = torch.randn(n, device="cuda").bfloat16()
    pre = torch.empty(m, n, device="cuda", dtype=torch.int16) if epi == "gelu" else None
    aux1 = None
    if epi in ("gated_residual", "accum", "gelu_bwd"):
        pre = torch.randn(m, n, device="cuda").bfloat16()
    if epi == "gelu_bwd":  # the factor as the GELU forward keeps it: rint(32767 * gelu_tanh'(F) / 2) (ops.GELU_Q)
        pre = ops.gelu_grad_q(pre)
    if epi == "gated_residual":
        aux1 = torch.randn(m // ROWS, n, device="cuda").bfloat16()
    if epi in ("accum", "gelu_bwd"):
        bias = None
    c = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
    kw = dict(bias=bias, epilogue=epi, aux0=pre, aux1=aux1, rows_per_batch=ROWS if aux1 is not None else 0)
    fl = 2.0 * m * n * k
    if args.only is not None:
        if args.torch:
            ms = timeit(lambda: torch.matmul(x, w.t()), args.iters)
        else:
            lib.ltx_gemm_set_variant(args.only)
            ms = timeit(lambda: ops.gemm(x, w, out=c, **kw), args.iters)
        print(f"{name} {'torch' if args.torch else 'v%d' % args.only} {fl / ms / 1e9:.1f} TF")
        continue
    if args.check:
        outs = {}
        for v in [int(s2) for s2 in args.variants.split(",")]:
            lib.ltx_gemm_set_variant(v)
            c.fill_(0)
            ops.gemm(x, w, out=c, **kw)
            torch.cuda.synchronize()
            outs[v] = c.clone()
        lib.ltx_gemm_set_variant(0)
        ref = x.float() @ w.float().t() + (bias.float() if bias is not None else 0)
        if epi == "gelu":
            ref = torch.nn.functional.gelu(ref.bfloat16().float(), approximate="tanh")
        elif epi == "gated_residual":
            ref = pre.float() + aux1.float().repeat_interleave(ROWS, 0) * ref
        elif epi == "accum":
            ref = pre.float() + ref
        elif epi == "gelu_bwd":
            ref = ref.bfloat16().float() * pre.float() / ops.GELU_Q
        v0 = list(outs)[0]
        for v, o in outs.items():
            rel = float((o.float() - ref).norm() / ref.norm())
            print(f"check {name} v{v}: equal_to_v{v0}={torch.equal(o, outs[v0])} rel_vs_fp32={rel:.2e}", flush=True)
    row = {}
    for rnd in range(3):
        for v in [int(s) for s in args.variants.split(",")]:
            lib.ltx_gemm_set_variant(v)
            ms = timeit(lambda: ops.gemm(x, w, out=c, **kw))
            row.setdefault(f"v{v}", []).append(fl / ms / 1e9)
        ms = timeit(lambda: torch.matmul(x, w.t()))
        row.setdefault("torch", []).append(fl / ms / 1e9)
    lib.ltx_gemm_set_variant(0)
    res[name] = {k2: round(max(v2), 1) for k2, v2 in row.items()}
    print(f"{name:12s} " + "  ".join(f"{k2} {v2:7.1f}" for k2, v2 in res[name].items()), flush=True)
print(json.dumps(res))
