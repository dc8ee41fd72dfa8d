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
          "n2048_k8192": (M, 2048, 8192, "store")}


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
    pre = torch.empty(m, n, device="cuda", dtype=torch.bfloat16) if epi == "gelu" else None
    c = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * m * n * k
    if args.only is not None:
        if args.torch:
            ms = timeit(lambda: torch.matmul(x, w.t()), args.iters)
        else:
            lib.ltx_gemm_set_variant(args.only)
            ms = timeit(lambda: ops.gemm(x, w, bias=bias, epilogue=epi, aux0=pre, out=c), args.iters)
        print(f"{name} {'torch' if args.torch else 'v%d' % args.only} {fl / ms / 1e9:.1f} TF")
        continue
    if args.check:
        outs = {}
        for v in [int(s2) for s2 in args.variants.split(",")]:
            lib.ltx_gemm_set_variant(v)
            c.fill_(0)
            ops.gemm(x, w, bias=bias, epilogue=epi, aux0=pre, out=c)
            torch.cuda.synchronize()
            outs[v] = c.clone()
        lib.ltx_gemm_set_variant(0)
        ref = (x.float() @ w.float().t() + bias.float())
        if epi == "gelu":
            ref = torch.nn.functional.gelu(ref.bfloat16().float(), approximate="tanh")
        v0 = list(outs)[0]
        for v, o in outs.items():
            rel = float((o.float() - ref).norm() / ref.norm())
            print(f"check {name} v{v}: equal_to_v{v0}={torch.equal(o, outs[v0])} rel_vs_fp32={rel:.2e}", flush=True)
    row = {}
    for rnd in range(3):
        for v in [int(s) for s in args.variants.split(",")]:
            lib.ltx_gemm_set_variant(v)
            ms = timeit(lambda: ops.gemm(x, w, bias=bias, epilogue=epi, aux0=pre, out=c))
            row.setdefault(f"v{v}", []).append(fl / ms / 1e9)
        ms = timeit(lambda: torch.matmul(x, w.t()))
        row.setdefault("torch", []).append(fl / ms / 1e9)
    lib.ltx_gemm_set_variant(0)
    res[name] = {k2: round(max(v2), 1) for k2, v2 in row.items()}
    print(f"{name:12s} " + "  ".join(f"{k2} {v2:7.1f}" for k2, v2 in res[name].items()), flush=True)
print(json.dumps(res))
