"""GEMM microbenchmark on the LTX-2B training shapes (M = 8 x 1792 tokens): TFLOP/s of the
libltxhip large-tile GEMM (variants of ltx_gemm_set_variant, default 0 = gemm_nt_kernel_t) and of
torch.matmul (hipBLASLt) on the same random bf16 operands, interleaved rounds in one process
(cdna_hip_programming.md 5.4 r24). Variants: env GEMM_VARIANTS (default "0,20")."""
import os, sys, json
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch
from ltx_amd import ops

M = 14336
SHAPES = [("qkv", M, 6144, 2048, "store"), ("out1", M, 2048, 2048, "store"),
          ("ff_up", M, 8192, 2048, "gelu"), ("ff_down", M, 2048, 8192, "store"),
          ("ff_up_dgrad", M, 2048, 8192, "store"), ("qkv_dgrad", M, 2048, 6144, "store"),
          ("ff_dgrad_gelu", M, 8192, 2048, "gelu_bwd")]
VARIANTS = [int(v) for v in os.environ.get("GEMM_VARIANTS", "0").split(",")]


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


res = {}
for name, m, n, k, epi in SHAPES:
    x = torch.randn(m, k, device="cuda").bfloat16()
    w = (torch.randn(n, k, device="cuda") / k ** 0.5).bfloat16()
    bias = torch.randn(n, device="cuda").bfloat16()
    pre = torch.empty(m, n, device="cuda", dtype=torch.int16) if epi == "gelu" else None
    if epi == "gelu_bwd":
        pre = (torch.rand(m, n, device="cuda") * 16384).to(torch.int16)  # the GELU derivative (snorm)
        bias = None
    out = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * m * n * k
    row = {}
    from ltx_amd import _lib
    for rnd in range(3):
        for var in VARIANTS:
            _lib.load().ltx_gemm_set_variant(var)
            ms = timeit(lambda: ops.gemm(x, w, bias=bias, epilogue=epi, aux0=pre, out=out))
            row.setdefault(f"ltx_v{var}", []).append(fl / ms / 1e9)
        _lib.load().ltx_gemm_set_variant(0)
        ms = timeit(lambda: torch.matmul(x, w.t()))
        row.setdefault("torch", []).append(fl / ms / 1e9)
    res[name] = {k2: round(max(v), 1) for k2, v in row.items()}
    print(f"{name:12s} M={m} N={n} K={k} {epi:6s} " + "  ".join(f"{k2} {v2:7.1f}" for k2, v2 in res[name].items()), flush=True)
print(json.dumps(res))
