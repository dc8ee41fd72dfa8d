"""Fixed vs per-K cost of the large-tile GEMM at M = 14336, N = 2048 (plain store and the
accumulate epilogue): time per launch for K = 256 .. 8192, HIP events, interleaved rounds."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch
from ltx_amd import ops

M, N = 14336, 2048


def timeit(fn, iters=30):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


ops_ = []
for K in (256, 512, 1024, 2048, 4096, 8192):
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ops_.append((f"store K={K}", K, lambda x=x, w=w, out=out: ops.gemm(x, w, out=out)))
    if K == 2048:
        res = torch.randn(M, N, device="cuda").bfloat16()
        ops_.append((f"accum K={K}", K, lambda x=x, w=w, out=out, res=res: ops.gemm(x, w, out=out, epilogue="accum", aux0=res)))
for rnd in range(2):
    for name, K, fn in ops_:
        us = timeit(fn)
        print(f"{name:>14}: {us:8.1f} us  {2.0 * M * N * K / us / 1e6:7.1f} TF", flush=True)

# the in-step K = 2048 forms: accumulate + LoRA K-extension (attn2 out-proj / q dgrad), store +
# delta row-dot (out-proj dgrads), gated residual (attn1 out-proj)
K = 2048
x = torch.randn(M, K, device="cuda").bfloat16()
w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
res = torch.randn(M, N, device="cuda").bfloat16()
K2 = ops.lora_k2(16)
a2 = torch.randn(M, K2, device="cuda").bfloat16()
w2 = torch.randn(N, K2, device="cuda").bfloat16() * 0.01
o = torch.randn(M, N, device="cuda").bfloat16()
delta = torch.empty(8, N // 64, M // 8, device="cuda", dtype=torch.float32)
gate = torch.randn(8, N, device="cuda").bfloat16()
bias = torch.randn(N, device="cuda").bfloat16()
forms = [("accum+ext", lambda: ops.gemm(x, w, out=out, epilogue="accum", aux0=res, ext=(a2, w2))),
         ("store+ext", lambda: ops.gemm(x, w, out=out, ext=(a2, w2))),
         ("rowdot", lambda: ops.gemm(x, w, out=out, epilogue="store_rowdot", aux0=o, aux1=delta, rank=64,
                                     rows_per_batch=M // 8)),
         ("gated_res", lambda: ops.gemm(x, w, bias=bias, out=out, epilogue="gated_residual", aux0=res,
                                        aux1=gate, rows_per_batch=M // 8))]
for rnd in range(2):
    for name, fn in forms:
        try:
            us = timeit(fn)
            print(f"{name:>14}: {us:8.1f} us  {2.0 * M * N * K / us / 1e6:7.1f} TF", flush=True)
        except Exception as e:  # noqa: BLE001
            print(name, "failed:", e)
