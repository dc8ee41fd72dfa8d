"""GEMM time vs K at fixed M x N (fixed cost = prologue + epilogue + tail, slope = main loop):
libltxhip vs torch.matmul (hipBLASLt). Usage: python tools/gemm_scaling.py"""
import os, sys, json
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch
from ltx_amd import ops


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


M = 14336
out = {}
for n in (8192, 2048):
    for epi in ("store", "gelu") if n == 8192 else ("store",):
        for k in (512, 1024, 2048, 4096, 8192):
            x = torch.randn(M, k, device="cuda").bfloat16()
            w = (torch.randn(n, k, device="cuda") / k ** 0.5).bfloat16()
            bias = torch.randn(n, device="cuda").bfloat16()
            pre = torch.empty(M, n, device="cuda", dtype=torch.int16) if epi == "gelu" else None
            c = torch.empty(M, n, device="cuda", dtype=torch.bfloat16)
            t_l, t_t = [], []
            for _ in range(3):
                t_l.append(timeit(lambda: ops.gemm(x, w, bias=bias, epilogue=epi, aux0=pre, out=c)))
                t_t.append(timeit(lambda: torch.matmul(x, w.t())))
            fl = 2.0 * M * n * k
            r = {"ltx_us": round(min(t_l) * 1e3, 1), "torch_us": round(min(t_t) * 1e3, 1),
                 "ltx_tf": round(fl / min(t_l) / 1e9, 1), "torch_tf": round(fl / min(t_t) / 1e9, 1)}
            out[f"N{n}_{epi}_K{k}"] = r
            print(f"N={n} {epi:5s} K={k:5d}  ltx {r['ltx_us']:8.1f} us {r['ltx_tf']:7.1f} TF   "
                  f"torch {r['torch_us']:8.1f} us {r['torch_tf']:7.1f} TF", flush=True)
            del x, w, c, pre
print(json.dumps(out))
