"""hipBLASLt probe (stream-K grid, LTX_BLASLT_BIAS): times ltx_gemm_blaslt_bf16 (through ops.gemm's library route)
on the plain-store training shapes at M = 8 x 1792 tokens. The TENSILE_STREAMK_* settings are
read once per process, so run this once per setting, e.g.
    TENSILE_STREAMK_DYNAMIC_GRID=0 python tools/blaslt_grid.py tag
and compare the JSON lines (us per launch, PF/s)."""
import json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch
from ltx_amd import ops

M = 14336
# (name, N, K, bias): the library products of one LoRA-mode block
SHAPES = [("qkv", 6144, 2048, True), ("ff_down", 2048, 8192, True), ("ff_up_dgrad", 2048, 8192, False),
          ("out1_dgrad", 2048, 2048, False), ("qkv_dgrad", 2048, 6144, False),
          ("qkv_nobias", 6144, 2048, False), ("ff_down_nobias", 2048, 8192, False),
          ("qkv_kpad", 6144, 2048 + 64, False), ("ff_down_kpad", 2048, 8192 + 64, False)]


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "default"
    iters = 30
    row = {"tag": tag, "env": {k: v for k, v in os.environ.items() if k.startswith("TENSILE_")}}
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, n, k, has_bias in SHAPES:
        a = torch.randn(M, k, device="cuda", generator=g).bfloat16()
        w = (torch.randn(n, k, device="cuda", generator=g) / k ** 0.5).bfloat16()
        b = torch.randn(n, device="cuda", generator=g).bfloat16() if has_bias else None
        out = torch.empty(M, n, device="cuda", dtype=torch.bfloat16)
        ops.gemm(a, w, bias=b, out=out)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            ops.gemm(a, w, bias=b, out=out)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / iters * 1e3
        ref = (a.float() @ w.float().t() + (b.float() if b is not None else 0)).bfloat16().float()
        err = ((out.float() - ref).norm() / ref.norm()).item()
        row[name] = {"us": round(us, 1), "pf": round(2.0 * M * n * k / us / 1e9, 3), "rel_err": err}
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
