"""Times the LoRA backward contractions at config A's size (M = 14336, K = N = 2048, r = 16)."""
import os, sys, json
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch
from ltx_amd import ops

M, K, r = 14336, 2048, 16
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
A = torch.randn(r, K, device="cuda", generator=g) / 45
Bm = torch.randn(K, r, device="cuda", generator=g) / 4
u = torch.randn(M, r, device="cuda", generator=g)
dA = torch.zeros(r, K, device="cuda")
dB = torch.zeros(K, r, device="cuda")


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

res = {"down_A_us": t(lambda: ops.lora_down(x, A)),
       "down_Bt_split_us": t(lambda: ops.lora_down(x, Bm, alpha=0.5, transposed=True, split=True)),
       "wgrad_B_us": t(lambda: ops.lora_wgrad(x, u, alpha=0.5, out=dB, accumulate=True)),
       "wgrad_A_us": t(lambda: ops.lora_wgrad(x, u, transpose_out=True, out=dA, accumulate=True))}
ref = (x.float() @ A.t())
res["down_rel"] = float((ops.lora_down(x, A) - ref).norm() / ref.norm())
xs = x[:256].contiguous()
us = u[:256].contiguous()
res["text_down_A_us"] = t(lambda: ops.lora_down(xs, A, split=True))
res["text_down_Bt_split_us"] = t(lambda: ops.lora_down(xs, Bm, alpha=0.5, transposed=True, split=True))
res["text_wgrad_B_us"] = t(lambda: ops.lora_wgrad(xs, us, alpha=0.5, out=dB, accumulate=True))
res["text_wgrad_A_us"] = t(lambda: ops.lora_wgrad(xs, us, transpose_out=True, out=dA, accumulate=True))
refs = xs.float() @ A.t()
res["text_down_rel"] = float((ops.lora_down(xs, A) - refs).norm() / refs.norm())
dB0 = torch.zeros_like(dB)
ops.lora_wgrad(xs, us, alpha=0.5, out=dB0, accumulate=True)
refw = 0.5 * xs.float().t() @ us
res["text_wgrad_rel"] = float((dB0 - refw).norm() / refw.norm())
print(json.dumps({k: round(v, 7) for k, v in res.items()}), flush=True)
# LDS-DMA row contraction on the bf16 pieces (ltx_lora_rows) vs the f32 kernel
pA = ops.lora_pieces(A)
pB = ops.lora_pieces(Bm, transposed=True)
r2 = {"rows_A_us": t(lambda: ops.lora_rows(x, pA, r)),
      "rows_Bt_split_us": t(lambda: ops.lora_rows(x, pB, r, alpha=0.5, split=True)),
      "pieces_us": t(lambda: ops.lora_pieces(A))}
o_new = ops.lora_rows(x, pA, r)
o_old = ops.lora_down(x, A)
r2["rows_rel_vs_f64"] = float((o_new.double() - x.double() @ A.double().t()).norm() / (x.double() @ A.double().t()).norm())
r2["down_rel_vs_f64"] = float((o_old.double() - x.double() @ A.double().t()).norm() / (x.double() @ A.double().t()).norm())
on, sn = ops.lora_rows(x, pB, r, alpha=0.5, split=True)
oo, so = ops.lora_down(x, Bm, alpha=0.5, transposed=True, split=True)
r2["rows_Bt_rel_vs_old"] = float((on - oo).norm() / oo.norm())
r2["split_equal_frac"] = float((sn == so).float().mean())
print(json.dumps({k: round(v, 9) for k, v in r2.items()}), flush=True)
