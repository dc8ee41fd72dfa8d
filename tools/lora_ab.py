"""Per-call time of the token-sized LoRA kernels at config A's adapter shape (M = 14336, K = N =
2048, r = 16), cycling over 6 distinct [M, 2048] operands (352 MB) so no call finds its input in
the 256 MB last-level cache -- the step's situation, where every adapter operand comes from HBM.
  forward:  lora_rows(x, A pieces, split)          -> u, su
  backward: lora_dy(dY, u, B^T pieces)             -> w, sw, dB
            lora_wgrad(x, w, transpose_out)        -> dA
Prints one JSON line (us per call, averaged over 60 calls each). Variants by env (LTX_*), one
process per variant (tools/ab_env.sh)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch
from ltx_amd import ops

M, K, r, NB = 14336, 2048, 16, 6
g = torch.Generator(device="cuda").manual_seed(0)
xs = [torch.randn(M, K, device="cuda", generator=g).bfloat16() for _ in range(NB)]
dys = [torch.randn(M, K, device="cuda", generator=g).bfloat16() for _ in range(NB)]
A = torch.randn(r, K, device="cuda", generator=g) / 45
Bm = torch.randn(K, r, device="cuda", generator=g) / 4
pA = ops.lora_pieces(A)
pB = ops.lora_pieces(Bm, transposed=True)
dA = torch.zeros(r, K, device="cuda")
dB = torch.zeros(K, r, device="cuda")
us = [ops.lora_rows(x, pA, r, split=True)[0] for x in xs]
ws = [ops.lora_dy(dy, u, pB, r, 0.5, dB)[0] for dy, u in zip(dys, us)]


def t(fn, it=60):
    for i in range(NB):
        fn(i)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(it):
        fn(i % NB)
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / it * 1e3, 2)


res = {
    "rows_split_us": t(lambda i: ops.lora_rows(xs[i], pA, r, split=True)),
    "dy_us": t(lambda i: ops.lora_dy(dys[i], us[i], pB, r, 0.5, dB)),
    "wgrad_dA_us": t(lambda i: ops.lora_wgrad(xs[i], ws[i], transpose_out=True, out=dA, accumulate=True)),
}
# accuracy against fp32 on the first operand set
x, dy, u, w = xs[0], dys[0], us[0], ws[0]
ref_u = x.float() @ A.t()
res["rows_rel"] = float((us[0] - ref_u).norm() / ref_u.norm())
ref_w = 0.5 * dy.float() @ Bm
res["dy_w_rel"] = float((w - ref_w).norm() / ref_w.norm())
d0 = ops.lora_wgrad(x, w, transpose_out=True)
ref_d = w.t() @ x.float()
res["wgrad_rel"] = float((d0 - ref_d).norm() / ref_d.norm())
res["env"] = {k: v for k, v in os.environ.items() if k.startswith("LTX_LORA")}
print(json.dumps(res), flush=True)
