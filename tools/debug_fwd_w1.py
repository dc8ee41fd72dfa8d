"""w1 forward vs the pipelined kernel on ramped logits: where do O / lse differ (debug aid)"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch
from ltx_amd import ops

B, H, N, d, jump = 1, 1, int(sys.argv[1]) if len(sys.argv) > 1 else 512, 64, int(sys.argv[2]) if len(sys.argv) > 2 else 1
gen = torch.Generator(device="cpu").manual_seed(64)
q = torch.randn(B, N, H, d, generator=gen) * 0.5
k = torch.randn(B, N, H, d, generator=gen) * 0.5
v = torch.randn(B * N, H * d, generator=gen).cuda().bfloat16()
q[..., 0] = torch.where(torch.rand(B, N, H, generator=gen) < 0.7, 4.0, -4.0)
t = torch.arange(N) // 64
k[..., 0] = (-60.0 + 24.0 * (t // jump).float() + torch.rand(N, generator=gen) * 3.0).clamp(max=60.0).view(1, N, 1)
q = q.reshape(B * N, H * d).cuda().bfloat16()
k = k.reshape(B * N, H * d).cuda().bfloat16()
res = {}
for w1 in ("0", "1"):
    os.environ["LTX_ATTN_FWD_W1"] = w1
    res[w1] = ops.attn_fwd(q, k, v, B, H, d, d ** -0.5)
torch.cuda.synchronize()
o0, l0 = res["0"]
o1, l1 = res["1"]
do = (o0.float() - o1.float()).abs().view(B, N, H, d)
dl = (l0 - l1).abs().view(B, H, N)
rows = (do.amax(-1) > 0).nonzero()
print("O rows differing:", rows.shape[0], "of", B * N * H, " max|dO|", float(do.max()))
print("lse differing:", int((dl > 0).sum()), " max|dlse|", float(dl.max()))
r = (do.amax(-1) > 0).view(-1).nonzero().view(-1)
print("first rows:", r[:40].tolist())
qi = r[:8].tolist()
for i in qi:
    print(i, "lse", float(l0.view(-1)[i]), float(l1.view(-1)[i]), "O[:4]", o0.view(-1, d)[i, :4].tolist(), o1.view(-1, d)[i, :4].tolist())
