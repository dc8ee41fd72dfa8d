"""Phase stamps of attn_fwd_w1_kernel (a stamps body: tools/build_fwd_variant.sh stamps[,novalu],
LTX_HIP_LIB=.../libltxhip_fv.so): s_memtime at the top of loop iteration SITER == 5 and after its two
units, plus loop start / end; medians over every wave of config A's self-attention forward."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch
from ltx_amd import ops

os.environ["LTX_ATTN_FWD_W1"] = "12"
B, N, H, d = 8, 1792, 32, 64
D = H * d
torch.manual_seed(0)
q = torch.randn(B * N, D, device="cuda").bfloat16()
k = torch.randn(B * N, D, device="cuda").bfloat16()
v = torch.randn(B * N, D, device="cuda").bfloat16()
ws = ops._gemm_workspace(q.device)
for _ in range(3):
    ws.zero_()
    ops.attn_fwd(q, k, v, B, H, d, d ** -0.5)
    torch.cuda.synchronize()
nwg = 7 * H * B
st = ws.view(torch.int64)[: nwg * 4 * 8].view(nwg * 4, 8).cpu().double()
u0 = st[:, 1] - st[:, 0]
u1 = st[:, 2] - st[:, 1]
loop = st[:, 7] - st[:, 6]
print(f"unit (even) median {u0.median():.0f} p10 {u0.quantile(.1):.0f} p90 {u0.quantile(.9):.0f}; unit (odd) median "
      f"{u1.median():.0f} cycles (32 MFMAs: floor 1024)")
print(f"whole loop median {loop.median():.0f} cycles over {(N // 64 - 2) // 2} iterations = "
      f"{loop.median() / ((N // 64 - 2) // 2) / 2:.0f} per unit")
