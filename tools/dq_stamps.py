"""Phase stamps of attn_dq_w1_kernel (diag build: LTX_HIP_LIB=libltxhip_diag.so; LTX_ATTN_DQ_W1 = 12 as
built, 13 without the softmax VALU): s_memtime at one loop body (counter == STAMP_BODY), medians over
every wave of config A's self-attention backward."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch
from ltx_amd import ops

os.environ["LTX_ATTN_DQ_W1"] = sys.argv[1] if len(sys.argv) > 1 else "12"
B, N, H, d = 8, 1792, 32, 64
D = H * d
torch.manual_seed(0)
qkv = torch.randn(B * N, 3 * D, device="cuda").bfloat16()
q, k, v = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
o, lse = ops.attn_fwd(q, k, v, B, H, d, d ** -0.5)
do = torch.randn(B * N, D, device="cuda").bfloat16()
ws = ops._gemm_workspace(q.device)
for _ in range(3):
    ws.zero_()
    ops.attn_bwd(q, k, v, o, do, lse, B, H, d, d ** -0.5)
    torch.cuda.synchronize()
nwg = 7 * H * B
if os.environ['LTX_ATTN_DQ_W1'] == "22":  # the persistent kernel: one workgroup per CU, 7 items each
    nwg = 256
st = ws.view(torch.int64)[: nwg * 4 * 8].view(nwg * 4, 8).cpu().double()
names = ["top", "barrier", "half A", "half B"]
prev = st[:, 0]
for i in range(1, 4):
    dlt = st[:, i] - prev
    print(f"{names[i - 1]:>8} -> {names[i]:<8} median {dlt.median():8.0f}  p10 {dlt.quantile(0.1):8.0f}  p90 {dlt.quantile(0.9):8.0f} cycles")
    prev = st[:, i]
body = st[:, 3] - st[:, 0]
loop = st[:, 7] - st[:, 6]
print(f"body total median {body.median():.0f} cycles (2 halves, 48 MFMAs: floor 1536)")
print(f"whole loop median {loop.median():.0f} cycles over {N // 64 - 1} bodies = {loop.median() / (N // 64 - 1):.0f} per body")

# kernel entry / exit (s_memtime, s_memrealtime) of every wave: the loop's share of the wave's time
ed = ws.view(torch.int64)[nwg * 4 * 8: nwg * 4 * 12].view(nwg * 4, 4).cpu().double()
tot = ed[:, 2] - ed[:, 0]
clk = tot / ((ed[:, 3] - ed[:, 1]) * 10.0)  # cycles per ns
pro = st[:, 6] - ed[:, 0]
epi = ed[:, 2] - st[:, 7]
print(f"wave total median {tot.median():.0f} cycles at {clk.median():.3f} GHz: prologue {pro.median():.0f}, "
      f"loop {(st[:, 7] - st[:, 6]).median():.0f}, tail + epilogue {epi.median():.0f}")
span = (ed[:, 3].max() - ed[:, 1].min()) / 100.0
wall = (ed[:, 3] - ed[:, 1]) / 100.0
print(f"launch span {span:.1f} us; per-wave wall median {wall.median():.2f} us (x 7 rounds = {7 * wall.median():.1f} us)")
if nwg == 256:
    print(f"persistent: per item {tot.median() / 7:.0f} cycles = {wall.median() / 7:.2f} us (loop of the last item {(st[:, 7] - st[:, 6]).median():.0f})")
