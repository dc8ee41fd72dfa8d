"""Item-phase stamps of the persistent dK / dV kernel (attn_dkdv_w1p_kernel<1>, diag library built by
tools/build_diag.sh: LTX_HIP_LIB=libltxhip_diag.so, LTX_ATTN_DKDV_W1=22). The "itemstamps" body
(tools/gen_attn_bwd.py istamp) takes s_memtime at each phase boundary of every item and stores the
last item's: where the ~11 k cycles per item beyond the tile loop go. Medians over every wave of
config A's self-attention backward."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch
from ltx_amd import ops

os.environ["LTX_ATTN_DKDV_W1"] = "22"
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
nwg = 256
st = ws.view(torch.int64)[: nwg * 4 * 8].view(nwg * 4, 8).cpu().double()
ed = ws.view(torch.int64)[nwg * 4 * 8: nwg * 4 * 12].view(nwg * 4, 4).cpu().double()
# slots: 0 item entry (after the previous epilogue), 1 after the tiles-ready barrier, 2 before A(0),
# 3 before half 0, 6 loop start, 7 tail start, 4 before the epilogue, 5 after it
order = [(0, "item entry"), (1, "barrier"), (2, "setup done"), (3, "A(0) done"), (6, "half 0 done"),
         (7, "loop done"), (4, "tail done"), (5, "epilogue done")]
tot_item = st[:, 5] - st[:, 0]
for (a, na), (b, nb) in zip(order, order[1:]):
    dl = st[:, b] - st[:, a]
    print(f"{na:>13} -> {nb:<14} median {dl.median():8.0f}  p10 {dl.quantile(0.1):8.0f}  p90 {dl.quantile(0.9):8.0f} cycles")
loop = st[:, 7] - st[:, 6]
print(f"item total median {tot_item.median():.0f} cycles; loop {loop.median():.0f} over {N // 64 - 1} bodies "
      f"= {loop.median() / (N // 64 - 1):.0f} per body; outside the loop {(tot_item - loop).median():.0f}")
tot = ed[:, 2] - ed[:, 0]
clk = tot / ((ed[:, 3] - ed[:, 1]) * 10.0)
span = (ed[:, 3].max() - ed[:, 1].min()) / 100.0
print(f"wave total median {tot.median():.0f} cycles at {clk.median():.3f} GHz; launch span {span:.1f} us "
      f"(stamps build: an lgkmcnt(0) after each stamp)")
