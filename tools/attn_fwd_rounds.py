"""Self-attention forward time against the batch (H = 32, N = 1792, d = 64): whether the launch's
workgroup rounds (1792 workgroups at B = 8 = 3.5 rounds of 512 resident slots) cost a tail.
Prints us per launch and us per batch element for each B."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch  # noqa: E402
from ltx_amd import _lib, ops  # noqa: E402

H, N, d = 32, 1792, 64
_lib.ensure_device("cuda")
g = torch.Generator(device="cpu").manual_seed(0)


def timeit(fn, iters=30):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


for B in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4,6,7,8,9,10,12,16").split(",")]:
    q, k, v = (torch.randn(B * N, H * d, generator=g).to("cuda", torch.bfloat16) for _ in range(3))
    t = timeit(lambda: ops.attn_fwd(q, k, v, B, H, d, d ** -0.5))
    print(f"B={B:2d} workgroups={B * H * 7:5d} rounds={B * H * 7 / 512:5.2f}  {t:7.1f} us  {t / B:6.1f} us/batch",
          flush=True)
    del q, k, v
