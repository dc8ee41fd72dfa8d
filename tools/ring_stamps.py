"""Where does a ring GEMM launch spend its time? Loads the stamps build (libltxhip_stamps.so,
`make -C video-generation-for-human-avatars_amd/csrc stamps`: s_memrealtime at kernel entry, after
the K loop (+ extension), after the epilogue, from wave 0 of every workgroup) and reports per
shape: launch span, K loop / epilogue durations (median, p10, p90), the start skew of the tile
rounds and the per-XCD spread of the loop time.
Usage: LTX_HIP_LIB=.../libltxhip_stamps.so python tools/ring_stamps.py [variant]"""
import collections
import ctypes
import os
import statistics as st
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch  # noqa: E402
from ltx_amd import _lib, ops  # noqa: E402

M = 14336
VARIANT = int(sys.argv[1]) if len(sys.argv) > 1 else 20
lib = _lib.load()
lib.ltx_gemm_set_stamps.argtypes = [ctypes.c_void_p]
SHAPES = [("qkv", 6144, 2048, "store"), ("out1_gres", 2048, 2048, "gated_residual"),
          ("ff_up_gelu", 8192, 2048, "gelu"), ("ff_down_gres", 2048, 8192, "gated_residual"),
          ("ffdgrad_gelubwd", 8192, 2048, "gelu_bwd"), ("ff1_dgrad", 2048, 8192, "store"),
          ("dh1_accum_gate", 2048, 2048, "accum"), ("do_rowdot", 2048, 2048, "store_rowdot")]


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


for name, n, k, epi in SHAPES:
    x = torch.randn(M, k, device="cuda").bfloat16()
    w = (torch.randn(n, k, device="cuda") / k ** 0.5).bfloat16()
    bias = torch.randn(n, device="cuda").bfloat16()
    aux0 = aux1 = None
    if epi == "gelu":
        aux0 = torch.empty(M, n, device="cuda", dtype=torch.int16)
    aux2, rank = None, 0
    if epi in ("gated_residual", "gelu_bwd", "accum", "store_rowdot"):
        aux0 = torch.randn(M, n, device="cuda").bfloat16()
    if epi == "gelu_bwd":  # the GELU derivative (int16 snorm)
        aux0 = (aux0.float().clamp(-1, 1) * 16384).to(torch.int16)
    if epi in ("gated_residual", "accum"):
        aux1 = torch.randn(8, n, device="cuda").bfloat16()
    if epi == "accum":
        aux2 = torch.empty(M, n, device="cuda", dtype=torch.bfloat16)
    if epi == "store_rowdot":
        aux1 = torch.empty(8, 32, M // 8, device="cuda", dtype=torch.float32)
        rank = 64
    if epi in ("gelu_bwd", "accum", "store_rowdot"):
        bias = None
    c = torch.empty(M, n, device="cuda", dtype=torch.bfloat16)
    lib.ltx_gemm_set_variant(VARIANT)
    kern = ops.gemm_kernel_name(M, n, k, 0, epi, rank)
    bmt = 224 if ", 7" in kern else 256
    tiles = ((M + bmt - 1) // bmt) * ((n + 255) // 256)
    stamps = torch.zeros(tiles * 8, dtype=torch.int64, device="cuda")
    lib.ltx_gemm_set_stamps(ctypes.c_void_p(stamps.data_ptr()))
    kw = dict(bias=bias, epilogue=epi, aux0=aux0, aux1=aux1, rows_per_batch=1792 if aux1 is not None else 0)
    if aux2 is not None:
        kw["aux2"] = aux2
    if rank:
        kw["rank"] = rank
    for _ in range(10):
        ops.gemm(x, w, out=c, **kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ops.gemm(x, w, out=c, **kw)
    e1.record()
    torch.cuda.synchronize()
    lib.ltx_gemm_set_variant(0)
    ms = e0.elapsed_time(e1)
    s = stamps.view(tiles, 8).cpu().tolist()
    t0 = min(r[0] for r in s)
    span = (max(r[3] for r in s) - t0) / 100.0
    loop = [(r[1] - r[0]) / 100 for r in s]
    epil = [(r[3] - r[1]) / 100 for r in s]
    clk = [(r[4] - r[2]) / max(1, r[1] - r[0]) * 0.1 for r in s]  # GHz: cycles / (ticks of 10 ns)
    kt = k // 64
    starts = sorted((r[0] - t0) / 100 for r in s)
    by_xcc = collections.defaultdict(list)
    for r, l in zip(s, loop):
        by_xcc[r[6]].append(l)
    fl = 2.0 * M * n * k
    print(f"{name:16s} {kern[:40]:40s} event {ms*1e3:7.1f} us ({fl / ms / 1e9:6.0f} TF)  span {span:7.1f} us  tiles {tiles}")
    print(f"   loop   med {st.median(loop):6.1f}  p10 {pct(loop, .1):6.1f}  p90 {pct(loop, .9):6.1f} us  "
          f"(MFMA-bound ideal at 2.0 GHz: {k / 64 * 8 * (bmt // 32) * 16 * 2 / 2.0e3 / 1.0:.1f} us)")
    print(f"   epilog med {st.median(epil):6.1f}  p10 {pct(epil, .1):6.1f}  p90 {pct(epil, .9):6.1f} us")
    cyc = [(r[4] - r[2]) / kt for r in s]
    print(f"   loop clock med {st.median(clk):.3f} GHz; cycles per 64-deep K-tile med {st.median(cyc):.0f} "
          f"(MFMA floor {8 * (bmt // 32) * 2 * 16})")
    nr = min(256, tiles)
    print(f"   starts: first round {starts[0]:.1f}..{starts[nr - 1]:.1f} us, later rounds from "
          f"{starts[nr] if tiles > nr else float('nan'):.1f} us")
    print("   loop by XCC: " + " ".join(f"{x}:{st.median(v):.1f}" for x, v in sorted(by_xcc.items())))
