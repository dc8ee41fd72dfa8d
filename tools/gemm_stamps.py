"""Where does a large-tile GEMM launch spend its time? Runs the stamp-instrumented t-kernel
(ltx_gemm_set_variant 19 = 224-row tiles, 20 = 256-row tiles; diagnostic build only) and
reports, from s_memrealtime stamps (100 MHz) of every workgroup: the launch span, the phase
durations (prologue wait, main loop, epilogue image, epilogue stores), the gap between
consecutive workgroups on one CU, and the spread of main-loop time across XCDs.
Usage: python tools/gemm_stamps.py"""
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
lib = _lib.load()


def run(n, k, variant):
    x = torch.randn(M, k, device="cuda").bfloat16()
    w = (torch.randn(n, k, device="cuda") / k ** 0.5).bfloat16()
    c = torch.empty(M, n, device="cuda", dtype=torch.bfloat16)
    bmt = 224 if variant == 19 else 256
    tiles = ((M + bmt - 1) // bmt) * ((n + 255) // 256)
    stamps = torch.zeros(tiles * 8, dtype=torch.int64, device="cuda")
    lib.ltx_gemm_set_stamps(ctypes.c_void_p(stamps.data_ptr()))
    lib.ltx_gemm_set_variant(variant)
    for _ in range(10):
        ops.gemm(x, w, out=c)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    ops.gemm(x, w, out=c)
    ev1.record()
    torch.cuda.synchronize()
    lib.ltx_gemm_set_variant(0)
    ms = ev0.elapsed_time(ev1)
    s = stamps.view(tiles, 8).cpu().tolist()
    t0 = min(r[0] for r in s)
    us = lambda v: (v - t0) / 100.0  # noqa: E731  100 MHz ticks -> us
    span = (max(r[4] for r in s) - t0) / 100.0
    pro = [(r[1] - r[0]) / 100 for r in s]
    loop = [(r[2] - r[1]) / 100 for r in s]
    img = [(r[3] - r[2]) / 100 for r in s]
    sto = [(r[4] - r[3]) / 100 for r in s]
    by_cu = collections.defaultdict(list)
    by_xcc = collections.defaultdict(list)
    for r in s:
        by_cu[(r[6], (r[5] >> 8) & 0xFFF)].append(r)
        by_xcc[r[6]].append((r[2] - r[1]) / 100)
    gaps = []
    per_cu = []
    for cu, rs in by_cu.items():
        rs.sort(key=lambda r: r[0])
        per_cu.append(len(rs))
        for a, b in zip(rs, rs[1:]):
            gaps.append((b[0] - a[4]) / 100)
    starts = sorted(us(r[0]) for r in s)
    ends = sorted(us(r[4]) for r in s)
    fl = 2.0 * M * n * k
    print(f"N={n} K={k} v{variant} tiles={tiles} event {ms * 1e3:.1f} us ({fl / ms / 1e9:.0f} TF) "
          f"stamp span {span:.1f} us; CUs seen {len(by_cu)} (WGs/CU min {min(per_cu)} max {max(per_cu)})")
    q = lambda v: f"med {st.median(v):6.2f} min {min(v):6.2f} max {max(v):6.2f}"  # noqa: E731
    print(f"  prologue wait {q(pro)} | main loop {q(loop)} | epi image {q(img)} | epi stores {q(sto)}")
    if gaps:
        print(f"  gap between WGs on a CU: {q(gaps)} (n={len(gaps)})")
    print("  start of WG #0/256/512/...: " + " ".join(f"{starts[i]:.1f}" for i in range(0, tiles, 256)))
    print("  last end per 256-WG rank : " + " ".join(f"{ends[min(i + 255, tiles - 1)]:.1f}" for i in range(0, tiles, 256)))
    print("  main-loop median per XCC : " + " ".join(f"{x}:{st.median(v):.1f}" for x, v in sorted(by_xcc.items())))
    print(f"  sum of per-WG busy time / (CUs x span) = {sum(r[4] - r[0] for r in s) / 100 / (len(by_cu) * span):.3f}")


for n, k in ((8192, 2048), (2048, 2048), (6144, 2048), (2048, 8192)):
    for v in (19, 20):
        run(n, k, v)
