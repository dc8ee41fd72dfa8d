"""The ring GEMM (gemm_ring.h: hand-scheduled K loop, 4 waves at one wave per SIMD) against the
large-tile kernel gemm_nt_kernel_t it replaces: every accumulator takes its K in the same 32-deep
steps in the same order and the epilogue is shared, so every output must be BITWISE equal, for each
fused epilogue of the training step, on the config-A shapes (M = 8 x 1792) and on ragged ones
(rows past M and columns past N clamped in the DMA, not stored). The default kernel is itself
checked against fp32 torch in test_kernels_gpu.py; one fp32 check here guards both."""
import pytest
import torch

from ltx_amd import _lib, ops

pytestmark = pytest.mark.gpu


def _set(v):
    _lib.load().ltx_gemm_set_variant(v)


REF = 15  # gemm_nt_kernel_t at the dispatcher's tile height


def _both(fn, variant=20):
    _set(REF)
    a = fn()
    torch.cuda.synchronize()
    _set(variant)
    try:
        b = fn()
        torch.cuda.synchronize()
    finally:
        _set(0)
    return a, b


def _same(a, b):
    """torch.equal, with the mismatch pattern in the failure message"""
    if torch.equal(a, b):
        return True
    d = (a != b)
    idx = d.nonzero()
    rows = idx[:, 0].unique()
    raise AssertionError(f"{int(d.sum())} of {d.numel()} differ; rows {rows[:8].tolist()}.. "
                         f"({rows.numel()} rows), cols {idx[:8, -1].tolist()}, max |diff| "
                         f"{float((a.float() - b.float()).abs().max())}")


def _name(M, N, K, epi, variant=20):
    _set(variant)
    ops._GEMM_NAMES.clear()  # the name cache does not key on the variant
    try:
        return ops.gemm_kernel_name(M, N, K, 0, epi)
    finally:
        _set(0)
        ops._GEMM_NAMES.clear()


SHAPES = [(14336, 2048, 2048), (14336, 6144, 2048), (14336, 2048, 8192), (14336, 8192, 2048),
          (14336, 2048, 128), (14336, 2048, 256), (7000, 6152, 384), (5376, 2048, 2048), (8192, 4096, 640)]


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm_ring_store_bitwise(M, N, K, variant=20):
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda", generator=g).bfloat16()
    name = _name(M, N, K, "store", variant)
    assert ("gemm_ring_kernel" in name) == (K % 128 == 0), name
    r0, r1 = _both(lambda: ops.gemm(a, w, bias=b), variant)
    assert _same(r0, r1)
    if (M, N, K) == (5376, 2048, 2048):
        ref = (a.float() @ w.float().t() + b.float())
        err = (r1.float() - ref).abs().max().item()
        assert err <= 0.02 * ref.abs().max().item()


# B = 7 (2048-row batches): 224-row tiles that straddle two batches (the per-row gate path; the
# config-A tiles each lie inside one batch and load the gate row once)
@pytest.mark.parametrize("M,N,K,B", [(14336, 2048, 2048, 8), (14336, 8192, 2048, 8), (7000, 6152, 384, 1),
                                     (14336, 2048, 2048, 7)])
def test_gemm_ring_epilogues_bitwise(M, N, K, B, variant=20):
    g = torch.Generator(device="cuda").manual_seed(7 + M + N + K)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda", generator=g).bfloat16()
    R = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    gate = torch.randn(B, N, device="cuda", generator=g).bfloat16()
    pre0 = torch.empty(M, N, device="cuda", dtype=torch.int16)
    pre1 = torch.empty(M, N, device="cuda", dtype=torch.int16)
    # GELU with the store of its derivative (int16 snorm; two separate aux buffers)
    _set(REF)
    o0 = ops.gemm(a, w, bias=b, epilogue="gelu", aux0=pre0)
    _set(variant)
    o1 = ops.gemm(a, w, bias=b, epilogue="gelu", aux0=pre1)
    _set(0)
    torch.cuda.synchronize()
    assert torch.equal(o0, o1) and torch.equal(pre0, pre1)
    r0, r1 = _both(lambda: ops.gemm(a, w, bias=b, epilogue="gated_residual", aux0=R, aux1=gate,
                                    rows_per_batch=M // B), variant)
    assert _same(r0, r1)
    r0, r1 = _both(lambda: ops.gemm(a, w, epilogue="gelu_bwd", aux0=pre0), variant)
    assert _same(r0, r1)
    acc0, acc1 = R.clone(), R.clone()
    d0, d1 = torch.empty_like(R), torch.empty_like(R)
    _set(REF)
    ops.gemm(a, w, epilogue="accum", aux0=acc0, out=acc0, aux1=gate, aux2=d0, rows_per_batch=M // B)
    _set(variant)
    ops.gemm(a, w, epilogue="accum", aux0=acc1, out=acc1, aux1=gate, aux2=d1, rows_per_batch=M // B)
    _set(0)
    torch.cuda.synchronize()
    assert torch.equal(acc0, acc1) and torch.equal(d0, d1)
    if N % 64 == 0 and M % B == 0:
        o = torch.randn(M, N, device="cuda", generator=g).bfloat16()
        dl0 = torch.empty(B, N // 64, M // B, device="cuda")
        dl1 = torch.empty_like(dl0)
        _set(REF)
        s0 = ops.gemm(a, w, epilogue="store_rowdot", aux0=o, aux1=dl0, rank=64, rows_per_batch=M // B)
        _set(variant)
        s1 = ops.gemm(a, w, epilogue="store_rowdot", aux0=o, aux1=dl1, rank=64, rows_per_batch=M // B)
        _set(0)
        torch.cuda.synchronize()
        assert torch.equal(s0, s1) and torch.equal(dl0, dl1)


@pytest.mark.parametrize("M,N,K,K2", [(14336, 2048, 2048, 64), (14336, 2048, 2048, 128), (7000, 2056, 384, 64),
                                      (14336, 8192, 2048, 64), (16384, 2048, 2048, 128)])
def test_gemm_ring_k_extension_bitwise(M, N, K, K2, variant=20):
    """The fused LoRA K-extension (attn2 q / out projections and their dgrads): the ring kernel runs
    the extension tiles after the main loop, in gemm_nt_kernel_t's order -- bitwise, for the plain
    store and the accumulate epilogue (<6>)."""
    g = torch.Generator(device="cuda").manual_seed(K2 + M)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    a2 = torch.randn(M, K2 + 8, device="cuda", generator=g).bfloat16()[:, :K2]  # strided view
    w2 = torch.randn(N, K2, device="cuda", generator=g).bfloat16()
    b = torch.randn(N, device="cuda", generator=g).bfloat16()
    _set(variant)
    ops._GEMM_NAMES.clear()
    try:
        name = ops.gemm_kernel_name(M, N, K, K2, "store")
        assert "gemm_ring_kernel<0, 0, " in name and name.endswith(f", {K2 // 64}>(ltx::GemmParams)"), name
    finally:
        _set(0)
        ops._GEMM_NAMES.clear()
    r0, r1 = _both(lambda: ops.gemm(a, w, bias=b, ext=(a2, w2)), variant)
    assert _same(r0, r1)
    R = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    c0, c1 = R.clone(), R.clone()
    _set(REF)
    ops.gemm(a, w, epilogue="accum", aux0=c0, out=c0, ext=(a2, w2))
    _set(variant)
    ops.gemm(a, w, epilogue="accum", aux0=c1, out=c1, ext=(a2, w2))
    _set(0)
    torch.cuda.synchronize()
    assert _same(c0, c1)
