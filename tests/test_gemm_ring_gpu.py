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


def _both(fn, variant=20):
    _set(0)
    a = fn()
    torch.cuda.synchronize()
    _set(variant)
    try:
        b = fn()
        torch.cuda.synchronize()
    finally:
        _set(0)
    return a, b


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


@pytest.mark.parametrize("variant", [20, 21, 22], ids=["ring", "ring2", "ring3"])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm_ring_store_bitwise(M, N, K, variant):
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda", generator=g).bfloat16()
    assert ("gemm_ring2_kernel" if variant >= 21 else "gemm_ring_kernel") in _name(M, N, K, "store", variant)
    r0, r1 = _both(lambda: ops.gemm(a, w, bias=b), variant)
    assert torch.equal(r0, r1)
    if (M, N, K) == (5376, 2048, 2048):
        ref = (a.float() @ w.float().t() + b.float())
        err = (r1.float() - ref).abs().max().item()
        assert err <= 0.02 * ref.abs().max().item()


@pytest.mark.parametrize("variant", [20, 21, 22], ids=["ring", "ring2", "ring3"])
@pytest.mark.parametrize("M,N,K", [(14336, 2048, 2048), (14336, 8192, 2048), (7000, 6152, 384)])
def test_gemm_ring_epilogues_bitwise(M, N, K, variant):
    g = torch.Generator(device="cuda").manual_seed(7 + M + N + K)
    B = 8 if M % 8 == 0 else 1
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda", generator=g).bfloat16()
    R = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    gate = torch.randn(B, N, device="cuda", generator=g).bfloat16()
    pre0, pre1 = torch.empty(M, N, device="cuda").bfloat16(), torch.empty(M, N, device="cuda").bfloat16()
    # GELU with the pre-activation store (two separate aux buffers)
    _set(0)
    o0 = ops.gemm(a, w, bias=b, epilogue="gelu", aux0=pre0)
    _set(variant)
    o1 = ops.gemm(a, w, bias=b, epilogue="gelu", aux0=pre1)
    _set(0)
    torch.cuda.synchronize()
    assert torch.equal(o0, o1) and torch.equal(pre0, pre1)
    r0, r1 = _both(lambda: ops.gemm(a, w, bias=b, epilogue="gated_residual", aux0=R, aux1=gate,
                                    rows_per_batch=M // B), variant)
    assert torch.equal(r0, r1)
    r0, r1 = _both(lambda: ops.gemm(a, w, epilogue="gelu_bwd", aux0=R), variant)
    assert torch.equal(r0, r1)
    acc0, acc1 = R.clone(), R.clone()
    d0, d1 = torch.empty_like(R), torch.empty_like(R)
    _set(0)
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
        _set(0)
        s0 = ops.gemm(a, w, epilogue="store_rowdot", aux0=o, aux1=dl0, rank=64, rows_per_batch=M // B)
        _set(variant)
        s1 = ops.gemm(a, w, epilogue="store_rowdot", aux0=o, aux1=dl1, rank=64, rows_per_batch=M // B)
        _set(0)
        torch.cuda.synchronize()
        assert torch.equal(s0, s1) and torch.equal(dl0, dl1)


@pytest.mark.parametrize("variant", [20, 22], ids=["ring", "ring3"])
@pytest.mark.parametrize("M,N,K,K2", [(14336, 2048, 2048, 64), (14336, 2048, 2048, 128), (7000, 2056, 384, 64),
                                      (14336, 8192, 2048, 64)])
def test_gemm_ring_k_extension_bitwise(M, N, K, K2, variant):
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
        assert ("gemm_ring2_kernel" if variant >= 21 else "gemm_ring_kernel") in ops.gemm_kernel_name(M, N, K, K2, "store")
    finally:
        _set(0)
        ops._GEMM_NAMES.clear()
    r0, r1 = _both(lambda: ops.gemm(a, w, bias=b, ext=(a2, w2)), variant)
    assert torch.equal(r0, r1)
    R = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    c0, c1 = R.clone(), R.clone()
    _set(0)
    ops.gemm(a, w, epilogue="accum", aux0=c0, out=c0, ext=(a2, w2))
    _set(variant)
    ops.gemm(a, w, epilogue="accum", aux0=c1, out=c1, ext=(a2, w2))
    _set(0)
    torch.cuda.synchronize()
    assert torch.equal(c0, c1)
