"""Per-kernel parity on the MI355X: every C-ABI entry point against a torch reference of the same
op (the oracle's eager bf16 op sequence where rounding points matter, an fp32 torch evaluation
for the MFMA contractions). Tolerances are written next to each check:
  * integer / index / permutation work: bit exact;
  * elementwise ops that mirror eager bf16 rounding: <= 1 bf16 ulp on a tiny fraction of entries;
  * MFMA contractions (f32 accumulate, bf16 out): rel-Frobenius <= 1e-2 vs the fp32 evaluation.
"""
import math
import os

import pytest
import torch
import torch.nn.functional as F

import ltx_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from ltx_amd import _lib as L
    L.ensure_device()
    return L


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


def ulps_bad(a, b, max_ulp=1):
    """fraction of bf16 entries that differ by more than max_ulp ulps"""
    ai = a.contiguous().view(torch.int16).to(torch.int32)
    bi = b.contiguous().view(torch.int16).to(torch.int32)
    return float(((ai - bi).abs() > max_ulp).float().mean())


def g(*shape, dtype=torch.bfloat16, scale=1.0, seed=0):
    gen = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=gen) * scale).to(dtype).to(DEV)


# ------------------------------------------------------------------------------------------ GEMM
@pytest.mark.parametrize("M,N,K", [(256, 128, 64), (300, 136, 128), (1024, 2048, 2048), (8, 768, 256),
                                   (256, 2048, 2048), (200, 1000, 4096),  # split-K grids
                                   (14336 // 7, 6144, 2048), (4000, 4104, 192), (14336, 2048, 8192)])
def test_gemm_store(M, N, K):
    from ltx_amd import ops
    a, w, b = g(M, K, seed=1), g(N, K, seed=2, scale=K ** -0.5), g(N, seed=3)
    out = ops.gemm(a, w, bias=b)
    ref = a.float() @ w.float().t() + b.float()
    assert rel(out, ref) < 1e-2
    # bf16-rounded result must be within 1 ulp of the fp32 result rounded once
    assert ulps_bad(out, ref.to(torch.bfloat16), 2) < 1e-3


def test_gemm_strided_views_and_no_bias():
    from ltx_amd import ops
    M, K, N = 384, 256, 256
    big = g(M, 3 * K, seed=4)
    a = big[:, K:2 * K]  # row stride 3K
    w = g(N, K, seed=5, scale=K ** -0.5)
    outbuf = torch.zeros(M, 2 * N, dtype=torch.bfloat16, device=DEV)
    ops.gemm(a, w, out=outbuf[:, N:])
    ref = a.float() @ w.float().t()
    assert rel(outbuf[:, N:], ref) < 1e-2
    assert float(outbuf[:, :N].abs().max()) == 0.0


@pytest.mark.parametrize("M,N,K", [(512, 256, 256), (256, 512, 2048),  # one pass / split-K
                                   (5376, 2048, 512)])  # 192 224-row tiles: large tile under one round
def test_gemm_epilogues(M, N, K):
    from ltx_amd import ops
    r, B = 16, 4
    a, w, b = g(M, K, seed=6), g(N, K, seed=7, scale=K ** -0.5), g(N, seed=8)
    y = (a.float() @ w.float().t() + b.float()).to(torch.bfloat16)
    # GELU + the backward's factor gelu_tanh'(y) (int16 snorm of d / 2): against ATen at the build's own bf16
    # y (recovered from the plain store; y itself differs from the fp32-accumulated reference by ulps)
    pre = torch.empty(M, N, dtype=torch.int16, device=DEV)
    out = ops.gemm(a, w, bias=b, epilogue="gelu", aux0=pre)
    yb = ops.gemm(a, w, bias=b)
    assert ulps_bad(yb, y, 2) < 1e-3
    ref = F.gelu(yb.float(), approximate="tanh").to(torch.bfloat16)
    assert ulps_bad(out, ref, 1) < 1e-3
    dq = ops.gelu_grad_q(yb)
    assert int((pre.int() - dq.int()).abs().max()) <= 1  # rint(32767 d / 2) up to the f32 rounding of d
    assert float((pre.float() / ops.GELU_Q - torch.ops.aten.gelu_backward(
        torch.ones_like(yb, dtype=torch.float32), yb.float(), approximate="tanh")).abs().max()) < 2 ** -14
    # gated residual
    R = g(M, N, seed=9)
    gate = g(B, N, seed=10)
    out = ops.gemm(a, w, bias=b, epilogue="gated_residual", aux0=R, aux1=gate, rows_per_batch=M // B)
    ybf = y
    ref = R + gate.repeat_interleave(M // B, 0) * ybf
    assert rel(out, ref.float()) < 1e-2
    # LoRA (+ residual)
    u = torch.randn(M, r, device=DEV)
    lb = torch.randn(N, r, device=DEV) * 0.1
    out = ops.gemm(a, w, bias=b, epilogue="lora", aux1=u, aux2=lb, alpha=0.5, rank=r)
    ref = (y.float() + 0.5 * (u @ lb.t())).to(torch.bfloat16)
    assert ulps_bad(out, ref, 2) < 2e-3
    out = ops.gemm(a, w, bias=b, epilogue="lora_residual", aux0=R, aux1=u, aux2=lb, alpha=0.5, rank=r)
    assert rel(out, R.float() + ref.float()) < 1e-2
    # GELU backward: dF = bf16((bf16(acc) * q) * 2 / 32767), q the int16 factor the forward epilogue
    # keeps (acc * q is exact in f32); end to end against ATen's gelu_backward at F
    Fpre = g(M, N, seed=11)
    q = ops.gelu_grad_q(Fpre)
    out = ops.gemm(a, w, epilogue="gelu_bwd", aux0=q)
    acc = (a.float() @ w.float().t()).to(torch.bfloat16).float()
    accb = ops.gemm(a, w).float()  # the build's own bf16(acc)
    assert torch.equal(out, ((accb * q.float()) * (2.0 / 32767.0)).to(torch.bfloat16))
    ref = torch.ops.aten.gelu_backward(acc, Fpre.float(), approximate="tanh")
    assert rel(out, ref) < 1e-2
    # accumulate (in place on R)
    R2 = R.clone()
    ops.gemm(a, w, epilogue="accum", aux0=R2, out=R2)
    assert rel(R2, R.float() + acc) < 1e-2
    # LoRA dgrad accumulate: [R +] acc + alpha * Wd . A
    Wd = torch.randn(M, r, device=DEV)
    A = torch.randn(r, N, device=DEV) * 0.1
    out = ops.gemm(a, w, epilogue="lora_dgrad_accum", aux0=R, aux1=Wd, aux2=A, alpha=1.0, rank=r)
    assert rel(out, R.float() + acc + (Wd @ A).to(torch.bfloat16).float()) < 1e-2


def test_gelu_derivative_tail():
    """The FF GELU pair's stored derivative in the tail (VERDICT r05 #5c): pre-activations
    y in [-8, -2] made exact by a one-hot GEMM (y = w[n, m % K], bias 0), the FF-up epilogue's int16
    code, then the FF-dgrad epilogue with dY = 1 exactly, against ATen's gelu_backward(1, y) (the
    reference's factor, computed in f32 from the bf16 pre-activation).

    The code is rint(32767 gelu'(y) / 2): absolute error <= 1/32767 in gelu' plus bf16's rounding of
    the product. So the relative bound 2^-8 holds where |gelu'| >= 2^-6 (y >~ -2.9) and below that the
    error is absolute, <= 2^-14 (gelu'(-3) = -1.2e-2, gelu'(-4) = -3.3e-4, gelu'(-6) = -6e-10): those
    factors are under the bf16 resolution of the dF tensor's own bulk (|gelu'| up to 1.13), which is
    the tolerance the 28-layer loss curve and the grad tests check end to end. INTEGRATION.md
    (parity notes) records the deviation."""
    from ltx_amd import ops
    M, N, K = 2048, 2048, 128
    a = torch.zeros(M, K, device=DEV, dtype=torch.bfloat16)
    a[torch.arange(M), torch.arange(M) % K] = 1.0
    gen = torch.Generator(device="cpu").manual_seed(77)
    w = (torch.rand(N, K, generator=gen) * -6.0 - 2.0).to(torch.bfloat16).to(DEV)  # [-8, -2]
    y = w.t()[torch.arange(M) % K]  # [M, N]: the exact pre-activations
    assert torch.equal(ops.gemm(a, w), y)
    pre = torch.empty(M, N, dtype=torch.int16, device=DEV)
    ops.gemm(a, w, bias=torch.zeros(N, device=DEV, dtype=torch.bfloat16), epilogue="gelu", aux0=pre)
    ones = torch.ones(N, K, device=DEV, dtype=torch.bfloat16)
    dF = ops.gemm(a, ones, epilogue="gelu_bwd", aux0=pre).double()
    ref = torch.ops.aten.gelu_backward(torch.ones_like(y, dtype=torch.float32), y.float(),
                                       approximate="tanh").double()
    err = (dF - ref).abs()
    big = ref.abs() >= 2 ** -6
    assert int(big.sum()) > 1000
    worst_rel = float((err[big] / ref.abs()[big]).max())
    assert worst_rel <= 2 ** -8, worst_rel
    assert bool((err <= 2 ** -8 * ref.abs() + 2 ** -14).all()), float((err - 2 ** -8 * ref.abs()).max())


@pytest.mark.parametrize("M,N,K,ext", [(14336, 2048, 2048, True),   # large tile + LoRA ext (dh1)
                                       (14336, 2048, 2048, False),
                                       (512, 256, 256, False),       # 128x128, one pass
                                       (256, 2048, 8192, True)])     # 128x128, split-K + ext
def test_gemm_accum_gated_copy(M, N, K, ext):
    """LTX_EPI_ACCUM with a gate (aux1) and aux2: C is bitwise the plain accumulate and aux2 is
    bitwise gate_mul(C, gate) (the backward's d_y1 = bf16(dh1 * g_msa) from dh1's own epilogue)."""
    from ltx_amd import ops
    B = 8
    a, w = g(M, K, seed=61), g(N, K, seed=62, scale=K ** -0.5)
    R = g(M, N, seed=63)
    mods = g(B, 6, N, seed=64)  # the gate is a [B, N] row view of the modulation tensor
    gate = mods[:, 2]
    kw = {}
    if ext:
        K2 = 64
        kw["ext"] = (g(M, K2, seed=65), g(N, K2, seed=66, scale=0.1))
    c0 = ops.gemm(a, w, epilogue="accum", aux0=R, **kw)
    d = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    c1 = ops.gemm(a, w, epilogue="accum", aux0=R, aux1=gate, aux2=d, rows_per_batch=M // B, **kw)
    assert torch.equal(c1, c0)
    assert torch.equal(d, ops.gate_mul(c0, gate, M // B))


@pytest.mark.parametrize("M,N,K,hd,ext", [(14336, 2048, 2048, 64, False),  # large tile (224 rows)
                                          (512, 256, 256, 64, False),     # 128x128, one pass
                                          (256, 2048, 8192, 64, True),    # 128x128, split-K + LoRA ext
                                          (600, 128, 128, 32, False)])    # head dim 32, ragged M
def test_gemm_store_rowdot(M, N, K, hd, ext):
    """LTX_EPI_STORE_ROWDOT: the dO GEMM also writes the attention backward's delta
    rowsum(dO*O) per head (f32 [B, H, rows]); C is bitwise the plain store."""
    from ltx_amd import ops
    B = 2 if M % 2 == 0 else 1
    a, w = g(M, K, seed=61), g(N, K, seed=62, scale=K ** -0.5)
    o = g(M, N, seed=63)
    kw = {}
    if ext:
        kw["ext"] = (g(M, 64, seed=64), g(N, 64, seed=65, scale=0.1))
    ref = ops.gemm(a, w, **kw)
    delta = torch.full((B, N // hd, M // B), float("nan"), device=DEV)
    out = ops.gemm(a, w, epilogue="store_rowdot", aux0=o, aux1=delta, rank=hd, rows_per_batch=M // B, **kw)
    assert torch.equal(out, ref)
    want = (out.float() * o.float()).view(B, M // B, N // hd, hd).sum(-1).permute(0, 2, 1)
    assert torch.isfinite(delta).all()
    assert (delta - want).abs().max().item() <= 1e-4 * want.abs().max().item() + 1e-5


# ------------------------------------------------------------------------------------- attention
def _sdpa_ref(q, k, v, B, H, d, bias=None, dtype=torch.float32):
    Nq, Nk = q.shape[0] // B, k.shape[0] // B
    qh = q.to(dtype).view(B, Nq, H, d).transpose(1, 2)
    kh = k.to(dtype).view(B, Nk, H, d).transpose(1, 2)
    vh = v.to(dtype).view(B, Nk, H, d).transpose(1, 2)
    mask = None if bias is None else bias.view(B, 1, 1, Nk).to(dtype)
    o = F.scaled_dot_product_attention(qh, kh, vh, attn_mask=mask)
    return o.transpose(1, 2).reshape(B * Nq, H * d)


@pytest.mark.parametrize("B,H,Nq,Nk,d,masked", [(2, 4, 128, 128, 64, False), (1, 3, 100, 77, 64, True),
                                                 (2, 4, 64, 4, 32, True), (2, 2, 256, 256, 32, False),
                                                 (1, 32, 1792, 256, 64, True), (2, 2, 640, 300, 64, False),
                                                 (1, 2, 200, 520, 64, True),
                                                 # split backward without key bias (the pipelined dQ and
                                                 # dK/dV kernels): ragged queries, one and several key tiles
                                                 (2, 3, 1000, 768, 64, False), (1, 2, 70, 320, 64, False),
                                                 (1, 2, 320, 1792, 64, False),
                                                 (1, 2, 50, 512, 64, False)])  # one ragged query tile
def test_attention_fwd_bwd(B, H, Nq, Nk, d, masked):
    from ltx_amd import ops
    scale = d ** -0.5
    q = g(B * Nq, H * d, seed=1)
    k = g(B * Nk, H * d, seed=2)
    v = g(B * Nk, H * d, seed=3)
    bias = None
    if masked:
        keep = torch.arange(Nk, device=DEV)[None, :] < (Nk - 3 - torch.arange(B, device=DEV)[:, None]).clamp(min=2)
        bias = ((1 - keep.to(torch.bfloat16)) * -10000.0).float()
    o, lse = ops.attn_fwd(q, k, v, B, H, d, scale, key_bias=bias)
    ref = _sdpa_ref(q, k, v, B, H, d, bias)
    # SURVEY 8(c)(4) noise criterion against fp32: within 1.25x torch's own bf16 SDPA error (+1e-3)
    ref16 = _sdpa_ref(q, k, v, B, H, d, bias, dtype=torch.bfloat16)
    assert rel(o, ref) <= 1.25 * rel(ref16, ref) + 1e-3, (rel(o, ref), rel(ref16, ref))
    # lse (log2 units) vs logsumexp of the scaled scores
    qh = q.float().view(B, Nq, H, d).transpose(1, 2)
    kh = k.float().view(B, Nk, H, d).transpose(1, 2)
    sc = qh @ kh.transpose(-1, -2) * scale
    if bias is not None:
        sc = sc + bias.view(B, 1, 1, Nk)
    lse_ref = torch.logsumexp(sc, -1) * (1 / math.log(2))
    assert float((lse - lse_ref).abs().max()) < 1e-2
    # backward vs fp32 autograd
    do = g(B * Nq, H * d, seed=4)
    qf, kf, vf = (t.float().clone().requires_grad_(True) for t in (q, k, v))
    _sdpa_ref(qf, kf, vf, B, H, d, bias).backward(do.float())
    dq, dk, dv = ops.attn_bwd(q, k, v, o, do, lse, B, H, d, scale, key_bias=bias)
    qh, kh, vh = (t.clone().requires_grad_(True) for t in (q, k, v))  # torch's bf16 SDPA backward
    _sdpa_ref(qh, kh, vh, B, H, d, bias, dtype=torch.bfloat16).backward(do)
    for ours, r32, r16 in ((dq, qf.grad, qh.grad), (dk, kf.grad, kh.grad), (dv, vf.grad, vh.grad)):
        assert rel(ours, r32) <= 1.25 * rel(r16, r32) + 1e-3, (rel(ours, r32), rel(r16, r32))
    dq32, _, _ = ops.attn_bwd(q, k, v, o, do, lse, B, H, d, scale, key_bias=bias, dq_f32=True)
    assert rel(dq32, qf.grad) <= 1.25 * rel(qh.grad, qf.grad) + 1e-3


def _cross_bias(Nk, Bk, valid):
    """Caption-style key bias bf16(-10000) on padded keys: `valid` None -> Nk - 5 - 3b keys of batch
    b kept; an int -> the first `valid` keys (the bench's prompt keeps 16 of 256)."""
    if valid is None:
        keep = torch.arange(Nk, device=DEV)[None, :] < (Nk - 5 - 3 * torch.arange(Bk, device=DEV)[:, None])
    else:
        keep = (torch.arange(Nk, device=DEV)[None, :] < valid).expand(Bk, Nk)
    return ((1 - keep.to(torch.bfloat16)) * -10000.0).float().contiguous()


@pytest.mark.parametrize("B,H,Nq,Nk,masked,shared,valid", [
    (2, 4, 1792, 256, False, False, None),  # no key bias
    (8, 4, 1792, 256, True, True, None),    # shared prompt, bias
    (8, 32, 1792, 256, True, True, 16),     # the bench's attn2: config A, 16 valid keys, shared
    (8, 4, 1792, 128, True, True, None),    # 128 keys: QS
    (1, 2, 300, 200, True, False, None),    # ragged both
    (2, 2, 64, 33, False, False, None),     # < 2 waves
    (1, 32, 7488, 256, True, False, None)])  # config X, B=1: query split
def test_attention_bwd_one_pass(B, H, Nq, Nk, masked, shared, valid, monkeypatch):
    """Nk <= 256 runs the one-pass backward (attn_bwd1_kernel: S/dP once, dQ from the dS image);
    LTX_ATTN_BWD1=0 forces the split dQ + dK/dV kernels. SURVEY 8(c)(4) noise criterion for dQ,
    dK and dV of both paths against fp32 autograd: rel-Frobenius within 1.25x torch's own bf16
    SDPA backward error (+1e-3); the one-pass error also within 1.25x the split path's (+1e-3)."""
    from ltx_amd import ops
    d = 64
    scale = d ** -0.5
    Bk = 1 if shared else B
    q = g(B * Nq, H * d, seed=11)
    k = g(Bk * Nk, H * d, seed=12)
    v = g(Bk * Nk, H * d, seed=13)
    do = g(B * Nq, H * d, seed=14)
    bias = _cross_bias(Nk, Bk, valid) if masked else None
    o, lse = ops.attn_fwd(q, k, v, B, H, d, scale, key_bias=bias, kv_shared=shared)
    kx = k.repeat(B, 1) if shared else k
    vx = v.repeat(B, 1) if shared else v
    bx = (bias.repeat(B, 1) if shared else bias) if bias is not None else None
    qf, kf, vf = (t.float().clone().requires_grad_(True) for t in (q, kx, vx))
    _sdpa_ref(qf, kf, vf, B, H, d, bx).backward(do.float())
    qh, kh, vh = (t.clone().requires_grad_(True) for t in (q, kx, vx))  # torch's bf16 SDPA backward
    _sdpa_ref(qh, kh, vh, B, H, d, bx, dtype=torch.bfloat16).backward(do)

    def batch_summed(t):  # shared keys: the per-batch rows of one key summed, then re-expanded
        return t.float().view(B, Nk, H * d).sum(0).repeat(B, 1) if shared else t
    refs32 = (qf.grad, batch_summed(kf.grad), batch_summed(vf.grad))
    refs16 = (qh.grad, batch_summed(kh.grad), batch_summed(vh.grad))
    e16 = tuple(rel(a, b_) for a, b_ in zip(refs16, refs32))
    errs = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("LTX_ATTN_BWD1", mode)
        for f32 in (False, True):
            dq, dk, dv = ops.attn_bwd(q, k, v, o, do, lse, B, H, d, scale, key_bias=bias, dq_f32=f32,
                                      kv_shared=shared)
            errs[mode, f32] = tuple(rel(a, b_) for a, b_ in zip((dq, batch_summed(dk), batch_summed(dv)),
                                                                refs32))
    for f32 in (False, True):
        for e1, e0, er in zip(errs["1", f32], errs["0", f32], e16):
            assert e1 <= 1.25 * er + 1e-3 and e0 <= 1.25 * er + 1e-3, (errs, e16)
            assert e1 <= 1.25 * e0 + 1e-3, (errs, e16)
    if H * B < 128 and (Nq + 63) // 64 >= 4:  # the one-pass kernel split over the queries
        monkeypatch.setenv("LTX_ATTN_BWD1", "1")
        ops._gemm_workspace(q.device)  # its dK / dV partials live in the stream's workspace
        outs = {}
        for qsplit in ("1", "0"):
            monkeypatch.setenv("LTX_ATTN_QSPLIT", qsplit)
            outs[qsplit] = ops.attn_bwd(q, k, v, o, do, lse, B, H, d, scale, key_bias=bias, kv_shared=shared)
        assert torch.equal(outs["1"][0], outs["0"][0])  # dQ: per query tile, unaffected
        for a, b_ in zip(outs["1"][1:], outs["0"][1:]):  # dK / dV: f32 partials summed in order
            assert rel(a, b_) < 1e-3
    if masked:  # every unmasked key in one 32-key block: per-wave sub-tiles (bwd1_few_keys) against
        # the 8 x 32-key schedule: dQ bitwise, dK / dV to the order of the 8 waves' partial sums
        monkeypatch.setenv("LTX_ATTN_BWD1", "1")
        outs = {}
        for few in ("1", "0"):
            monkeypatch.setenv("LTX_ATTN_BWD1_FEW", few)
            outs[few] = ops.attn_bwd(q, k, v, o, do, lse, B, H, d, scale, key_bias=bias, kv_shared=shared)
        assert torch.equal(outs["1"][0], outs["0"][0])
        for a, b_, r32, er in zip(outs["1"][1:], outs["0"][1:], refs32[1:], e16[1:]):
            assert rel(a, b_) < 1e-2
            assert rel(batch_summed(a), r32) <= 1.25 * er + 1e-3, (rel(batch_summed(a), r32), er)
        monkeypatch.delenv("LTX_ATTN_BWD1_FEW")
    if Nk <= 128:  # the query-split one-pass kernel (QS) against the 8 x 32-key one: dQ bitwise
        monkeypatch.setenv("LTX_ATTN_BWD1", "1")
        outs = {}
        for qs in ("1", "0"):
            monkeypatch.setenv("LTX_ATTN_BWD1_QS", qs)
            outs[qs] = ops.attn_bwd(q, k, v, o, do, lse, B, H, d, scale, key_bias=bias,
                                    kv_shared=shared)
        assert torch.equal(outs["1"][0], outs["0"][0])
        for a, r32, er in zip(outs["1"][1:], refs32[1:], e16[1:]):  # QS dK / dV: noise criterion
            assert rel(batch_summed(a), r32) <= 1.25 * er + 1e-3, (rel(batch_summed(a), r32), er)


@pytest.mark.parametrize("B,H,Nq,Nk,masked,shared,valid", [(2, 4, 1792, 256, False, False, None),
                                                            (8, 4, 1792, 256, True, True, None),
                                                            (8, 32, 1792, 256, True, True, 16),  # bench attn2
                                                            (1, 2, 300, 200, True, False, None),
                                                            (2, 2, 40, 64, False, False, None),
                                                            (1, 32, 7488, 256, True, False, None)])  # 8 WGs/head
def test_attention_fwd_one_pass(B, H, Nq, Nk, masked, shared, valid, monkeypatch):
    """Nk <= 256 runs attn_fwd1_kernel (K/V staged once per (batch, head)); its per-slice
    arithmetic is the tiled kernel's, so O and lse are bitwise those of LTX_ATTN_FWD1=0; O against
    fp32 SDPA by the SURVEY 8(c)(4) noise criterion (within 1.25x torch's bf16 SDPA error + 1e-3)."""
    from ltx_amd import ops
    d = 64
    Bk = 1 if shared else B
    q = g(B * Nq, H * d, seed=21)
    k = g(Bk * Nk, H * d, seed=22)
    v = g(Bk * Nk, H * d, seed=23)
    bias = _cross_bias(Nk, Bk, valid) if masked else None
    monkeypatch.setenv("LTX_ATTN_FWD1", "1")
    o1, l1 = ops.attn_fwd(q, k, v, B, H, d, d ** -0.5, key_bias=bias, kv_shared=shared)
    monkeypatch.setenv("LTX_ATTN_FWD1_ROWS", "0")  # O in 32-B pieces instead of LDS-staged rows
    o2, l2 = ops.attn_fwd(q, k, v, B, H, d, d ** -0.5, key_bias=bias, kv_shared=shared)
    monkeypatch.delenv("LTX_ATTN_FWD1_ROWS")
    assert torch.equal(o1, o2) and torch.equal(l1, l2)
    monkeypatch.setenv("LTX_ATTN_FWD1", "0")
    monkeypatch.setenv("LTX_ATTN_FWD_PIPE", "0")  # the tiled kernel whose arithmetic fwd1 mirrors
    o0, l0 = ops.attn_fwd(q, k, v, B, H, d, d ** -0.5, key_bias=bias, kv_shared=shared)
    assert torch.equal(o1, o0)
    assert torch.equal(l1, l0)
    kx = k.repeat(B, 1) if shared else k
    vx = v.repeat(B, 1) if shared else v
    bx = (bias.repeat(B, 1) if shared else bias) if bias is not None else None
    ref = _sdpa_ref(q, kx, vx, B, H, d, bx)
    ref16 = _sdpa_ref(q, kx, vx, B, H, d, bx, dtype=torch.bfloat16)
    assert rel(o1, ref) <= 1.25 * rel(ref16, ref) + 1e-3, (rel(o1, ref), rel(ref16, ref))


@pytest.mark.parametrize("B,H,Nq,Nk,valid,shared", [(8, 4, 1792, 256, 16, True),   # bench's attn2
                                                     (2, 3, 300, 256, 70, False),
                                                     (2, 2, 200, 200, 5, False)])
def test_attention_padding_blocks_skipped_exactly(B, H, Nq, Nk, valid, shared, monkeypatch):
    """The one-pass cross-attention kernels skip key blocks that are all caption padding (bias
    -10000): the skipped probabilities underflow to exactly 0, so O, lse, dQ, dK and dV are bitwise
    those with every block computed (LTX_ATTN_SKIP=0), and dK / dV of padding keys are 0."""
    from ltx_amd import ops
    d = 64
    scale = d ** -0.5
    Bk = 1 if shared else B
    q = g(B * Nq, H * d, seed=51)
    k = g(Bk * Nk, H * d, seed=52)
    v = g(Bk * Nk, H * d, seed=53)
    do = g(B * Nq, H * d, seed=54)
    keep = torch.arange(Nk, device=DEV)[None, :] < (valid + torch.arange(Bk, device=DEV)[:, None])
    bias = ((1 - keep.to(torch.bfloat16)) * -10000.0).float()
    res = {}
    monkeypatch.setenv("LTX_ATTN_BWD1_QS", "0")  # the 8 x 32-key kernel: bitwise skip invariance
    monkeypatch.setenv("LTX_ATTN_BWD1_FEW", "0")
    for mode in ("1", "0"):
        monkeypatch.setenv("LTX_ATTN_SKIP", mode)
        o, lse = ops.attn_fwd(q, k, v, B, H, d, scale, key_bias=bias, kv_shared=shared)
        dq, dk, dv = ops.attn_bwd(q, k, v, o, do, lse, B, H, d, scale, key_bias=bias, kv_shared=shared)
        res[mode] = (o, lse, dq, dk, dv)
    for a, b_ in zip(res["1"], res["0"]):
        assert torch.equal(a, b_)
    # one active 32-key block (bwd1_few_keys, the default there): dQ bitwise, dK / dV to the order
    # of the waves' partial sums, every padding key's rows exactly 0
    monkeypatch.setenv("LTX_ATTN_BWD1_FEW", "1")
    monkeypatch.setenv("LTX_ATTN_SKIP", "1")
    dq3, dk3, dv3 = ops.attn_bwd(q, k, v, res["1"][0], do, res["1"][1], B, H, d, scale, key_bias=bias,
                                 kv_shared=shared)
    assert torch.equal(dq3, res["1"][2])
    assert rel(dk3, res["1"][3]) < 1e-2 and rel(dv3, res["1"][4]) < 1e-2
    pad3 = ~(keep.repeat(B, 1) if shared else keep).reshape(-1)
    assert float(dk3.view(-1, H * d)[pad3].abs().max()) == 0.0
    assert float(dv3.view(-1, H * d)[pad3].abs().max()) == 0.0
    monkeypatch.setenv("LTX_ATTN_BWD1_FEW", "0")
    # the query-split backward (every unmasked key below 128 here): dQ bitwise, dK / dV to the
    # order of two partial sums, padding rows exactly 0
    monkeypatch.setenv("LTX_ATTN_SKIP", "1")
    monkeypatch.setenv("LTX_ATTN_BWD1_QS", "1")
    o, lse = res["1"][:2]
    dq2, dk2, dv2 = ops.attn_bwd(q, k, v, o, do, lse, B, H, d, scale, key_bias=bias, kv_shared=shared)
    assert torch.equal(dq2, res["1"][2])
    assert rel(dk2, res["1"][3]) < 1e-2 and rel(dv2, res["1"][4]) < 1e-2
    for t in (dk2, dv2):
        assert torch.isfinite(t.float()).all()
    o, lse, dq, dk, dv = res["1"]
    pad2 = ~(keep.repeat(B, 1) if shared else keep).reshape(-1)
    assert float(dk2.view(-1, H * d)[pad2].abs().max()) == 0.0
    assert float(dv2.view(-1, H * d)[pad2].abs().max()) == 0.0
    kx = k.repeat(B, 1) if shared else k
    vx = v.repeat(B, 1) if shared else v
    bx = bias.repeat(B, 1) if shared else bias
    ref = _sdpa_ref(q, kx, vx, B, H, d, bx)
    ref16 = _sdpa_ref(q, kx, vx, B, H, d, bx, dtype=torch.bfloat16)
    assert rel(o, ref) <= 1.25 * rel(ref16, ref) + 1e-3, (rel(o, ref), rel(ref16, ref))
    pad = ~(keep.repeat(B, 1) if shared else keep).reshape(-1)
    assert float(dk.view(-1, H * d)[pad].abs().max()) == 0.0
    assert float(dv.view(-1, H * d)[pad].abs().max()) == 0.0


def test_attention_strided_fused_qkv():
    """Q/K/V read in place from the fused [M, 3*H*d] projection buffer (attn1 layout)."""
    from ltx_amd import ops
    B, H, N, d = 2, 4, 192, 64
    D = H * d
    qkv = g(B * N, 3 * D, seed=5)
    q, k, v = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
    o, _ = ops.attn_fwd(q, k, v, B, H, d, d ** -0.5)
    ref = _sdpa_ref(q, k, v, B, H, d)
    ref16 = _sdpa_ref(q, k, v, B, H, d, dtype=torch.bfloat16)
    assert rel(o, ref) <= 1.25 * rel(ref16, ref) + 1e-3, (rel(o, ref), rel(ref16, ref))


# ---------------------------------------------------------------------------------- normalisation
def test_rmsnorm_modulate_fwd_bwd():
    from ltx_amd import ops
    B, N, D = 2, 96, 2048
    x = g(B * N, D, seed=1)
    sst = g(6, D, seed=2, scale=D ** -0.5)
    tmod = g(B, 6 * D, seed=3)
    mod, onep = ops.ada_modulation(sst, tmod, scale_mask=(1 << 1) | (1 << 4))
    ada = sst[None] + tmod.view(B, 6, D)
    assert torch.equal(mod, ada)
    assert torch.equal(onep[:, 1], 1 + ada[:, 1])
    shift, one = mod[:, 0], onep[:, 1]
    y, rstd = ops.rmsnorm_modulate_fwd(x, shift, one, mod.stride(0), N, 1e-6)
    xr = x.view(B, N, D).clone().requires_grad_(True)
    ref = O.rmsnorm(xr, 1e-6) * (1 + ada[:, 1][:, None]) + ada[:, 0][:, None]
    assert ulps_bad(y, ref.detach().view(B * N, D), 1) < 1e-3
    dy = g(B * N, D, seed=4)
    dres = g(B * N, D, seed=5)
    dx = ops.rmsnorm_modulate_bwd(dy, x, rstd, one, mod.stride(0), N, dres=dres)
    ref.backward(dy.view(B, N, D))
    assert rel(dx, xr.grad.view(B * N, D).float() + dres.float()) < 5e-3
    # the gated form (the previous block's FF-output gradient from the same pass): dx unchanged,
    # gout bitwise gate_mul(dx, gate)
    gate = mod[:, 5]
    dx2, gout = ops.rmsnorm_modulate_bwd(dy, x, rstd, one, mod.stride(0), N, dres=dres, gate=gate)
    assert torch.equal(dx2, dx)
    assert torch.equal(gout, ops.gate_mul(dx, gate, N))


def test_layernorm_modulate_fwd_bwd():
    from ltx_amd import ops
    B, N, D = 2, 64, 2048
    x = g(B * N, D, seed=6)
    sst = g(2, D, seed=7, scale=D ** -0.5)
    emb = g(B, D, seed=8)
    mod, onep = ops.ada_modulation(sst, emb, scale_mask=1 << 1, broadcast=True)
    # reference: transformer3d.py:554-560 (shift = row 0, scale = row 1, both sst + emb)
    ssv = sst[None] + emb[:, None]
    y, mean, rstd = ops.layernorm_modulate_fwd(x, mod[:, 0], onep[:, 1], mod.stride(0), N, 1e-6)
    xr = x.view(B, N, D).clone().requires_grad_(True)
    ref = F.layer_norm(xr, (D,), eps=1e-6) * (1 + ssv[:, 1][:, None]) + ssv[:, 0][:, None]
    assert ulps_bad(y, ref.detach().view(B * N, D), 1) < 2e-3
    dy = g(B * N, D, seed=9)
    dx = ops.layernorm_modulate_bwd(dy, x, mean, rstd, onep[:, 1], mod.stride(0), N)
    ref.backward(dy.view(B, N, D))
    assert rel(dx, xr.grad.view(B * N, D)) < 5e-3


@pytest.mark.parametrize("D,grid_float", [(2048, False), (128, False), (2048, True)])
def test_qk_norm_rope_fwd_bwd(D, grid_float):
    from ltx_amd import ops
    B, F_, H_, W_ = 2, 3, 4, 5
    N = F_ * H_ * W_
    coords = O.latent_coords(F_, H_, W_, B, DEV)
    if grid_float:
        coords = coords.float() * torch.tensor([8.0, 32.0, 32.0], device=DEV).view(1, 3, 1) / 25.0
    rope = ops.RopeSpec(coords, D, 10000.0, [20, 2048, 2048])
    qkv = g(B * N, 3 * D, seed=1)
    qw, kw = g(D, seed=2, scale=0.1) + 1, g(D, seed=3, scale=0.1) + 1
    q_out, k_out, rq, rk = ops.qk_norm_rope_fwd(qkv[:, :D], qkv[:, D:2 * D], qw, kw, rope)
    cos, sin = O.rope_freqs(coords.cpu(), D, 10000.0, [20, 2048, 2048], torch.bfloat16)
    cos, sin = cos.to(DEV), sin.to(DEV)
    qi = qkv[:, :D].reshape(B, N, D).clone().requires_grad_(True)
    ki = qkv[:, D:2 * D].reshape(B, N, D).clone().requires_grad_(True)
    qr = O.apply_rotary_emb(O.rmsnorm(qi, 1e-5, qw), cos, sin)
    kr = O.apply_rotary_emb(O.rmsnorm(ki, 1e-5, kw), cos, sin)
    # device sincos vs host libm can flip a bf16 table entry: allow a small fraction of 1-ulp
    assert ulps_bad(q_out, qr.detach().reshape(B * N, D), 1) < 5e-3
    assert rel(q_out, qr.detach().reshape(B * N, D)) < 5e-3
    assert rel(k_out, kr.detach().reshape(B * N, D)) < 5e-3
    dq = g(B * N, D, seed=4)
    dk = g(B * N, D, seed=5)
    dq_raw, dk_raw = ops.qk_norm_rope_bwd(dq, qkv[:, :D], qw, rq, dk, qkv[:, D:2 * D], kw, rk, rope)
    (qr * dq.view(B, N, D)).sum().backward()
    (kr * dk.view(B, N, D)).sum().backward()
    assert rel(dq_raw, qi.grad.reshape(B * N, D)) < 1e-2
    assert rel(dk_raw, ki.grad.reshape(B * N, D)) < 1e-2
    # batch-broadcast coordinates -> one shared cos/sin table: bit-identical to per-batch tables
    shared = ops.RopeSpec(coords[:1].expand(B, -1, -1), D, 10000.0, [20, 2048, 2048])
    assert shared.cs_batch_rows == 0 and shared.cs.shape[0] == N
    assert torch.equal(shared.cs, rope.cs[:N])
    q_s, k_s, _, _ = ops.qk_norm_rope_fwd(qkv[:, :D], qkv[:, D:2 * D], qw, kw, shared)
    assert torch.equal(q_s, q_out) and torch.equal(k_s, k_out)
    dq_s, dk_s = ops.qk_norm_rope_bwd(dq, qkv[:, :D], qw, rq, dk, qkv[:, D:2 * D], kw, rk, shared)
    assert torch.equal(dq_s, dq_raw) and torch.equal(dk_s, dk_raw)
    # q-only / no-rope variant (attn2 q_norm) + f32 incoming gradient
    q2, _, rq2, _ = ops.qk_norm_rope_fwd(qkv[:, :D], None, qw, None, None, B=B, N=N)
    assert ulps_bad(q2, O.rmsnorm(qkv[:, :D], 1e-5, qw), 1) < 1e-3
    dq2, _ = ops.qk_norm_rope_bwd(dq.float(), qkv[:, :D], qw, rq2, B=B, N=N)
    qi2 = qkv[:, :D].clone().requires_grad_(True)
    O.rmsnorm(qi2, 1e-5, qw).backward(dq)
    assert rel(dq2, qi2.grad) < 1e-2


@pytest.mark.parametrize("B,F_,H_,W_", [(4, 2, 4, 8), (8, 7, 4, 4)])
def test_qk_norm_rope_shared_table_item_order(B, F_, H_, W_):
    """One batch-shared RoPE table (cs_batch_rows = 0) against B copies of it, at config-A-like
    batch counts and grids of a multiple of 8 blocks: bitwise the same outputs."""
    from ltx_amd import ops
    D, N = 2048, F_ * H_ * W_
    coords = O.latent_coords(F_, H_, W_, 1, DEV)
    per_batch = ops.RopeSpec(coords.expand(B, -1, -1).contiguous(), D, 10000.0, [20, 2048, 2048])
    shared = ops.RopeSpec(coords.expand(B, -1, -1), D, 10000.0, [20, 2048, 2048])
    assert per_batch.cs_batch_rows == N and shared.cs_batch_rows == 0
    assert (B * N * 2 // 4) % 8 == 0
    qkv = g(B * N, 3 * D, seed=11)
    qw, kw = g(D, seed=12, scale=0.1) + 1, g(D, seed=13, scale=0.1) + 1
    a = ops.qk_norm_rope_fwd(qkv[:, :D], qkv[:, D:2 * D], qw, kw, per_batch)
    b = ops.qk_norm_rope_fwd(qkv[:, :D], qkv[:, D:2 * D], qw, kw, shared)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    dq, dk = g(B * N, D, seed=14), g(B * N, D, seed=15)
    ga = ops.qk_norm_rope_bwd(dq, qkv[:, :D], qw, a[2], dk, qkv[:, D:2 * D], kw, a[3], per_batch)
    gb = ops.qk_norm_rope_bwd(dq, qkv[:, :D], qw, a[2], dk, qkv[:, D:2 * D], kw, a[3], shared)
    for x, y in zip(ga, gb):
        assert torch.equal(x, y)


def test_qk_norm_grouped_matches_per_group():
    """ltx_qk_norm_{fwd,bwd}_grouped (every block's text k_norm in one launch) against one
    qk_norm_rope_{fwd,bwd} call per group: bitwise, at LTX-2B widths with strided group views."""
    from ltx_amd import ops
    G, L, D = 5, 256, 2048
    kv = g(L, 2 * G * D, seed=21)                          # [k_0 | v_0 | k_1 | v_1 | ...]
    w = torch.stack([g(D, seed=30 + i, scale=0.1) + 1 for i in range(G)]).contiguous()
    y, rstd = ops.qk_norm_fwd_grouped(kv, 2 * D, w)
    dy = g(G, L, D, seed=22)
    dx = torch.zeros(L, 2 * G * D, dtype=torch.bfloat16, device=DEV)
    ops.qk_norm_bwd_grouped(dy.view(G * L, D), L * D, kv, 2 * D, w, rstd, dx, 2 * D)
    # in place on a strided stack (the batched text side's dkv k columns)
    dk_inplace = torch.zeros(L, 2 * G * D, dtype=torch.bfloat16, device=DEV)
    for i in range(G):
        dk_inplace[:, 2 * i * D:(2 * i + 1) * D] = dy[i]
    ops.qk_norm_bwd_grouped(dk_inplace, 2 * D, kv, 2 * D, w, rstd, dk_inplace, 2 * D)
    assert torch.equal(dk_inplace, dx)
    for i in range(G):
        xi = kv[:, 2 * i * D:(2 * i + 1) * D]
        yi, _, ri, _ = ops.qk_norm_rope_fwd(xi, None, w[i], None, None, B=1, N=L)
        assert torch.equal(y[i], yi) and torch.equal(rstd[i], ri)
        dxi, _ = ops.qk_norm_rope_bwd(dy[i], xi, w[i], ri, B=1, N=L)
        assert torch.equal(dx[:, 2 * i * D:(2 * i + 1) * D], dxi)
        assert float(dx[:, (2 * i + 1) * D:(2 * i + 2) * D].abs().max()) == 0.0  # v columns untouched


# ------------------------------------------------------------------------- patchify / rf / misc
def test_patchify_coords_bit_exact():
    from ltx_amd import ops
    for (B, C, F_, H_, W_) in [(2, 128, 7, 16, 16), (1, 8, 3, 4, 5), (2, 3, 1, 8, 8)]:
        lat = g(B, C, F_, H_, W_, seed=1)
        tok = ops.patchify(lat)
        ref, coords = O.patchify(lat)
        assert torch.equal(tok, ref)
        assert torch.equal(ops.latent_coords(B, F_, H_, W_, DEV), coords)
        assert torch.equal(ops.unpatchify(tok, F_, H_, W_), lat)


def test_rf_prepare_tokens():
    from ltx_amd import ops
    B, C, F_, H_, W_ = 2, 128, 3, 8, 8
    lat, ref, pose = g(B, C, F_, H_, W_, seed=1), g(B, C, 1, H_, W_, seed=2), g(B, C, F_, H_, W_, seed=3)
    tok, _ = O.patchify(lat)
    noise = g(*tok.shape, seed=4)
    t = torch.tensor([0.3, 0.77], device=DEV)
    x_t, model_in, v = ops.rf_prepare_tokens(lat, ref, pose, noise, t, want_x_t=True)
    x_ref = O.add_noise(tok, noise, t).to(torch.bfloat16)
    v_ref = O.velocity_target(tok, noise, t).to(torch.bfloat16)
    assert torch.equal(x_t, x_ref)
    assert torch.equal(v, v_ref)
    u = O.unpatchify(x_ref.clone(), H_, W_, C)
    u[:, :, 0:1] = torch.lerp(u[:, :, 0:1], ref, 0.85)
    u[:, :, 1:] = torch.lerp(u[:, :, 1:], pose[:, :, 1:], 0.5)
    mi_ref, _ = O.patchify(u)
    assert torch.equal(model_in, mi_ref)
    assert torch.equal(ops.condition_lerp(x_t, ref, pose), mi_ref)
    x2, v2 = ops.rf_noise_velocity(tok, noise, t)
    assert torch.equal(x2, x_ref) and torch.equal(v2, v_ref)


def test_scheduler_add_noise_and_velocity_are_f32_like_the_reference():
    """RectifiedFlowScheduler.add_noise / build_velocity_target (rf.py:376-386, 400-426) return
    f32 for f32 timesteps: bitwise the oracle's f32 values, bf16 or f32 inputs."""
    from ltx_amd.scheduler import RectifiedFlowScheduler
    sch = RectifiedFlowScheduler()
    t = torch.tensor([0.3, 0.77, 0.05], device=DEV)
    for dt in (torch.bfloat16, torch.float32):
        tok = g(3, 192, 128, seed=5).to(dt)
        noise = g(3, 192, 128, seed=6).to(dt)
        x = sch.add_noise(tok, noise, t)
        v = sch.build_velocity_target(tok, noise, t)
        assert x.dtype == torch.float32 and v.dtype == torch.float32
        assert torch.equal(x, O.add_noise(tok, noise, t))
        assert torch.equal(v, O.velocity_target(tok, noise, t))


def test_timestep_silu_transpose_colsum():
    from ltx_amd import ops
    t = torch.tensor([0.01, 0.5, 0.999, 0.25], device=DEV)
    emb = ops.timestep_embedding(t, 1000.0)
    ref = O.timestep_embedding(1000 * t).to(torch.bfloat16)
    assert ulps_bad(emb, ref, 1) < 1e-2 and rel(emb, ref) < 5e-3
    x = g(37, 2048, seed=3)
    assert ulps_bad(ops.silu(x), F.silu(x), 1) < 1e-3
    x = g(300, 136, seed=4)
    assert torch.equal(ops.transpose(x), x.t().contiguous())
    # 16-B vector path: ragged tiles, a strided source view and a padded destination (_tpad)
    x = g(1000, 136, seed=5)
    assert torch.equal(ops.transpose(x), x.t().contiguous())
    big = g(1000, 3 * 136, seed=6)
    xt = ops._tpad(big[:, 136:272], 1024)
    assert torch.equal(xt[:, :1000], big[:, 136:272].t()) and float(xt[:, 1000:].abs().max()) == 0
    cs = ops.colsum(x)
    assert rel(cs, x.float().sum(0)) < 5e-3


@pytest.mark.parametrize("M,r", [(1000, 16), (2048, 16), (333, 8), (517, 32), (4480, 8), (14336, 16)])
def test_lora_kernels(M, r):
    from ltx_amd import ops
    K, N = 2048, 2048
    x = g(M, K, seed=1)
    A = torch.randn(r, K, device=DEV) / K ** 0.5
    Bm = torch.randn(N, r, device=DEV) * 0.05
    u, su = ops.lora_down(x, A, split=True)
    assert rel(u, x.float() @ A.t()) < 1e-5
    assert torch.equal(su, ops.lora_split(u, "act"))  # fused split == standalone split
    dy = g(M, N, seed=2)
    w = ops.lora_down(dy, Bm, alpha=0.5, transposed=True)
    assert rel(w, 0.5 * dy.float() @ Bm) < 1e-5
    dB = ops.lora_wgrad(dy, u, alpha=0.5)
    assert rel(dB, 0.5 * dy.float().t() @ u) < 1e-5
    dA = ops.lora_wgrad(x, w, transpose_out=True)
    assert rel(dA, w.t() @ x.float()) < 1e-5
    # accumulate into an existing buffer (the .grad path): buf + product
    buf = torch.randn(N, r, device=DEV)
    ref = buf + 0.5 * dy.float().t() @ u
    ops.lora_wgrad(dy, u, alpha=0.5, out=buf, accumulate=True)
    assert rel(buf, ref) < 1e-5


@pytest.mark.parametrize("M,N,r", [(1792, 2048, 16), (1760, 1024, 16), (4480, 512, 8), (32, 512, 16)])
def test_lora_dy_one_pass(M, N, r):
    """ltx_lora_dy = lora_down(dY, B, transposed, split) + lora_wgrad(dY, u, accumulate) in one
    pass over dY: the same f32 products to summation order (fp32 reference), the split operand
    exactly lora_split of its own w, dB added into the existing buffer. Ragged row splits (M not a
    multiple of 224) and a single 32-row group included."""
    from ltx_amd import ops
    dy = g(M, N, seed=3)
    u = torch.randn(M, r, device=DEV)
    Bm = torch.randn(N, r, device=DEV) * 0.05
    pieces = ops.lora_pieces(Bm, transposed=True)
    assert ops.lora_dy_fits(dy, r)
    buf = torch.randn(N, r, device=DEV)
    ref_dB = buf + 0.5 * dy.float().t() @ u
    w, sp = ops.lora_dy(dy, u, pieces, r, 0.5, buf)
    assert rel(w, 0.5 * dy.float() @ Bm) < 1e-5
    assert torch.equal(sp, ops.lora_split(w, "act"))
    assert rel(buf, ref_dB) < 1e-5
    # against the two-kernel path it replaces
    w2, sp2 = ops.lora_rows(dy, pieces, r, alpha=0.5, split=True)
    assert rel(w, w2) < 1e-6
    buf2 = torch.zeros(N, r, device=DEV)
    ops.lora_dy(dy, u, pieces, r, 0.5, buf2, accumulate=False)
    assert rel(buf2, ops.lora_wgrad(dy, u, alpha=0.5)) < 1e-6
    # with the adapter's dA = x^T . w in the same call (ltx_lora_dy_dA: the x pass reads w from the
    # dY pass's partials, one finish for all): w, split and dB bitwise the call above; dA bitwise
    # ltx_lora_wgrad(x, w) where that takes its token-sized path (M >= 2048), else to f32 order
    K = 1024 if N != 1024 else 512
    x = g(M, K, seed=9)
    bB1, bA1 = torch.randn(N, r, device=DEV), torch.randn(r, K, device=DEV)
    bB2, bA2 = bB1.clone(), bA1.clone()
    w1, sp1 = ops.lora_dy(dy, u, pieces, r, 0.5, bB1)
    ops.lora_wgrad(x, w1, transpose_out=True, out=bA1, accumulate=True)
    w2, sp2 = ops.lora_dy(dy, u, pieces, r, 0.5, bB2, x=x, dA_out=bA2)
    assert torch.equal(w1, w2) and torch.equal(sp1, sp2) and torch.equal(bB1, bB2)
    if M >= 2048:
        assert torch.equal(bA1, bA2)
    else:
        assert rel(bA2, bA1) < 1e-6
    bA3 = torch.zeros(r, K, device=DEV)
    ops.lora_dy(dy, u, pieces, r, 0.5, torch.zeros(N, r, device=DEV), x=x, dA_out=bA3, dA_accumulate=False)
    assert rel(bA3, w1.t() @ x.float()) < 1e-5


@pytest.mark.parametrize("M,K,r", [(14336, 2048, 16), (4480, 1024, 8), (2048, 512, 16)])
def test_lora_rows_token_sized(M, K, r):
    """ltx_lora_rows at token-sized M (the column-split lora_dy_kernel path + its finish): u against
    fp32, the split operand exactly lora_split of its own u, and a strided out / split_out view."""
    from ltx_amd import ops
    x = g(M, K, seed=7)
    A = torch.randn(r, K, device=DEV) / K ** 0.5
    pieces = ops.lora_pieces(A)
    u, su = ops.lora_rows(x, pieces, r, alpha=0.5, split=True)
    assert rel(u, 0.5 * x.float() @ A.t()) < 1e-5
    assert torch.equal(su, ops.lora_split(u, "act"))
    K2 = ops.lora_k2(r)
    big = torch.full((M, 2 * K2), 7.0, dtype=torch.bfloat16, device=DEV)
    outb = torch.full((M, 2 * r), 3.0, device=DEV)
    u2, _ = ops.lora_rows(x, pieces, r, alpha=0.5, out=outb[:, r:], split=True, split_out=big[:, K2:])
    assert torch.equal(u2, u) and torch.equal(big[:, K2:], su)
    assert float((big[:, :K2] - 7.0).abs().max()) == 0 and float((outb[:, :r] - 3.0).abs().max()) == 0


def test_mse_and_adamw():
    from ltx_amd import ops
    o, v = g(2, 64, 128, seed=1), g(2, 64, 128, seed=2)
    stats, dout = ops.mse_fwd_bwd(o, v, grad_scale=1 / 16)
    n = o.numel()
    oo = o.clone().requires_grad_(True)
    loss = F.mse_loss(oo, v)
    (loss / 16).backward()
    assert abs(float(stats[0]) / n - float(loss)) < 1e-2 * float(loss)
    assert ulps_bad(dout, oo.grad, 1) < 1e-3
    std = torch.sqrt((stats[2] - stats[1] ** 2 / n) / (n - 1))
    assert abs(float(std) - float(v.float().std())) < 1e-3
    # deterministic (fixed-order partials, no atomics), ragged size with a scalar tail
    o2, v2 = g(3, 1001, 7, seed=4), g(3, 1001, 7, seed=5)
    s_a, d_a = ops.mse_fwd_bwd(o2, v2)
    s_b, d_b = ops.mse_fwd_bwd(o2, v2)
    assert torch.equal(s_a, s_b) and torch.equal(d_a, d_b)
    oo2 = o2.clone().requires_grad_(True)
    l2 = F.mse_loss(oo2, v2)
    l2.backward()
    assert abs(float(s_a[0]) / o2.numel() - float(l2)) < 1e-2 * float(l2)
    assert ulps_bad(d_a, oo2.grad, 1) < 1e-3
    for dtype in (torch.float32, torch.bfloat16):
        p0 = g(4096, dtype=dtype, seed=3)
        grads = [g(4096, dtype=dtype, seed=10 + i) for i in range(3)]
        pt = torch.nn.Parameter(p0.clone())
        opt = torch.optim.AdamW([pt], lr=1e-4)
        mine = p0.clone()
        m = torch.zeros_like(mine)
        vv = torch.zeros_like(mine)
        for step, gr in enumerate(grads, start=1):
            pt.grad = gr.clone()
            opt.step()
            ops.adamw_step(mine, gr, m, vv, 1e-4, 0.9, 0.999, 1e-8, 0.01, step)
        if dtype == torch.float32:
            assert rel(mine, pt.detach()) < 1e-6
        else:
            assert ulps_bad(mine, pt.detach(), 1) < 1e-3


def test_gemm_k_extension_lora_fusion():
    """LoRA fused into the K loop: [x | split(u)] . [W | split(s*B)]^T == x.W^T + b + s*u.B^T
    with u = x.A^T in f32 (peft), for both tile kernels and for the dgrad orientation."""
    from ltx_amd import ops
    for M, N, K in ((512, 256, 256), (14336 // 2, 2048, 2048), (256, 2048, 2048)):  # + split-K
        r, s = 16, 0.5
        x, w, b = g(M, K, seed=21), g(N, K, seed=22, scale=K ** -0.5), g(N, seed=23)
        A = torch.randn(r, K, device=DEV) / K ** 0.5
        Bm = torch.randn(N, r, device=DEV) * 0.1
        u = ops.lora_down(x, A)
        out = ops.gemm(x, w, bias=b, ext=(ops.lora_split(u, "act"), ops.lora_split(Bm, "weight", s)))
        ref = x.float() @ w.float().t() + b.float() + s * (u @ Bm.t())
        assert rel(out, ref) < 1e-2
        assert ulps_bad(out, ref.to(torch.bfloat16), 2) < 2e-3
        # dgrad orientation: dy . W + w . A with w = s * dy . B  (A^T split as the weight side)
        dy = g(M, N, seed=24)
        wd = ops.lora_down(dy, Bm, alpha=s, transposed=True)
        wT = ops.transpose(w)
        dx = ops.gemm(dy, wT, ext=(ops.lora_split(wd, "act"), ops.lora_split(A, "weight", transposed=True)))
        ref = dy.float() @ w.float() + wd @ A
        assert rel(dx, ref) < 1e-2
        # the 3-term split reproduces the f32 rank-r product to ~1e-5
        sa, sw = ops.lora_split(u, "act").float(), ops.lora_split(Bm, "weight", s).float()
        assert rel(sa @ sw.t(), s * (u @ Bm.t())) < 1e-4


@pytest.mark.parametrize("M,N,K", [(2048, 2048, 14336), (256, 2048, 2048 * 8), (512, 768, 4096)])
def test_gemm_large_tile_split_k(M, N, K):
    """Grids under one round of 256x256 tiles with a long K (full-mode weight grads) take the
    split-K large-tile kernel: store and accumulate epilogues vs fp32, rounded once."""
    from ltx_amd import ops
    a, w = g(M, K, seed=31), g(N, K, seed=32, scale=K ** -0.5)
    ref = a.float() @ w.float().t()
    out = ops.gemm(a, w)
    assert ulps_bad(out, ref.to(torch.bfloat16), 2) < 1e-3
    acc = g(M, N, seed=33)
    exp = (acc.float() + ref.to(torch.bfloat16).float()).to(torch.bfloat16)
    ops.gemm(a, w, epilogue="accum", aux0=acc, out=acc)
    assert ulps_bad(acc, exp, 2) < 1e-3


@pytest.mark.parametrize("M,N,K", [(14336, 2048, 2048), (1000, 136, 320), (256, 2048, 4096)])
def test_gemm_store_bias_and_wgrad(M, N, K):
    """Plain store + bias on the hand-written kernels, and the nn.Linear weight gradient dy^T . x
    over the token axis (ops.wgrad: token-major operands transposed, the token axis zero-padded
    to a multiple of 64), fresh and accumulated with autograd's AccumulateGrad roundings."""
    from ltx_amd import ops
    a, w, b = g(M, K, seed=41), g(N, K, seed=42, scale=K ** -0.5), g(N, seed=43)
    ref = (a.float() @ w.float().t() + b.float()).to(torch.bfloat16)
    out = ops.gemm(a, w, bias=b)
    assert ulps_bad(out, ref, 2) < 1e-3
    dy = g(M, N, seed=44, scale=M ** -0.5)
    wg = ops.wgrad(dy, a)
    refw = (dy.float().t() @ a.float()).to(torch.bfloat16)
    assert ulps_bad(wg, refw, 2) < 1e-3
    acc = g(N, K, seed=45)
    exp = (acc.float() + refw.float()).to(torch.bfloat16)
    ops.wgrad_into(acc, dy, a)
    assert ulps_bad(acc, exp, 2) < 1e-3
    # strided column slices (the fused q/k/v gradient rows of dQKV)
    big = g(M, 3 * N, seed=46, scale=M ** -0.5)
    wg2 = ops.wgrad(big[:, N:2 * N], a)
    assert ulps_bad(wg2, (big[:, N:2 * N].float().t() @ a.float()).to(torch.bfloat16), 2) < 1e-3


def test_gated_residual_long_k():
    """Long-K gated residual (FF-down, K = 8192) with the pre-gate y store (full mode): the fused
    epilogue's roundings y = bf16(x.W^T + b), out = bf16(R + bf16(gate * y))."""
    from ltx_amd import ops
    M, N, K, B = 1792 * 2, 2048, 8192, 2
    a, w, b = g(M, K, seed=51), g(N, K, seed=52, scale=K ** -0.5), g(N, seed=53)
    R, gate = g(M, N, seed=54), g(B, N, seed=55)
    y = (a.float() @ w.float().t() + b.float()).to(torch.bfloat16)
    ref = (R.float() + (gate.repeat_interleave(M // B, 0).float() * y.float()).to(torch.bfloat16).float()
           ).to(torch.bfloat16)
    ykeep = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    out = ops.gemm(a, w, bias=b, epilogue="gated_residual", aux0=R, aux1=gate, aux2=ykeep,
                   rows_per_batch=M // B)
    assert ulps_bad(ykeep, y, 2) < 1e-3
    assert ulps_bad(out, ref, 2) < 2e-3


def test_add_bf16_accumulate_grad_semantics():
    """ltx_add_bf16: bf16(x + y) like autograd's bf16 AccumulateGrad, in place, strided rows."""
    from ltx_amd import ops
    big = g(300, 3 * 136, seed=61)
    x = big[:, 136:272]
    y = g(300, 136, seed=62)
    exp = (x.float() + y.float()).to(torch.bfloat16)
    ops.add_into(x, y)
    assert torch.equal(x, exp)
    assert torch.equal(big[:, :136], g(300, 3 * 136, seed=61)[:, :136])


def test_fused_adamw_multi_tensor_bitwise():
    """FusedAdamW's one-launch-per-dtype path (ltx_adamw_multi) == the per-tensor kernels, bitwise,
    over mixed f32 (LoRA) / bf16 (caption projection) tensors, several steps."""
    from ltx_amd.training import FusedAdamW
    shapes = [((16, 2048), torch.float32), ((2048, 16), torch.float32), ((3000,), torch.bfloat16),
              ((64, 130), torch.bfloat16), ((5,), torch.float32)]

    def run(multi):
        ps = [torch.nn.Parameter(g(*sh, dtype=dt, seed=70 + i)) for i, (sh, dt) in enumerate(shapes)]
        opt = FusedAdamW(ps, lr=1e-2, multi_tensor=multi)
        for k in range(3):
            for i, p in enumerate(ps):
                p.grad = g(*p.shape, dtype=p.dtype, seed=100 * k + i)
            opt.step()
        return [p.detach().clone() for p in ps]
    a, b = run(True), run(False)
    for x, y in zip(a, b):
        assert torch.equal(x, y)



@pytest.mark.parametrize("B,H,Nq,Nk", [(2, 3, 1000, 768), (1, 4, 1792, 1792), (1, 2, 70, 320), (1, 2, 50, 512),
                                       (2, 2, 320, 1792), (1, 3, 64, 256), (1, 2, 129, 192)])
def test_attention_dkdv_w1_matches_pipe_bitwise(B, H, Nq, Nk, monkeypatch):
    """attn_dkdv_w1_kernel (one wave per SIMD, 64 keys per wave, hand-scheduled loop from
    tools/gen_attn_bwd.py; LTX_ATTN_DKDV_W1=1) keeps attn_dkdv_pipe_kernel's arithmetic and
    accumulation order: dK and dV bitwise equal, including ragged query tiles (rows past Nq read as
    zeros through the shrinking buffer descriptor) and key blocks past Nk; dQ is the same kernel."""
    from ltx_amd import ops
    d = 64
    scale = d ** -0.5
    qkv = g(B * Nq, 3 * H * d, seed=71)
    q = qkv[:, :H * d]
    k = g(B * Nk, H * d, seed=72)
    v = g(B * Nk, H * d, seed=73)
    do = g(B * Nq, H * d, seed=74)
    o, lse = ops.attn_fwd(q, k, v, B, H, d, scale)
    outs = {}
    for w1 in ("0", "1"):
        monkeypatch.setenv("LTX_ATTN_DKDV_W1", w1)
        outs[w1] = ops.attn_bwd(q, k, v, o, do, lse, B, H, d, scale)
    for a, b_ in zip(outs["1"], outs["0"]):
        assert torch.equal(a, b_)


@pytest.mark.parametrize("B,H,Nq,Nk,jump", [(8, 32, 1792, 1792, 0), (2, 3, 1000, 768, 0), (1, 2, 70, 320, 0),
                                            (2, 4, 300, 256, 0), (2, 2, 1792, 1792, 4), (1, 2, 7488, 7488, 16),
                                            (1, 3, 500, 1344, 1)])
def test_attention_fwd_w1_matches_pipe_bitwise(B, H, Nq, Nk, jump, monkeypatch):
    """attn_fwd_w1_kernel (one wave per SIMD, 64 queries per wave, hand-scheduled loop from
    tools/gen_attn_fwd.py; LTX_ATTN_FWD_W1=1 in the opt-in `make fwdw1` library) keeps attn_fwd_pipe_kernel<true>'s arithmetic,
    deferred-max decisions and accumulation order: O and lse bitwise equal, ragged query blocks and odd
    tile counts included. jump > 0: the keys' logits step up by ~17 log2 units every `jump` tiles, so
    most rows take the out-of-line redo (the tile max, alpha, the O / l rescale) several times."""
    from ltx_amd import ops
    d = 64
    scale = d ** -0.5
    q = g(B * Nq, H * d, seed=61)
    k = g(B * Nk, H * d, seed=62)
    v = g(B * Nk, H * d, seed=63)
    if jump:
        gen = torch.Generator(device="cpu").manual_seed(64)
        qh = q.float().view(B, Nq, H, d).cpu()
        kh = k.float().view(B, Nk, H, d).cpu()
        qh[..., 0] = torch.where(torch.rand(B, Nq, H, generator=gen) < 0.7, 4.0, -4.0)
        t = torch.arange(Nk) // 64
        kh[..., 0] = (-60.0 + 24.0 * (t // jump).float() + torch.rand(Nk, generator=gen) * 3.0).clamp(max=60.0).view(1, Nk, 1)
        q = qh.reshape(B * Nq, H * d).cuda().bfloat16()
        k = kh.reshape(B * Nk, H * d).cuda().bfloat16()
    from ltx_amd import _lib as L
    lib = os.path.join(os.path.dirname(L.LIB_PATH), "libltxhip_fwdw1.so")
    if not os.path.exists(lib):
        pytest.skip("the one-wave forward is not in the shipping library: `make -C csrc fwdw1` builds it")
    saved = L._lib
    L._lib = None
    outs = {}
    try:
        L.load(lib)
        for w1 in ("0", "1"):
            monkeypatch.setenv("LTX_ATTN_FWD_W1", w1)
            outs[w1] = ops.attn_fwd(q, k, v, B, H, d, scale)
    finally:
        L._lib = saved
    assert torch.equal(outs["1"][0], outs["0"][0])
    assert torch.equal(outs["1"][1], outs["0"][1])


# (8, 32, 1792, 1792): config A's self-attention, 7 blocks per workgroup; (4, 16, 7488, 7488): config
# X-like, 30 blocks per workgroup; the small ones give every block its own workgroup
@pytest.mark.parametrize("B,H,Nq,Nk", [(8, 32, 1792, 1792), (4, 16, 7488, 7488), (2, 3, 1000, 768), (1, 2, 70, 320),
                                       (2, 2, 320, 1792), (1, 3, 64, 256), (1, 2, 129, 192), (3, 40, 200, 1300)])
def test_attention_dkdv_w1p_matches_w1_bitwise(B, H, Nq, Nk, monkeypatch):
    """attn_dkdv_w1p_kernel (persistent: one workgroup per CU walks 256-key blocks, the next block's
    K / V fragments and first Q / dO tiles loaded under the previous block's tail and stores;
    LTX_ATTN_DKDV_W1=2) runs attn_dkdv_w1_kernel's loop per block: dK and dV bitwise equal, ragged
    key blocks (K / V past Nk read as zeros, their rows not stored) and query tiles included."""
    from ltx_amd import ops
    d = 64
    scale = d ** -0.5
    q = g(B * Nq, H * d, seed=91)
    k = g(B * Nk, H * d, seed=92)
    v = g(B * Nk, H * d, seed=93)
    do = g(B * Nq, H * d, seed=94)
    o, lse = ops.attn_fwd(q, k, v, B, H, d, scale)
    outs = {}
    for w1 in ("1", "2"):
        monkeypatch.setenv("LTX_ATTN_DKDV_W1", w1)
        outs[w1] = ops.attn_bwd(q, k, v, o, do, lse, B, H, d, scale)
    for a, b_ in zip(outs["2"], outs["1"]):
        assert torch.equal(a, b_)


@pytest.mark.parametrize("B,H,Nq,Nk", [(8, 32, 1792, 1792), (4, 16, 7488, 7488), (2, 3, 1000, 768), (1, 2, 70, 320),
                                       (2, 2, 320, 1792), (1, 3, 300, 64), (1, 2, 129, 192), (3, 40, 1300, 200)])
def test_attention_dq_w1p_matches_w1_bitwise(B, H, Nq, Nk, monkeypatch):
    """attn_dq_w1p_kernel (persistent: one workgroup per CU walks 256-query blocks, the next block's
    Q / dO fragments, lse and delta loaded under the previous block's tail and stores;
    LTX_ATTN_DQ_W1=2) runs attn_dq_w1_kernel's loop per block: bf16 dQ bitwise equal, ragged query
    blocks (rows past Nq read as zeros, not stored) included; the f32 dQ keeps the per-block kernel."""
    from ltx_amd import ops
    d = 64
    scale = d ** -0.5
    q = g(B * Nq, H * d, seed=95)
    k = g(B * Nk, H * d, seed=96)
    v = g(B * Nk, H * d, seed=97)
    do = g(B * Nq, H * d, seed=98)
    o, lse = ops.attn_fwd(q, k, v, B, H, d, scale)
    outs = {}
    for w1 in ("1", "2"):
        monkeypatch.setenv("LTX_ATTN_DQ_W1", w1)
        outs[w1] = ops.attn_bwd(q, k, v, o, do, lse, B, H, d, scale)
    for a, b_ in zip(outs["2"], outs["1"]):
        assert torch.equal(a, b_)


@pytest.mark.parametrize("B,H,Nq,Nk", [(2, 3, 1000, 768), (1, 4, 1792, 1792), (1, 2, 70, 320), (1, 2, 50, 512),
                                       (2, 2, 320, 1792), (1, 3, 300, 64), (1, 2, 129, 192)])
def test_attention_dq_w1_matches_pipe_bitwise(B, H, Nq, Nk, monkeypatch):
    """attn_dq_w1_kernel (one wave per SIMD, 64 queries per wave, hand-scheduled loop from
    tools/gen_attn_bwd.py; LTX_ATTN_DQ_W1, default on) keeps attn_dq_pipe_kernel's arithmetic and
    accumulation order: dQ bitwise equal in bf16 and in f32, ragged query blocks included."""
    from ltx_amd import ops
    d = 64
    scale = d ** -0.5
    qkv = g(B * Nq, 3 * H * d, seed=81)
    q = qkv[:, :H * d]
    k = g(B * Nk, H * d, seed=82)
    v = g(B * Nk, H * d, seed=83)
    do = g(B * Nq, H * d, seed=84)
    o, lse = ops.attn_fwd(q, k, v, B, H, d, scale)
    for f32 in (False, True):
        outs = {}
        for w1 in ("0", "1"):
            monkeypatch.setenv("LTX_ATTN_DQ_W1", w1)
            outs[w1] = ops.attn_bwd(q, k, v, o, do, lse, B, H, d, scale, dq_f32=f32)
        for a, b_ in zip(outs["1"], outs["0"]):
            assert torch.equal(a, b_), f32
