"""Attention with LARGE logits (attention.py:1057-1064 with learned q/k norms, attention.py:434-436,
can give scaled scores of tens): the online-softmax paths that N(0, 1) inputs never take.

* The deferred-max rescale: the running max is only moved (and O, l rescaled) when a 64-key tile's
  max exceeds it by more than RESCALE_TAU = 8 log2 units (attention_common.h); here the key rows
  are built so the max of many query rows jumps by ~17 log2 units every few tiles.
* The speculative-sum fallback of the pipelined forward (attention_pipe.hip): a tile is first
  exponentiated at the running max and recomputed when a lane's probabilities sum past 2^TAU --
  every such jump takes it.
* Single dominant keys (one key ~20 natural units above the rest of its row).

Every case is checked (1) against fp32 SDPA under SURVEY 8(c)(4)'s noise criterion:
err(build, fp32) <= 1.25 * err(torch bf16 SDPA, fp32) + 1e-3 (rel-Frobenius), for O, dQ, dK, dV,
and (2) against the same kernels built with RESCALE_TAU = 0 (libltxhip_tau0.so: every growth of the
running max rescales, the textbook online softmax). That the rescale branch runs is asserted from
the inputs: the test computes, per query row, the 64-key tile maxima of the scores in log2 units
and requires jumps past the running max by more than 8 in a large share of rows -- the kernel's own
branch condition (its tiles are the 64-key tiles the test walks).
"""
import contextlib
import math
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
TAU = 8.0
HERE = os.path.dirname(os.path.abspath(__file__))
TAU0_LIB = os.path.join(os.path.dirname(HERE), "video-generation-for-human-avatars_amd", "ltx_amd",
                        "libltxhip_tau0.so")


@pytest.fixture(scope="module", autouse=True)
def _dev():
    from ltx_amd import _lib as L
    L.ensure_device()


@contextlib.contextmanager
def library(path):
    """Route ltx_amd.ops through another build of the library for the duration."""
    from ltx_amd import _lib as L
    saved = L._lib
    L._lib = None
    try:
        L.load(path)
        yield
    finally:
        L._lib = saved


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


def make_inputs(B, Bk, H, Nq, Nk, d, jump_every, seed):
    """q, k, v [rows, H*d] bf16 with scores s = (q.k) * d^-0.5 ~ b_i * a_t / 2 (+ noise): a_t steps
    up by 24 every `jump_every` 64-key tiles (the row max jumps by 12 natural = 17.3 log2 units),
    b_i = +-4 per query row (rows with b < 0 peak in the first tiles instead), plus one spike key
    per (batch, head) that dominates its rows by ~20 natural units; scores span about +-60."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    q = torch.randn(B, Nq, H, d, generator=g) * 0.5
    k = torch.randn(Bk, Nk, H, d, generator=g) * 0.5
    v = torch.randn(Bk, Nk, H, d, generator=g)
    b = torch.where(torch.rand(B, Nq, H, generator=g) < 0.7, 4.0, -4.0)
    q[..., 0] = b
    t = torch.arange(Nk) // 64
    a = -60.0 + 24.0 * (t // jump_every).float() + torch.rand(Nk, generator=g) * 3.0
    a = a.clamp(max=60.0)
    k[..., 0] = a.view(1, Nk, 1)
    spike = torch.randint(0, Nk, (Bk, H), generator=g)
    for bb in range(Bk):
        for hh in range(H):
            k[bb, spike[bb, hh], hh, 0] = min(float(a.max()) + 40.0, 118.0)
    return (q.reshape(B * Nq, H * d).to(DEV).bfloat16(), k.reshape(Bk * Nk, H * d).to(DEV).bfloat16(),
            v.reshape(Bk * Nk, H * d).to(DEV).bfloat16())


def scores_log2(q, k, B, Bk, H, Nq, Nk, d, bias):
    qh = q.float().view(B, Nq, H, d).transpose(1, 2)
    kh = k.float().view(Bk, Nk, H, d).transpose(1, 2).expand(B, H, Nk, d)
    s = (qh @ kh.transpose(-1, -2)) * d ** -0.5
    if bias is not None:
        s = s + bias.view(-1, 1, 1, Nk).expand(B, 1, 1, Nk)
    return s * (1.0 / math.log(2.0))


def rescale_share(s2):
    """share of query rows whose running 64-key-tile max grows by more than TAU at least once
    after the first tile (the kernels' rescale condition)"""
    Nk = s2.shape[-1]
    T = (Nk + 63) // 64
    tm = torch.stack([s2[..., 64 * i:64 * (i + 1)].amax(-1) for i in range(T)], -1)
    run = tm[..., :1]
    hit = torch.zeros_like(run[..., 0], dtype=torch.bool)
    m = run[..., 0]
    for i in range(1, T):
        jump = tm[..., i] > m + TAU
        hit |= jump
        m = torch.where(jump, tm[..., i], m)  # the kernel keeps the stale max below TAU
    return float(hit.float().mean())


def sdpa(q, k, v, B, Bk, H, Nq, Nk, d, bias, dtype):
    qh = q.to(dtype).view(B, Nq, H, d).transpose(1, 2)
    kh = k.to(dtype).view(Bk, Nk, H, d).transpose(1, 2).expand(B, H, Nk, d)
    vh = v.to(dtype).view(Bk, Nk, H, d).transpose(1, 2).expand(B, H, Nk, d)
    mask = None if bias is None else bias.view(-1, 1, 1, Nk).expand(B, 1, 1, Nk).to(dtype)
    return F.scaled_dot_product_attention(qh, kh, vh, attn_mask=mask).transpose(1, 2).reshape(B * Nq, H * d)


def reference(q, k, v, do, B, Bk, H, Nq, Nk, d, bias, dtype):
    qf, kf, vf = (t.detach().to(dtype).clone().requires_grad_(True) for t in (q, k, v))
    o = sdpa(qf, kf, vf, B, Bk, H, Nq, Nk, d, bias, dtype)
    o.backward(do.to(dtype))
    return o.detach().float(), qf.grad.float(), kf.grad.float(), vf.grad.float()


CASES = [
    # B, Bk, H, Nq, Nk, valid keys (None: no key bias), tiles per jump
    pytest.param(2, 2, 2, 1792, 1792, None, 4, id="self-N1792"),        # pipelined fwd / dQ / dK dV
    pytest.param(1, 1, 2, 7488, 7488, None, 16, id="self-N7488"),       # config X
    pytest.param(4, 1, 4, 1792, 256, 200, 1, id="cross-shared-200"),    # one-pass kernels, key bias
    pytest.param(2, 2, 4, 1792, 256, 16, 1, id="cross-16-valid"),       # config A's caption: one tile
]


@pytest.mark.parametrize("B,Bk,H,Nq,Nk,valid,jump_every", CASES)
def test_attention_large_logits(B, Bk, H, Nq, Nk, valid, jump_every):
    from ltx_amd import ops
    d = 64
    scale = d ** -0.5
    shared = Bk == 1 and B > 1
    q, k, v = make_inputs(B, Bk, H, Nq, Nk, d, jump_every, seed=Nq + Nk + H)
    do = (torch.randn(B * Nq, H * d, generator=torch.Generator(device="cpu").manual_seed(9)) * 0.5).to(DEV).bfloat16()
    bias = None
    if valid is not None:
        keep = torch.arange(Nk, device=DEV)[None, :] < valid
        bias = ((1 - keep.to(torch.bfloat16)) * -10000.0).float().expand(Bk, Nk).contiguous()
    s2 = scores_log2(q, k, B, Bk, H, Nq, Nk, d, bias)
    span = float(s2.abs().max()) * math.log(2.0) if bias is None else float(
        s2.masked_fill(s2 < -1000, 0).abs().max()) * math.log(2.0)
    assert 30.0 <= span <= 100.0, span
    if valid is None or valid > 64:  # the rescale branch must be taken in many rows
        assert rescale_share(s2) >= 0.3, rescale_share(s2)

    def run():
        o, lse = ops.attn_fwd(q, k, v, B, H, d, scale, key_bias=bias, kv_shared=shared)
        dq, dk, dv = ops.attn_bwd(q, k, v, o, do, lse, B, H, d, scale, key_bias=bias, kv_shared=shared)
        if shared:  # the kernels return per-batch dK / dV rows of the shared keys: sum them
            dk = dk.float().view(B, Nk, H * d).sum(0)
            dv = dv.float().view(B, Nk, H * d).sum(0)
        torch.cuda.synchronize()
        return o.float(), dq.float(), dk.float(), dv.float()

    ours = run()
    assert all(torch.isfinite(t).all() for t in ours)
    tau0 = None  # the TAU = 0 build is test-only (__graft_entry__.build() makes it when it can)
    if os.path.exists(TAU0_LIB):
        with library(TAU0_LIB):
            tau0 = run()
    r32 = reference(q, k, v, do, B, Bk, H, Nq, Nk, d, bias, torch.float32)
    r16 = reference(q, k, v, do, B, Bk, H, Nq, Nk, d, bias, torch.bfloat16)
    names = ("O", "dQ", "dK", "dV")
    for i, (n, a, x32, x16) in enumerate(zip(names, ours, r32, r16)):
        e_ref = rel(x16, x32)
        e = rel(a, x32)
        assert e <= 1.25 * e_ref + 1e-3, (n, e, e_ref)
        if tau0 is not None:  # without the build the comparison is reported as skipped below
            a0 = tau0[i]
            e0 = rel(a0, x32)
            assert e0 <= 1.25 * e_ref + 1e-3, (n, e0, e_ref)
            assert rel(a, a0) <= 2.0 * e_ref + 1e-3, (n, rel(a, a0), e_ref)
    if tau0 is None:
        pytest.skip("libltxhip_tau0.so not built: the fp32 checks passed, the RESCALE_TAU = 0 comparison did not run")
