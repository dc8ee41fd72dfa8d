"""Typed torch-tensor wrappers over the C ABI (one function per entry point of ltx_hip.h).

Tensors are only plumbing here: device memory, shapes, strides and the current HIP stream.
Every computation happens in libltxhip.so. 2-D operands may be strided row views (unit column
stride, any row stride that is a multiple of 8 elements), so fused buffers such as the
[M, 6144] QKV projection are consumed in place without copies.
"""
import ctypes
import os

import torch

from . import _lib
from ._lib import EPI, call

BF16 = torch.bfloat16
F32 = torch.float32


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _s():
    return _lib.stream_ptr()


def _rows(t, name):
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"{name}: expected a 2-D row-major view, got shape {tuple(t.shape)} "
                         f"strides {t.stride()}")
    return t.stride(0)


def _need(t, dtype, name):
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_cuda:
        raise _lib.LtxHipError(f"{name}: tensor is not on a ROCm device (no CPU fallback)")


# ---------------------------------------------------------------------------------------------
# patchifier / rectified flow / conditioning
# ---------------------------------------------------------------------------------------------
def patchify(latents):
    _need(latents, BF16, "patchify")
    B, C, F, H, W = latents.shape
    latents = latents.contiguous()
    out = torch.empty(B, F * H * W, C, dtype=BF16, device=latents.device)
    call("ltx_patchify_bf16", _p(latents), _p(out), B, C, F, H, W, _s())
    return out


def unpatchify(tokens, F, H, W):
    _need(tokens, BF16, "unpatchify")
    B, N, C = tokens.shape
    assert N == F * H * W
    tokens = tokens.contiguous()
    out = torch.empty(B, C, F, H, W, dtype=BF16, device=tokens.device)
    call("ltx_unpatchify_bf16", _p(tokens), _p(out), B, C, F, H, W, _s())
    return out


def latent_coords(B, F, H, W, device):
    out = torch.empty(B, 3, F * H * W, dtype=torch.int64, device=device)
    call("ltx_latent_coords", _p(out), B, F, H, W, _s())
    return out


def rf_prepare_tokens(latents, ref, pose, noise, t, want_x_t=False):
    """Fused patchify + add_noise + velocity target + conditioning lerp (train step prologue)."""
    for x, n in ((latents, "latents"), (ref, "ref"), (pose, "pose"), (noise, "noise")):
        _need(x, BF16, n)
    _need(t, F32, "t")
    B, C, F, H, W = latents.shape
    N = F * H * W
    dev = latents.device
    x_t = torch.empty(B, N, C, dtype=BF16, device=dev) if want_x_t else None
    model_in = torch.empty(B, N, C, dtype=BF16, device=dev)
    v = torch.empty(B, N, C, dtype=BF16, device=dev)
    call("ltx_rf_prepare_tokens", _p(latents.contiguous()), _p(ref.contiguous()),
         _p(pose.contiguous()), _p(noise.contiguous()), _p(t.contiguous()), _p(x_t),
         _p(model_in), _p(v), B, C, F, H, W, _s())
    return x_t, model_in, v


def rf_noise_velocity(tokens, noise, t):
    _need(tokens, BF16, "tokens")
    _need(noise, BF16, "noise")
    _need(t, F32, "t")
    B = tokens.shape[0]
    tokens = tokens.contiguous()
    x_t = torch.empty(tokens.shape, dtype=BF16, device=tokens.device)
    v = torch.empty(tokens.shape, dtype=BF16, device=tokens.device)
    call("ltx_rf_noise_velocity", _p(tokens), _p(noise.contiguous()),
         _p(t.contiguous()), _p(x_t), _p(v), B, tokens[0].numel(), _s())
    return x_t, v


def rf_noise_velocity_f32(tokens, noise, t, want_x=True, want_v=True):
    """(x_t, v) in f32, the reference scheduler's result dtype (rf.py:376-386, 400-426): tokens /
    noise bf16 or f32 [B, ...], t [B]. Returns None for the quantity not wanted."""
    for x, n in ((tokens, "tokens"), (noise, "noise")):
        if x.dtype not in (BF16, F32):
            raise TypeError(f"{n}: bf16 or f32 expected, got {x.dtype}")
        if not x.is_cuda:
            raise _lib.LtxHipError(f"{n}: tensor is not on a ROCm device (no CPU fallback)")
    if noise.shape != tokens.shape:
        raise ValueError("rf_noise_velocity_f32: tokens and noise shapes differ")
    B = tokens.shape[0]
    t = t.to(device=tokens.device, dtype=F32).reshape(-1)
    if t.numel() != B:
        raise ValueError(f"rf_noise_velocity_f32: {t.numel()} timesteps for batch {B}")
    x_t = torch.empty(tokens.shape, dtype=F32, device=tokens.device) if want_x else None
    v = torch.empty(tokens.shape, dtype=F32, device=tokens.device) if want_v else None
    call("ltx_rf_noise_velocity_f32", _p(tokens.contiguous()), 1 if tokens.dtype == F32 else 0,
         _p(noise.contiguous()), 1 if noise.dtype == F32 else 0, _p(t.contiguous()), _p(x_t), _p(v),
         B, tokens[0].numel(), _s())
    return x_t, v


def condition_lerp(tokens, ref, pose, out=None):
    """transformer3d.py:447-466 on token-major input (returns a new tensor unless out given)."""
    _need(tokens, BF16, "tokens")
    B, C, F, H, W = pose.shape
    tokens = tokens.contiguous()
    out = torch.empty(tokens.shape, dtype=BF16, device=tokens.device) if out is None else out
    call("ltx_condition_lerp", _p(tokens), _p(ref.contiguous()),
         _p(pose.contiguous()), _p(out), B, C, F, H, W, _s())
    return out


# ---------------------------------------------------------------------------------------------
# normalisation
# ---------------------------------------------------------------------------------------------
def ada_modulation(sst, tmod, scale_mask, broadcast=False):
    """sst [P,D] bf16 + tmod rows -> (mod [B,P,D], onep [B,P,D]). tmod is [B, P*D] (block AdaLN)
    or, with broadcast=True, [B, D] added to every one of the P rows (output head)."""
    P, D = sst.shape
    B = tmod.shape[0]
    ld = _rows(tmod, "tmod")
    out = torch.empty(B, P, D, dtype=BF16, device=sst.device)
    onep = torch.empty(B, P, D, dtype=BF16, device=sst.device)
    call("ltx_ada_modulation", _p(sst.contiguous()), _p(tmod), ld, 0 if broadcast else D, _p(out),
         _p(onep), B, P, D, scale_mask, _s())
    return out, onep


def gate_mul(dy, gate, rows_per_batch):
    """bf16(dy * gate[m // rows_per_batch]); gate is a [B, D] row view."""
    M, D = dy.shape
    dy = dy.contiguous()
    out = torch.empty(M, D, dtype=BF16, device=dy.device)
    call("ltx_gate_mul_bf16", _p(dy), _p(gate), _rows(gate, "gate"), _p(out), M, D, rows_per_batch,
         _s())
    return out


def _dense(t, name):
    if not t.is_contiguous():
        raise ValueError(f"{name}: expected a dense [M, D] tensor")
    return t


def rmsnorm_modulate_fwd(x, shift, onep, ld_mod, rows_per_batch, eps, out=None):
    M, D = _dense(x, "x").shape
    y = torch.empty(M, D, dtype=BF16, device=x.device) if out is None else out
    rstd = torch.empty(M, dtype=F32, device=x.device)
    call("ltx_rmsnorm_modulate_fwd", _p(x), _p(shift), _p(onep), ld_mod, _p(y), _p(rstd), M, D,
         rows_per_batch, eps, _s())
    return y, rstd


def rmsnorm_modulate_bwd(dy, x, rstd, onep, ld_mod, rows_per_batch, dres=None, out=None,
                         gate=None):
    """dx (= dres + the norm/modulate backward). gate (a [B, D] row view): also returns
    gate_mul(dx, gate, rows_per_batch), bitwise, from the same pass (ltx_rmsnorm_modulate_bwd_gated)."""
    M, D = _dense(x, "x").shape
    _dense(dy, "dy")
    dx = torch.empty(M, D, dtype=BF16, device=x.device) if out is None else out
    if gate is None:
        call("ltx_rmsnorm_modulate_bwd", _p(dy), _p(x), _p(rstd), _p(onep), ld_mod, _p(dres),
             _p(dx), M, D, rows_per_batch, _s())
        return dx
    gout = torch.empty(M, D, dtype=BF16, device=x.device)
    call("ltx_rmsnorm_modulate_bwd_gated", _p(dy), _p(x), _p(rstd), _p(onep), ld_mod, _p(dres),
         _p(dx), M, D, rows_per_batch, _p(gate), _rows(gate, "gate"), _p(gout), _s())
    return dx, gout


def layernorm_modulate_fwd(x, shift, onep, ld_mod, rows_per_batch, eps):
    M, D = _dense(x, "x").shape
    y = torch.empty(M, D, dtype=BF16, device=x.device)
    mean = torch.empty(M, dtype=F32, device=x.device)
    rstd = torch.empty(M, dtype=F32, device=x.device)
    call("ltx_layernorm_modulate_fwd", _p(x), _p(shift), _p(onep), ld_mod, _p(y), _p(mean),
         _p(rstd), M, D, rows_per_batch, eps, _s())
    return y, mean, rstd


def layernorm_modulate_bwd(dy, x, mean, rstd, onep, ld_mod, rows_per_batch):
    M, D = _dense(x, "x").shape
    _dense(dy, "dy")
    dx = torch.empty(M, D, dtype=BF16, device=x.device)
    call("ltx_layernorm_modulate_bwd", _p(dy), _p(x), _p(mean), _p(rstd), _p(onep), ld_mod,
         _p(dx), M, D, rows_per_batch, _s())
    return dx


_ROPE_OMEGA = {}  # (dim, theta, device) -> the f32 device frequency vector


class RopeSpec:
    """Per-forward RoPE state: the bf16 cos/sin table of precompute_freqs_cis
    (transformer3d.py:209-277), built once on the device by ltx_rope_table and read by every
    block's q/k kernels, forward and backward.

    ``omega`` is computed exactly as the reference does (transformer3d.py:231-250):
    ``theta ** linspace(log(1,theta), log(theta,theta), dim//6) * pi / 2`` in f32 -- a 341-entry
    constant, computed on the host. When ``indices_grid`` is a batch-broadcast view (stride 0 on
    dim 0, as train_step passes it), one table serves every batch (cs_batch_rows = 0)."""

    def __init__(self, indices_grid, dim, theta, max_pos):
        import math
        self.B, _, self.N = indices_grid.shape
        self.D = dim
        shared = self.B > 1 and indices_grid.stride(0) == 0
        grid = (indices_grid[:1] if shared else indices_grid).contiguous()
        self.is_float = 0 if grid.dtype == torch.int64 else 1
        if self.is_float and grid.dtype != F32:
            grid = grid.to(F32)
        self.grid = grid
        # the frequency vector is built on the host once per (dim, theta, device): a blocking
        # H2D copy per forward would drain the device queue (PyTorch syncs the stream after it)
        key = (dim, float(theta), str(indices_grid.device))
        omega = _ROPE_OMEGA.get(key)
        if omega is None:
            idx = theta ** torch.linspace(math.log(1, theta), math.log(theta, theta), dim // 6,
                                          dtype=torch.float32)
            idx = idx.to(torch.float32) * math.pi / 2
            omega = _ROPE_OMEGA[key] = idx.to(indices_grid.device)
        self.omega = omega
        self.max_pos = [float(m) for m in max_pos]
        bt = grid.shape[0]
        self.cs_batch_rows = 0 if shared else self.N
        self.cs = torch.empty(bt * self.N, dim // 2, dtype=torch.int32, device=indices_grid.device)
        call("ltx_rope_table", _p(grid), self.is_float, bt, self.N, dim, _p(self.omega),
             self.max_pos[0], self.max_pos[1], self.max_pos[2], _p(self.cs), _s())


class RopePair:
    """RoPE state from the reference's own (cos, sin) pair (precompute_freqs_cis's return value,
    transformer3d.py:270-277: bf16 [B, N, D], each value repeated for the element pair 2i, 2i+1),
    packed by ltx_rope_pack_bf16 into the ltx_rope_table layout: what the Attention.set_processor
    plug-in receives as freqs_cis (attention.py:1010-1012). A batch-broadcast pair (stride 0 on
    dim 0) packs one batch shared by all (cs_batch_rows = 0)."""

    def __init__(self, cos, sin):
        if cos.shape != sin.shape or cos.dim() != 3:
            raise ValueError(f"freqs_cis: (cos, sin) of equal [B, N, D] shape expected, got "
                             f"{tuple(cos.shape)} / {tuple(sin.shape)}")
        _need(cos, BF16, "freqs_cis cos")
        _need(sin, BF16, "freqs_cis sin")
        self.B, self.N, self.D = cos.shape
        shared = self.B > 1 and cos.stride(0) == 0 and sin.stride(0) == 0
        c = (cos[:1] if shared else cos).reshape(-1, self.D).contiguous()
        s = (sin[:1] if shared else sin).reshape(-1, self.D).contiguous()
        self.cs_batch_rows = 0 if shared else self.N
        self.cs = torch.empty(c.shape[0], self.D // 2, dtype=torch.int32, device=cos.device)
        call("ltx_rope_pack_bf16", _p(c), _p(s), self.D, c.shape[0], self.D, _p(self.cs), _s())


def qk_norm_rope_fwd(q_in, k_in, q_w, k_w, rope: RopeSpec = None, B=None, N=None, eps=1e-5,
                     q_out=None, k_out=None):
    """q_in/k_in [M,D] row views -> (q_out, k_out, rstd_q, rstd_k). k_in may be None."""
    M, D = q_in.shape
    dev = q_in.device
    q_out = torch.empty(M, D, dtype=BF16, device=dev) if q_out is None else q_out
    rq = torch.empty(M, dtype=F32, device=dev)
    rk = None
    if k_in is not None:
        k_out = torch.empty(M, D, dtype=BF16, device=dev) if k_out is None else k_out
        rk = torch.empty(M, dtype=F32, device=dev)
    if rope is not None:
        B, N = rope.B, rope.N
    assert B * N == M
    call("ltx_qk_norm_rope_fwd", _p(q_in), _rows(q_in, "q_in"), _p(k_in),
         _rows(k_in, "k_in") if k_in is not None else 0, _p(q_out), _rows(q_out, "q_out"),
         _p(k_out), _rows(k_out, "k_out") if k_in is not None else 0, _p(q_w), _p(k_w), _p(rq),
         _p(rk), _p(rope.cs) if rope else None, rope.cs_batch_rows if rope else 0, B, N, D,
         1 if rope else 0, eps, _s())
    return q_out, (k_out if k_in is not None else None), rq, rk


def qk_norm_rope_bwd(dq, q_raw, q_w, rq, dk=None, k_raw=None, k_w=None, rk=None,
                     rope: RopeSpec = None, B=None, N=None, dq_out=None, dk_out=None):
    M, D = q_raw.shape
    dev = q_raw.device
    dq_out = torch.empty(M, D, dtype=BF16, device=dev) if dq_out is None else dq_out
    if dk is not None and dk_out is None:
        dk_out = torch.empty(M, D, dtype=BF16, device=dev)
    if rope is not None:
        B, N = rope.B, rope.N
    call("ltx_qk_norm_rope_bwd", _p(dq), _rows(dq, "dq"), 1 if dq.dtype == F32 else 0, _p(dk),
         _rows(dk, "dk") if dk is not None else 0,
         1 if (dk is not None and dk.dtype == F32) else 0, _p(q_raw), _rows(q_raw, "q_raw"),
         _p(k_raw), _rows(k_raw, "k_raw") if k_raw is not None else 0, _p(q_w), _p(k_w), _p(rq),
         _p(rk), _p(dq_out), _rows(dq_out, "dq_out"), _p(dk_out),
         _rows(dk_out, "dk_out") if dk is not None else 0, _p(rope.cs) if rope else None,
         rope.cs_batch_rows if rope else 0, B, N, D, 1 if rope else 0, _s())
    return dq_out, (dk_out if dk is not None else None)


def qk_norm_fwd_grouped(x, x_gs, weights, eps=1e-5):
    """The attn2 k_norm of every block's text keys in one launch (ltx_qk_norm_fwd_grouped):
    group g is the [rows, D] view starting x_gs elements after x's first element (row stride
    x.stride(0)), normalised with weights[g]. Returns y [G, rows, D] bf16 and rstd [G, rows] f32,
    bitwise the per-group qk_norm_rope_fwd(x_g, None, weights[g], ...) calls."""
    G, D = weights.shape
    rows = x.shape[0]
    _need(weights, BF16, "weights")
    assert weights.is_contiguous() and x.shape[1] >= D and x_gs >= 0
    # group G-1's last row must lie inside x (the C entry checks alignment, not extents)
    assert x.numel() >= (G - 1) * x_gs + (rows - 1) * x.stride(0) + D, "x too small for G groups"
    y = torch.empty(G, rows, D, dtype=BF16, device=x.device)
    rstd = torch.empty(G, rows, dtype=F32, device=x.device)
    call("ltx_qk_norm_fwd_grouped", _p(x), _rows(x, "x"), x_gs, _p(y), D, rows * D, _p(weights), D,
         _p(rstd), rows, rows, G, D, eps, _s())
    return y, rstd


def qk_norm_bwd_grouped(dy, dy_gs, x, x_gs, weights, rstd, dx, dx_gs):
    """Backward of qk_norm_fwd_grouped: group g's incoming gradient is the [rows, D] view of the
    2-D dy starting g * dy_gs elements in (row stride dy.stride(0)); its input gradient goes to
    the view of dx starting g * dx_gs elements in. dx may be dy (in place: each row is read whole
    before it is written)."""
    G, D = weights.shape
    rows = x.shape[0]
    assert weights.is_contiguous() and rstd.is_contiguous()
    assert rstd.shape == (G, rows) and dx.shape[0] == rows
    assert dy.numel() >= (G - 1) * dy_gs + (rows - 1) * dy.stride(0) + D
    assert x.numel() >= (G - 1) * x_gs + (rows - 1) * x.stride(0) + D, "x too small for G groups"
    assert dx.numel() >= (G - 1) * dx_gs + (rows - 1) * dx.stride(0) + D, "dx too small for G groups"
    assert min(dy_gs, x_gs, dx_gs) >= 0
    call("ltx_qk_norm_bwd_grouped", _p(dy), _rows(dy, "dy"), dy_gs, _p(x), _rows(x, "x"), x_gs,
         _p(weights), D, _p(rstd), rows, _p(dx), _rows(dx, "dx"), dx_gs, rows, G, D, _s())
    return dx


# ---------------------------------------------------------------------------------------------
# attention
# ---------------------------------------------------------------------------------------------
def _env_on(var):
    """A/B switch the library reads per call (attention_pipe.hip): unset or non-zero = on."""
    v = os.environ.get(var)
    return v is None or v.strip() not in ("0", "")


_ATTN_ENV = ("LTX_ATTN_XCD", "LTX_ATTN_BWD1", "LTX_ATTN_W8", "LTX_ATTN_SKIP", "LTX_ATTN_FWD1",
             "LTX_ATTN_BWD1_QS", "LTX_ATTN_BWD1_FEW", "LTX_ATTN_QSPLIT", "LTX_ATTN_DKDV_W1",
             "LTX_ATTN_DQ_W1", "LTX_ATTN_DQ_PIPE", "LTX_ATTN_DQ_NBUF", "LTX_ATTN_FWD_W1",
             "LTX_ATTN_FWD_PIPE", "LTX_ATTN_FWD_F32SUM", "LTX_ATTN_DKDV_PIPE", "LTX_ATTN_DKDV_NBUF",
             "LTX_ATTN_FWD1_ROWS")
_attn_env_seen = [None]


def _attn_env_sync():
    """The library reads its LTX_ATTN_* switches once (attention_common.h AttnSwitches); when this
    process changed one since the last attention call (an A/B test), have it read them again."""
    cur = tuple(os.environ.get(k) for k in _ATTN_ENV)
    if cur != _attn_env_seen[0]:
        call("ltx_attn_reload_switches")
        _attn_env_seen[0] = cur


def attn_fwd(q, k, v, B, H, d, scale, key_bias=None, out=None, kv_shared=False):
    """q [B*Nq, >=H*d] row view, k/v [B*Nk, ...] -> (o [B*Nq, H*d], lse [B,H,Nq] f32 log2).
    kv_shared: k/v/key_bias hold ONE batch ([Nk, ...], [1, Nk]) attended by every query batch."""
    Nq = q.shape[0] // B
    Nk = k.shape[0] if kv_shared else k.shape[0] // B
    _attn_env_sync()
    _gemm_workspace(q.device)  # split-query partials / diagnostic stamps use the stream's workspace
    o = torch.empty(B * Nq, H * d, dtype=BF16, device=q.device) if out is None else out
    lse = torch.empty(B, H, Nq, dtype=F32, device=q.device)
    bias = "true" if (key_bias is not None or Nk % 64) else "false"
    if d == 64 and Nk <= 256 and os.environ.get("LTX_ATTN_FWD1", "1") != "0":
        label = f"attention forward: ltx::attn_fwd1_kernel<{d}, {bias}>"  # K/V staged once
    elif d == 64 and bias == "false" and _env_on("LTX_ATTN_FWD_PIPE"):  # attention_pipe.hip
        f32sum = "false" if os.environ.get("LTX_ATTN_FWD_F32SUM", "1")[:1] == "0" else "true"
        label = f"attention forward: ltx::attn_fwd_pipe_kernel<{f32sum}>"
    elif d == 64 and int(os.environ.get("LTX_ATTN_W8", "1")) & 1:  # 8 waves x 32 queries
        label = f"attention forward: ltx::attn_q_kernel<{d}, 0, {bias}, 8>"
    else:
        label = f"attention forward: ltx::attn_q_kernel<{d}, 0, {bias}, 4>"
    timer = _timer if (_timer is not None and _timer.wants(label)) else None
    ev0 = timer.start() if timer is not None else None
    call("ltx_attn_fwd", _p(q), _rows(q, "q"), _p(k), _rows(k, "k"), _p(v), _rows(v, "v"), _p(o),
         _rows(o, "o"), _p(lse), _p(key_bias), B, H, Nq, Nk, 0 if kv_shared else Nk, d, scale, _s())
    if timer is not None:
        bk = 1 if kv_shared else B  # q, k, v read once, o + lse written once
        timer.stop(label, 4.0 * B * H * Nq * Nk * d, ev0, 2.0 * H * d * (2 * B * Nq + 2 * bk * Nk) + 4.0 * B * H * Nq)
    return o, lse


def attn_bwd(q, k, v, o, do, lse, B, H, d, scale, key_bias=None, dq_f32=False, dq=None,
             dk=None, dv=None, kv_shared=False, delta=None):
    """Gradients (dq [B*Nq], dk/dv [B*Nk] per query batch -- with kv_shared their batch_sum is
    the gradient of the shared rows). delta: the f32 [B, H, Nq] rowsum(dO*O), when the GEMM that
    produced dO already wrote it (gemm epilogue 'store_rowdot'); else the delta pass runs here."""
    Nq = q.shape[0] // B
    Nk = k.shape[0] if kv_shared else k.shape[0] // B
    dev = q.device
    _attn_env_sync()
    _gemm_workspace(dev)  # split-query / few-key partials live in the stream's workspace
    dq = torch.empty(B * Nq, H * d, dtype=F32 if dq_f32 else BF16, device=dev) if dq is None else dq
    dk = torch.empty(B * Nk, H * d, dtype=BF16, device=dev) if dk is None else dk
    dv = torch.empty(B * Nk, H * d, dtype=BF16, device=dev) if dv is None else dv
    ready = delta is not None
    if ready:
        assert delta.dtype == F32 and delta.is_contiguous() and delta.numel() == B * H * Nq
    else:
        delta = torch.empty(B, H, Nq, dtype=F32, device=dev)
    bias = "true" if key_bias is not None else "false"
    if d == 64 and Nk <= 256 and os.environ.get("LTX_ATTN_BWD1", "1") != "0":
        # every key in one workgroup: the one-pass kernel (attention.hip attn_bwd1_kernel)
        # the name rocprofv3 prints: <d, biased, query-split>, the split read from the same switch
        # the library reads (attention.hip bwd1_qs_flag: on only with LTX_ATTN_BWD1_QS=1)
        biased = key_bias is not None or Nk != 256
        qs = "true" if (biased and os.environ.get("LTX_ATTN_BWD1_QS", "0") == "1") else "false"
        kern = f"ltx::attn_bwd1_kernel<{d}, {'true' if biased else 'false'}, {qs}>"
    elif d == 64 and _env_on("LTX_ATTN_DKDV_PIPE"):  # the pipelined kernels (attention_pipe.hip)
        kb = "true" if (key_bias is not None or Nk % 64) else "false"
        # LDS buffers of the pipelined kernels (attention_pipe.hip dq_nbuf / dkdv_nbuf: 4 unless "3")
        nq = "3" if os.environ.get("LTX_ATTN_DQ_NBUF", "4")[:1] == "3" else "4"
        nk = "3" if os.environ.get("LTX_ATTN_DKDV_NBUF", "4")[:1] == "3" else "4"
        # one wave per SIMD, hand-scheduled loops (attention_pipe.hip): LTX_ATTN_DQ_W1 /
        # LTX_ATTN_DKDV_W1 = 2 (default) the persistent kernels, 1 one workgroup per block
        dq_mode = os.environ.get("LTX_ATTN_DQ_W1", "2").strip() or "2"
        dk_mode = os.environ.get("LTX_ATTN_DKDV_W1", "2").strip() or "2"
        if kb == "false" and dq_mode[:1] != "0":
            dqk = ("ltx::attn_dq_w1p_kernel<0>" if dq_mode == "2" and dq.dtype != F32
                   else "ltx::attn_dq_w1_kernel<0>")
        else:
            dqk = (f"ltx::attn_dq_pipe_kernel<{nq}>" if kb == "false" and _env_on("LTX_ATTN_DQ_PIPE")
                   else f"ltx::attn_q_kernel<{d}, 1, {kb}, 4>")
        if kb == "false" and dk_mode != "0":
            dkk = "ltx::attn_dkdv_w1p_kernel<0>" if dk_mode == "2" else "ltx::attn_dkdv_w1_kernel<0>"
            kern = f"{dkk} + {dqk}"
        else:
            kern = f"ltx::attn_dkdv_pipe_kernel<{kb}, {nk}> + {dqk}"
    else:
        kern = f"ltx::attn_dkdv_kernel<{d}, {bias}, 4> + ltx::attn_q_kernel<{d}, 1, {bias}, 4>"
    label = ("attention backward: " + ("" if ready else f"ltx::attn_delta_kernel<{d}> + ") + kern)
    timer = _timer if (_timer is not None and _timer.wants(label)) else None
    ev0 = timer.start() if timer is not None else None
    call("ltx_attn_bwd_ex", _p(q), _rows(q, "q"), _p(k), _rows(k, "k"), _p(v), _rows(v, "v"),
         _p(o), _rows(o, "o") if o is not None else 0, _p(do), _rows(do, "do"), _p(lse),
         _p(key_bias), _p(delta), 1 if ready else 0, _p(dq), _rows(dq, "dq"),
         1 if dq.dtype == F32 else 0, _p(dk), _rows(dk, "dk"), _p(dv), _rows(dv, "dv"), B, H, Nq,
         Nk, 0 if kv_shared else Nk, d, scale, _s())
    if timer is not None:
        bk = 1 if kv_shared else B  # q, do, k, v, lse, delta read once; dq, dk, dv written once
        nb = 2.0 * H * d * (3 * B * Nq + 2 * bk * Nk + 2 * B * Nk) + 8.0 * B * H * Nq
        timer.stop(label, 8.0 * B * H * Nq * Nk * d, ev0, nb)
    return dq, dk, dv


def batch_sum(x, B, out=None):
    """x [B*rows, cols] bf16 -> [rows, cols]: sum over the batch (f32 accumulation)."""
    rows = x.shape[0] // B
    cols = x.shape[1]
    out = torch.empty(rows, cols, dtype=BF16, device=x.device) if out is None else out
    call("ltx_batch_sum_bf16", _p(x), _rows(x, "x"), B, rows, cols, _p(out), _rows(out, "out"), _s())
    return out


# ---------------------------------------------------------------------------------------------
# GEMM + LoRA
# ---------------------------------------------------------------------------------------------
class LaunchTimer:
    """bench.py's live per-kernel timing: HIP events recorded on the launch stream around every
    GEMM and attention launch while installed (set_launch_timer), each tagged with the kernel
    rocprofv3 names for it (GEMMs: ltx_gemm_describe, the dispatcher's own choice) and the
    launch's ALGORITHMIC FLOPs (GEMM 2*M*N*K without the LoRA K-extension; attention forward
    4*B*H*Nq*Nk*d, backward twice that -- SURVEY 8d, no recompute) and ALGORITHMIC bytes (every
    operand read once and every output written once at its stored dtype: for a GEMM
    2*(M*K + N*K + M*N) + its epilogue's aux rows and K-extension tiles)."""

    def __init__(self, only=None):
        self.records = []  # (label, flops, bytes, ev0, ev1)
        self.only = only   # time only the launches of this label (None: every launch)

    def start(self):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def stop(self, label, flops, ev0, nbytes=0.0):
        ev1 = torch.cuda.Event(enable_timing=True)
        ev1.record()
        self.records.append((label, float(flops), float(nbytes), ev0, ev1))

    def wants(self, label):
        return self.only is None or self.only == label

    def summary(self):
        """[{kernel, launches, ms, flops, bytes}] per label, largest total time first."""
        torch.cuda.synchronize()
        agg = {}
        for label, flops, nbytes, a, b in self.records:
            e = agg.setdefault(label, {"kernel": label, "launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0})
            e["launches"] += 1
            e["ms"] += a.elapsed_time(b)
            e["flops"] += flops
            e["bytes"] += nbytes
        return sorted(agg.values(), key=lambda e: -e["ms"])


_timer = None


def set_launch_timer(timer):
    global _timer
    _timer = timer


_GEMM_NAMES = {}


def gemm_kernel_name(M, N, K, K2, epilogue, rank=0):
    """The kernel ltx_gemm_bf16_nt_ext launches for this call on the current stream."""
    key = (M, N, K, K2, epilogue, rank, _s().value)
    if key not in _GEMM_NAMES:
        buf = ctypes.create_string_buffer(256)
        call("ltx_gemm_describe", M, N, K, K2, EPI[epilogue], rank, _s(), buf, 256)
        _GEMM_NAMES[key] = buf.value.decode()
    return _GEMM_NAMES[key]


_GEMM_WS = {}
GEMM_WS_BYTES = 128 << 20  # split-K partials: S x M x N f32 (S=4 at 2048 x 2048 = 64 MiB)


def _gemm_workspace(device):
    """The split-K workspace of the current stream, handed to the library once per (device,
    stream) (caller-owned memory): the default stream's doubles as the library default, other
    streams (the text side stream) get their own, so concurrent GEMMs never share partials."""
    stream = _s()
    key = (str(device), stream.value)
    if key not in _GEMM_WS:
        ws = torch.empty(GEMM_WS_BYTES // 4, dtype=F32, device=device)
        if not any(k[0] == key[0] for k in _GEMM_WS):
            call("ltx_gemm_set_workspace", _p(ws), GEMM_WS_BYTES)
        call("ltx_gemm_set_stream_workspace", stream, _p(ws), GEMM_WS_BYTES)
        _GEMM_WS[key] = ws
    return _GEMM_WS[key]


def gemm(a, w, bias=None, epilogue="store", out=None, aux0=None, aux1=None, aux2=None,
         alpha=1.0, rank=0, rows_per_batch=0, ext=None, ext_group=None):
    """out[M,N] = epilogue(a[M,K] . w[N,K]^T (+ bias) [+ a2 . w2^T]); see LTX_EPI_* in ltx_hip.h.
    ext = (a2 [M,K2], w2 [N,K2]) appends K-extension tiles (the fused LoRA branch).
    ext_group = (G, stride): output columns [g*G, (g+1)*G) read a2 from column g*stride on
    (ltx_gemm_bf16_nt_gext: one launch for many LoRA-carrying projections of one input)."""
    _need(a, BF16, "gemm a")
    _need(w, BF16, "gemm w")
    _gemm_workspace(a.device)
    M, K = a.shape
    N, K2 = w.shape
    if K != K2:
        raise ValueError(f"gemm: K mismatch {K} vs {K2}")
    out = torch.empty(M, N, dtype=BF16, device=a.device) if out is None else out
    ld0 = _rows(aux0, "aux0") if aux0 is not None else 0
    if epilogue in ("gelu", "gelu_bwd") and aux0 is not None:  # the GELU derivative, int16 snorm
        _need(aux0, torch.int16, f"gemm {epilogue} aux0 (int16 snorm of gelu_tanh' / 2)")
    if epilogue == "store_rowdot":  # aux1: the dense f32 [B, N / head_dim, rows_per_batch] delta
        _need(aux1, F32, "gemm store_rowdot delta")
        if not aux1.is_contiguous() or aux1.numel() != M * (N // max(rank, 1)):
            raise ValueError("gemm store_rowdot: delta must be a dense [B, N/head_dim, rows] f32")
        ld1 = 0
    else:
        ld1 = _rows(aux1, "aux1") if aux1 is not None else 0
    ld2 = _rows(aux2, "aux2") if aux2 is not None else 0
    a2, w2 = ext if ext is not None else (None, None)
    K2 = w2.shape[1] if w2 is not None else 0
    gcols, gstride = ext_group if ext_group is not None else (0, 0)
    timer = _timer
    if timer is not None:
        label = gemm_kernel_name(M, N, K, K2, epilogue, rank)
        timer = timer if timer.wants(label) else None
    ev0 = timer.start() if timer is not None else None
    call("ltx_gemm_bf16_nt_gext", _p(a), _rows(a, "a"), _p(w), _rows(w, "w"), _p(a2),
         _rows(a2, "a2") if a2 is not None else 0, _p(w2), _rows(w2, "w2") if w2 is not None else 0,
         K2, gcols, gstride, _p(out), _rows(out, "out"), M, N, K, EPI[epilogue], _p(bias),
         _p(aux0), ld0, _p(aux1), ld1, _p(aux2), ld2, float(alpha), rank, rows_per_batch, _s())
    if timer is not None:
        timer.stop(label, 2.0 * M * N * K, ev0, gemm_algorithmic_bytes(M, N, K, K2, epilogue, aux0 is not None,
                                                                       aux2 is not None))
    return out


_AUX_ROW_READ = {"gated_residual", "gelu_bwd", "accum", "store_rowdot", "lora_residual"}


GELU_Q = 32767.0 / 2.0  # the GELU epilogue's derivative store: int16 q = rint(GELU_Q * gelu_tanh'(y))


def gelu_grad_q(y):
    """the GELU epilogue's aux0 for a pre-activation y (torch statement of what the kernel stores):
    int16 rint(32767 * clamp(gelu_tanh'(y) / 2, -1, 1)); the backward multiplies by q / GELU_Q"""
    d = torch.ops.aten.gelu_backward(torch.ones_like(y, dtype=torch.float32), y.float(), approximate="tanh")
    return torch.round((d * 0.5).clamp(-1, 1) * 32767.0).to(torch.int16)


def gemm_algorithmic_bytes(M, N, K, K2, epilogue, has_aux0, has_aux2):
    """Bytes one ltx_gemm launch must move at minimum: A, W (and the K-extension A2, W2) read once,
    C written once, plus the epilogue's [M, N] 2-byte aux rows (residual / GELU derivative /
    accumulator / attention output for delta) read or written once."""
    b = 2.0 * (M * K + N * K + M * N) + 2.0 * (M + N) * K2
    if epilogue in _AUX_ROW_READ or (epilogue == "lora_dgrad_accum" and has_aux0):
        b += 2.0 * M * N
    if (epilogue == "gelu" and has_aux0) or (epilogue in ("gated_residual", "accum") and has_aux2):
        b += 2.0 * M * N  # GELU-derivative / pre-gate store, or the accumulate's gated copy
    return b


_LORA_ROWS = os.environ.get("LTX_LORA_ROWS", "1") != "0"  # A/B switch: 0 = the f32 kernel only


def lora_down(x, wr, alpha=1.0, transposed=False, out=None, split=False, split_out=None,
              groups=1, group_strides=(0, 0, 0, 0), pieces=None):
    """out[m,j] = alpha * x[m,:] . Wr[j,:]; Wr = lora_A [r,K]; transposed=True takes lora_B [K,r]
    (i.e. uses B^T) for the dgrad w = s * dY . B. split=True also returns the activation
    K-extension operand of the rows (what lora_split(out, "act") makes), written by the same
    kernel. groups > 1 runs `groups` adapters in one launch (ltx_lora_down_grouped): wr is the
    first adapter, group_strides = element offsets per group of (x, wr, out, split); the caller
    passes out (and split_out) covering every group. pieces = lora_pieces(wr, transposed) (the
    caller's cache) routes token-sized calls to the bf16-matrix-core kernel (ltx_lora_rows); a
    callable is invoked only when that route is taken (the pieces are built lazily)."""
    M, K = x.shape
    if pieces is not None and _LORA_ROWS and groups == 1 and M >= 8192 and K % 256 == 0:
        pieces = pieces() if callable(pieces) else pieces
        return lora_rows(x, pieces, wr.shape[1] if transposed else wr.shape[0], alpha=alpha,
                         out=out, split=split, split_out=split_out)
    if transposed:
        r = wr.shape[1]
        wj, wk = 1, wr.stride(0)
    else:
        r = wr.shape[0]
        wj, wk = wr.stride(0), 1
    if groups > 1 and (out is None or (split and split_out is None)):
        raise ValueError("lora_down: grouped calls write into caller-provided out / split_out")
    out = torch.empty(M, r, dtype=F32, device=x.device) if out is None else out
    sp, K2, lds = None, 0, 0
    if split:  # split_out: a [M, K2] column block of a wider operand (the merged text K/V GEMMs)
        K2 = lora_k2(r)
        sp = torch.empty(M, K2, dtype=BF16, device=x.device) if split_out is None else split_out
        lds = _rows(sp, "split_out")
    gx, gw, go, gs = group_strides
    call("ltx_lora_down_grouped", _p(x), _rows(x, "x"), _p(wr), wj, wk, _p(out), _rows(out, "out"),
         M, K, r, float(alpha), _p(sp), lds, K2, groups, gx, gw, go, gs, _s())
    return (out, sp) if split else out


def lora_pieces(wr, transposed=False, out=None):
    """bf16 [3*RP, K] pieces (hi, mid, lo) of lora_A [r, K] (or of B^T for lora_B [K, r] with
    transposed=True): the weight operand of lora_rows."""
    if transposed:
        K, r = wr.shape
        rs, cs = wr.stride(1), wr.stride(0)
    else:
        r, K = wr.shape
        rs, cs = wr.stride(0), wr.stride(1)
    RP = max(r, 16)
    out = torch.empty(3 * RP, K, dtype=BF16, device=wr.device) if out is None else out
    call("ltx_lora_pieces", _p(wr), rs, cs, r, K, _p(out), _rows(out, "out"), _s())
    return out


def lora_rows(x, w3, r, alpha=1.0, out=None, split=False, split_out=None):
    """lora_down for token-sized M from the weight's lora_pieces (ltx_lora_rows)."""
    M, K = x.shape
    out = torch.empty(M, r, dtype=F32, device=x.device) if out is None else out
    sp, K2, lds = None, 0, 0
    if split:
        K2 = lora_k2(r)
        sp = torch.empty(M, K2, dtype=BF16, device=x.device) if split_out is None else split_out
        lds = _rows(sp, "split_out")
    _gemm_workspace(x.device)  # token-sized calls keep column-split partials in the workspace
    call("ltx_lora_rows", _p(x), _rows(x, "x"), _p(w3), _rows(w3, "w3"), _p(out), _rows(out, "out"),
         M, K, r, float(alpha), _p(sp), lds, K2, _s())
    return (out, sp) if split else out


_WEIGHT_GENERATION = [0]


def weight_generation():
    """Counter bumped by every FusedAdamW step: its kernel updates parameters in place without
    touching torch's version counters, so caches keyed on weights (LoRA operand splits) also
    key on this."""
    return _WEIGHT_GENERATION[0]


def bump_weight_generation():
    _WEIGHT_GENERATION[0] += 1


def lora_k2(r):
    return (3 * r + 63) // 64 * 64


def lora_split(src, role, scale=1.0, transposed=False, out=None):
    """K-extension operand from an f32 [R, r] matrix (transposed=True reads src as [r, R], e.g.
    lora_A [r, K] used as A^T): role 'act' -> rows [hi|hi|lo|0], 'weight' -> [hi|lo|hi|0]."""
    if transposed:
        r, R = src.shape
        rs, cs = src.stride(1), src.stride(0)
    else:
        R, r = src.shape
        rs, cs = src.stride(0), src.stride(1)
    K2 = lora_k2(r)
    out = torch.empty(R, K2, dtype=BF16, device=src.device) if out is None else out
    call("ltx_lora_split_bf16", _p(src), rs, cs, float(scale), R, r, 0 if role == "act" else 1,
         _p(out), _rows(out, "out"), K2, _s())
    return out


def lora_wgrad(y, u, alpha=1.0, transpose_out=False, out=None, accumulate=False, groups=1,
               group_strides=(0, 0)):
    """dW[n,j] = alpha * sum_m y[m,n] u[m,j] -> [N,r] (or [r,N] when transpose_out). With
    out/accumulate the product is added into an existing dense f32 buffer (e.g. p.grad).
    groups > 1 (ltx_lora_wgrad_grouped): out is a dense [groups, N, r] (or [groups, r, N]) stack,
    y / u are the first group's operands, group_strides = element offsets per group of (y, u)."""
    M, N = y.shape
    r = u.shape[1]
    shape = (r, N) if transpose_out else (N, r)
    if groups > 1:
        shape = (groups,) + shape
    if out is None:
        out = torch.empty(shape, dtype=F32, device=y.device)
        accumulate = False
    assert tuple(out.shape) == shape and out.dtype == F32 and out.is_contiguous()
    on, oj = (1, N) if transpose_out else (r, 1)
    gy, gu = group_strides
    _gemm_workspace(y.device)  # the row-split partials live in the stream's workspace
    call("ltx_lora_wgrad_grouped", _p(y), _rows(y, "y"), _p(u), _rows(u, "u"), _p(out), on, oj, M,
         N, r, float(alpha), 1 if accumulate else 0, groups, gy, gu, N * r, _s())
    return out


def lora_dy_enabled():
    """LTX_LORA_DY=0 (read per call): the backward keeps ltx_lora_wgrad + ltx_lora_rows on dY."""
    return os.environ.get("LTX_LORA_DY", "1") != "0"


def lora_dy_da_enabled():
    """LTX_LORA_DY_DA=0 (read per call): the adapter's dA stays a separate ltx_lora_wgrad call."""
    return os.environ.get("LTX_LORA_DY_DA", "1") != "0"


def lora_dy_da_fits(y, x, r):
    """lora_dy(y, ..., x=x) applies (and LTX_LORA_DY_DA is not 0). Only at M >= 2048, where
    ltx_lora_wgrad takes the same token-sized path, so the merged call is bitwise the separate ones
    (below it ltx_lora_wgrad runs the f32-MFMA kernel: another rounding of dA)."""
    return (lora_dy_da_enabled() and lora_dy_fits(x, r) and y.shape[1] <= 2048 and x.shape[0] == y.shape[0]
            and y.shape[0] >= 2048)


def lora_dy_fits(y, r):
    M, N = y.shape
    return r in (8, 16) and M % 32 == 0 and N % 512 == 0 and y.stride(1) == 1 and y.stride(0) % 8 == 0


def lora_dy(y, u, w3, r, alpha, dB_out, accumulate=True, transpose_out=False, x=None, dA_out=None,
            dA_accumulate=True):
    """One pass over dY (ltx_lora_dy): returns (w, split) as lora_down(y, B, transposed=True,
    split=True) does, and adds alpha * y^T . u into dB_out ([N, r], or [r, N] with transpose_out)
    as lora_wgrad(y, u, alpha, out=dB_out, accumulate=accumulate) does. With x ([M, K] bf16,
    lora_dy_fits; N <= 2048) and dA_out ([r, K] f32): also dA_out (+)= x^T . w as lora_wgrad(x, w,
    transpose_out=True, out=dA_out, accumulate=dA_accumulate) does, bitwise, with one launch fewer
    than the two calls (ltx_lora_dy_dA)."""
    M, N = y.shape
    shape = (r, N) if transpose_out else (N, r)
    assert tuple(dB_out.shape) == shape and dB_out.dtype == F32 and dB_out.is_contiguous()
    on, oj = (1, N) if transpose_out else (r, 1)
    K2 = lora_k2(r)
    w = torch.empty(M, r, dtype=F32, device=y.device)
    sp = torch.empty(M, K2, dtype=BF16, device=y.device)
    n = ctypes.c_int64(0)
    if x is not None:
        K = x.shape[1]
        assert x.shape[0] == M and x.dtype == BF16 and lora_dy_fits(x, r) and N <= 2048
        assert tuple(dA_out.shape) == (r, K) and dA_out.dtype == F32 and dA_out.is_contiguous()
        call("ltx_lora_dy_dA_workspace", M, N, K, r, ctypes.byref(n))
        ws = torch.empty(n.value, dtype=F32, device=y.device)
        call("ltx_lora_dy_dA", _p(y), _rows(y, "y"), _p(u), _rows(u, "u"), _p(w3), _rows(w3, "w3"),
             _p(x), _rows(x, "x"), M, N, K, r, float(alpha), _p(w), _rows(w, "w"), _p(sp),
             _rows(sp, "split"), K2, _p(dB_out), on, oj, 1 if accumulate else 0, 1.0, _p(dA_out), 1,
             K, 1 if dA_accumulate else 0, _p(ws), _s())
        return w, sp
    call("ltx_lora_dy_workspace", M, N, r, ctypes.byref(n))
    ws = torch.empty(n.value, dtype=F32, device=y.device)
    call("ltx_lora_dy", _p(y), _rows(y, "y"), _p(u), _rows(u, "u"), _p(w3), _rows(w3, "w3"), M, N, r,
         float(alpha), _p(w), _rows(w, "w"), _p(sp), _rows(sp, "split"), K2, _p(dB_out), on, oj,
         1 if accumulate else 0, _p(ws), _s())
    return w, sp


# ---------------------------------------------------------------------------------------------
# small ops
# ---------------------------------------------------------------------------------------------
def timestep_embedding(t, scale, dim=256):
    _need(t, F32, "t")
    B = t.shape[0]
    out = torch.empty(B, dim, dtype=BF16, device=t.device)
    call("ltx_timestep_embedding", _p(t.contiguous()), float(scale), _p(out), B, dim, _s())
    return out


def silu(x):
    x = x.contiguous()
    y = torch.empty(x.shape, dtype=BF16, device=x.device)
    call("ltx_silu_bf16", _p(x), _p(y), x.numel(), _s())
    return y


def transpose(x, out=None):
    R, C = x.shape
    out = torch.empty(C, R, dtype=BF16, device=x.device) if out is None else out
    call("ltx_transpose_bf16", _p(x), _rows(x, "x"), _p(out), _rows(out, "out"), R, C, _s())
    return out


def colsum(x):
    """bf16 [N]: column sums of x [M, N] (f32 accumulation, one rounding)."""
    M, N = x.shape
    out = torch.empty(N, dtype=BF16, device=x.device)
    if N % 8 == 0 and x.stride(1) == 1 and x.stride(0) % 8 == 0 and M >= 64:
        return colsum_into(out, x, accumulate=False)  # split over rows: fills the chip
    call("ltx_colsum_bf16", _p(x), _rows(x, "x"), _p(out), M, N, _s())
    return out


def mse_fwd_bwd(out, v, grad_scale=1.0, want_grad=True):
    """Returns (stats[4] f32 device: sum sq-err, sum v, sum v^2, -, dout bf16 or None)."""
    n = out.numel()
    out, v = out.contiguous(), v.contiguous()
    stats = torch.empty(4 + 3 * 256, dtype=F32, device=out.device)  # + per-block partials
    dout = torch.empty(out.shape, dtype=BF16, device=out.device) if want_grad else None
    call("ltx_mse_fwd_bwd", _p(out), _p(v), _p(dout), _p(stats), n,
         float(grad_scale), _s())
    return stats[:4], dout


def adamw_step(param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, step):
    is_bf16 = 1 if param.dtype == BF16 else 0
    call("ltx_adamw_step", _p(param), _p(grad), _p(exp_avg), _p(exp_avg_sq), param.numel(),
         is_bf16, float(lr), float(beta1), float(beta2), float(eps), float(weight_decay),
         int(step), _s())


# ---------------------------------------------------------------------------------------------
# inference denoising step (csrc/denoise.hip)
# ---------------------------------------------------------------------------------------------
def pixel_coords(B, F, H, W, device, scale_factors=(8, 32, 32), causal_fix=True, frame_rate=25.0):
    """(float indices_grid [B,3,N] with the time axis / frame_rate, int64 pixel coords [B,3,N])
    (vae_encode.py:215-226, pipeline_ltx_video.py:1121-1122)."""
    out = torch.empty(B, 3, F * H * W, dtype=F32, device=device)
    pix = torch.empty(B, 3, F * H * W, dtype=torch.int64, device=device)
    call("ltx_pixel_coords_f32", _p(out), _p(pix), B, F, H, W, int(scale_factors[0]),
         int(scale_factors[1]), int(scale_factors[2]), 1 if causal_fix else 0, float(frame_rate),
         _s())
    return out, pix


def skip_blend(a, c, mask, rows_per_batch, out=None):
    """bf16(bf16(a * m) + bf16(c * bf16(1 - m))), m = mask[row // rows_per_batch] (bf16 [B])."""
    _need(a, BF16, "a")
    _need(c, BF16, "c")
    M, D = a.shape
    mask = mask.to(BF16).contiguous()
    out = torch.empty(M, D, dtype=BF16, device=a.device) if out is None else out
    call("ltx_skip_blend_bf16", _p(a), _rows(a, "a"), _p(c), _rows(c, "c"), _p(mask), _p(out),
         _rows(out, "out"), M, D, rows_per_batch, _s())
    return out


def rf_euler_step(model_output, timestep, sample, timesteps, cond_mask=None, t_cond=0.0):
    """RectifiedFlowScheduler.step (rf.py:305-374, deterministic) with eager dtype semantics:
    0-dim timestep -> global dt (a bf16 prediction rounds dt and dt*v to bf16), [B,N] timestep ->
    per-token dt in f32. Output dtype = torch's promotion of (sample, dt * v). cond_mask [B,N]:
    denoising_step's keep (pipeline_ltx_video.py:1378-1379) at scalar t_cond."""
    if model_output.shape != sample.shape:
        raise ValueError("rf_euler_step: model_output and sample shapes differ")
    for t, n in ((model_output, "model_output"), (sample, "sample")):
        if t.dtype not in (F32, BF16):
            raise TypeError(f"{n}: f32 or bf16 expected")
        if not t.is_cuda:
            raise _lib.LtxHipError(f"{n}: tensor is not on a ROCm device (no CPU fallback)")
    dev = sample.device
    per_token = timestep.ndim != 0
    if per_token and timestep.ndim != 2:
        raise ValueError("per-token timesteps must be [B, N]")
    ts = timestep.to(device=dev, dtype=F32).contiguous().reshape(-1)
    sched = timesteps.to(device=dev, dtype=F32).contiguous()
    v_f32 = model_output.dtype == F32
    prod_dtype = F32 if (per_token or v_f32) else BF16
    out_dtype = torch.promote_types(sample.dtype, prod_dtype)
    C = sample.shape[-1]
    BN = sample.numel() // C
    out = torch.empty(sample.shape, dtype=out_dtype, device=dev)
    cm = None if cond_mask is None else cond_mask.to(device=dev, dtype=F32).contiguous()
    call("ltx_rf_euler_step", _p(sample.contiguous()), 1 if sample.dtype == F32 else 0,
         _p(model_output.contiguous()), 1 if v_f32 else 0, _p(ts), 1 if per_token else 0,
         _p(sched), sched.numel(), _p(cm), float(t_cond), 0 if (per_token or v_f32) else 1,
         _p(out), 1 if out_dtype == F32 else 0, BN, C, _s())
    return out


def guidance(noise_pred, batch_size, do_cfg, do_stg, guidance_scale=1.0, stg_scale=0.0,
             rescaling_scale=1.0, cfg_star_rescale=False):
    """CFG / CFG* / STG / rescaling (pipeline_ltx_video.py:1229-1268) of the batched bf16
    prediction [nc*B, ...] -> [B, ...] bf16."""
    _need(noise_pred, BF16, "noise_pred")
    nc = 1 + int(bool(do_cfg)) + int(bool(do_stg))
    if noise_pred.shape[0] != nc * batch_size:
        raise ValueError(f"noise_pred batch {noise_pred.shape[0]} != {nc} x {batch_size}")
    pred = noise_pred.contiguous()
    L = pred[0].numel()
    out = torch.empty((batch_size,) + tuple(pred.shape[1:]), dtype=BF16, device=pred.device)
    ws = torch.empty(batch_size * 258, dtype=F32, device=pred.device)
    call("ltx_guidance_bf16", _p(pred), batch_size, L, int(bool(do_cfg)), int(bool(do_stg)),
         float(guidance_scale), float(stg_scale), float(rescaling_scale),
         int(bool(cfg_star_rescale)), _p(ws), ws.numel(), _p(out), _s())
    return out


# ---------------------------------------------------------------------------------------------
# train_mode='full' parameter gradients (csrc/paramgrad.hip, norms.hip:qk_norm_wgrad)
# ---------------------------------------------------------------------------------------------
def _splits(rows, D, groups):
    """row splits per group so that groups x splits ~ 512 blocks, >= 8 rows each"""
    s = max(1, min(rows // 8, 512 // max(1, groups)))
    return max(1, min(s, rows))


def colsum_into(out, a, b=None, r=None, mean=None, mode=0, rows_per_group=None, sum_groups=True,
                accumulate=True):
    """out (bf16) [+]= bf16 column sums of `mode`-products over row groups of a [M, D] (see
    ltx_group_colsum): sum_groups -> out [D] (sum over all groups), else out [G, D]."""
    M, D = a.shape
    rpg = M if rows_per_group is None else rows_per_group
    G = M // rpg
    S = _splits(rpg, D, G)
    part = torch.empty(G, S, D, dtype=F32, device=a.device)
    call("ltx_group_colsum", _p(a), _rows(a, "a"), _p(b), _rows(b, "b") if b is not None else 0,
         _p(r), _p(mean), int(mode), M, D, rpg, S, _p(part), _s())
    ldo = out.stride(0) if out.dim() == 2 else D
    call("ltx_colsum_finish", _p(part), G, S, D, 1 if sum_groups else 0, 1 if accumulate else 0,
         _p(out), ldo, _s())
    return out


def group_colsum(a, b=None, r=None, mean=None, mode=0, rows_per_group=None):
    """bf16 [G, D]: per-group column sums (no accumulation)."""
    M, D = a.shape
    rpg = M if rows_per_group is None else rows_per_group
    out = torch.empty(M // rpg, D, dtype=BF16, device=a.device)
    return colsum_into(out, a, b, r, mean, mode, rpg, sum_groups=False, accumulate=False)


def qk_norm_wgrad_into(dq, q_raw, rstd_q, gq, dk=None, k_raw=None, rstd_k=None, gk=None,
                       rope: "RopeSpec" = None, B=None, N=None):
    """q/k RMSNorm weight grads accumulated into gq / gk (bf16 [D])."""
    M, D = q_raw.shape
    if rope is not None:
        B, N = rope.B, rope.N
    S = _splits(M, D, 2 if dk is not None else 1)
    nsel = 2 if dk is not None else 1
    part = torch.empty(nsel, S, D, dtype=F32, device=q_raw.device)
    call("ltx_qk_norm_wgrad", _p(dq), _rows(dq, "dq"), 1 if dq.dtype == F32 else 0, _p(dk),
         _rows(dk, "dk") if dk is not None else 0, 1 if (dk is not None and dk.dtype == F32) else 0,
         _p(q_raw), _rows(q_raw, "q_raw"), _p(k_raw), _rows(k_raw, "k_raw") if k_raw is not None else 0,
         _p(rstd_q), _p(rstd_k), _p(rope.cs) if rope is not None else None,
         rope.cs_batch_rows if rope is not None else 0, B, N, D, 1 if rope is not None else 0, S,
         _p(part), _s())
    call("ltx_colsum_finish", _p(part[0]), 1, S, D, 1, 1, _p(gq), D, _s())
    if dk is not None:
        call("ltx_colsum_finish", _p(part[1]), 1, S, D, 1, 1, _p(gk), D, _s())


def silu_bwd(x, dy, dres=None):
    out = torch.empty_like(dy)
    call("ltx_silu_bwd_bf16", _p(x.contiguous()), _p(dy.contiguous()),
         _p(dres.contiguous()) if dres is not None else None, _p(out), dy.numel(), _s())
    return out


def _tpad(x, npad):
    """[M, C] -> [C, npad] bf16 transpose, zero-padded on the token axis (GEMM K % 64 == 0)."""
    M, C = x.shape
    buf = torch.empty(C, npad, dtype=BF16, device=x.device) if npad == M else \
        torch.zeros(C, npad, dtype=BF16, device=x.device)
    transpose(x, out=buf[:, :M])
    return buf


def wgrad_into(grad, dy, x, accumulate=True):
    """grad [N, K] (bf16) (+)= dy^T . x over the M token rows (dy [M, N], x [M, K]): the weight
    gradient of an nn.Linear. Both operands are transposed token-major ([N, M'], [K, M'], the
    token axis zero-padded to a multiple of 64) so the token axis becomes the NT GEMM's K; the
    product is rounded to bf16 once and accumulated as autograd's AccumulateGrad does
    (grad = bf16(grad + bf16(dy^T x)), the LTX_EPI_ACCUM epilogue)."""
    M, N = dy.shape
    M2, K = x.shape
    if M != M2 or tuple(grad.shape) != (N, K):
        raise ValueError(f"wgrad: shapes dy {tuple(dy.shape)} x {tuple(x.shape)} grad {tuple(grad.shape)}")
    _need(dy, BF16, "wgrad dy")
    _need(x, BF16, "wgrad x")
    _need(grad, BF16, "wgrad grad")
    mp = (M + 63) // 64 * 64
    dyT, xT = _tpad(dy, mp), _tpad(x, mp)
    if accumulate:
        return gemm(dyT, xT, epilogue="accum", aux0=grad, out=grad)
    return gemm(dyT, xT, out=grad)


def wgrad(dy, x):
    """bf16 [N, K] = dy^T . x (a fresh weight gradient)."""
    out = torch.empty(dy.shape[1], x.shape[1], dtype=BF16, device=dy.device)
    return wgrad_into(out, dy, x, accumulate=False)



def add_into(x, y):
    """x (bf16 [M, N]) = bf16(x + y): autograd's bf16 `.grad += new_grad`."""
    M, N = x.shape
    call("ltx_add_bf16", _p(x), _rows(x, "x"), _p(y), _rows(y, "y"), _p(x), _rows(x, "x"), M, N, _s())
    return x
