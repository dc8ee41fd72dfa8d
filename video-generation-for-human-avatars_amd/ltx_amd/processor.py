"""HipAttnProcessor: the operator-level plug-in for ``Attention.set_processor`` (attention.py:532-552),
called exactly like ``AttnProcessor2_0.__call__`` (attention.py:943-955):

    processor(attn, hidden_states, freqs_cis, encoder_hidden_states=None, attention_mask=None,
              temb=None, skip_layer_mask=None, skip_layer_strategy=None)

It runs one attention call (attention.py:996-1114) with the HIP kernels the fused block uses:
q/k/v projections (peft LoRA fused into the GEMM K loop), q/k RMSNorm across heads + RoPE for
self-attention, flash SDPA with the additive key bias, to_out -- and is differentiable: a
``torch.autograd.Function`` whose backward returns the gradients of hidden_states,
encoder_hidden_states, the peft adapters (f32) and, where they require grad (train_mode='full'),
the projection weights / biases and the q/k norm weights.

It works on the REFERENCE's Attention module (attention.py:325-932) and reads only its attributes:
``heads`` (head_dim = to_q.out_features // heads, as attention.py:1017-1018 derives it),
``scale``, ``use_rope``, ``q_norm`` / ``k_norm`` (RMSNorm ``weight`` + ``eps``), ``to_q`` /
``to_k`` / ``to_v`` / ``to_out[0]`` (``nn.Linear`` or a peft ``lora.Linear``: ``base_layer``,
``lora_A/lora_B['default']``, ``scaling['default']``), ``residual_connection``,
``rescale_output_factor``, ``spatial_norm``, ``group_norm``, ``norm_cross`` -- and on
``ltx_amd.transformer3d.Attention`` (same attribute names).

``freqs_cis`` is the reference's ``(cos, sin)`` pair from ``precompute_freqs_cis``
(transformer3d.py:221-277, bf16 [B, N, D]) or an ``ops.RopeSpec``. ``attention_mask`` is the
additive key bias as transformer3d.py:441-445 prepares it ([B, 1, L]; [B, L] and the head-repeated
[B, H, 1, L] / [B*H, 1, L] forms of prepare_attention_mask are accepted).
"""
import torch

from . import ops


def _linear_parts(m):
    """(weight, bias, lora_A, lora_B, scaling) of an nn.Linear or a peft lora.Linear."""
    if hasattr(m, "base_layer"):
        base = m.base_layer
        drop = getattr(m, "lora_dropout", None)
        if drop is not None and "default" in drop and getattr(drop["default"], "p", 0.0) > 0 and m.training:
            raise NotImplementedError("HipAttnProcessor: LoRA dropout > 0 is not supported")
        sc = m.scaling["default"] if isinstance(m.scaling, dict) else m.scaling
        return base.weight, base.bias, m.lora_A["default"].weight, m.lora_B["default"].weight, float(sc)
    return m.weight, m.bias, None, None, 1.0


def _key_bias(mask, B, L):
    """Additive key bias [B, L] f32 from the reference's prepared mask forms."""
    if mask is None:
        return None
    if mask.dim() == 4:          # [B, H, 1, L] (head-repeated)
        m = mask[:, 0, 0, :]
    elif mask.dim() == 3:        # [B, 1, L] or [B*H, 1, L]
        m = mask.reshape(B, -1, mask.shape[-1])[:, 0, :]
    elif mask.dim() == 2:        # [B, L]
        m = mask
    else:
        raise ValueError(f"attention_mask of shape {tuple(mask.shape)}")
    if m.shape != (B, L):
        raise ValueError(f"attention_mask covers {tuple(m.shape)} keys, expected {(B, L)}")
    return m.float().contiguous()


class _Proj:
    """One (possibly LoRA-wrapped) projection: y = x W^T + b [+ s (x A^T) B^T]."""

    def __init__(self, lin):
        self.W, self.b, self.A, self.Bw, self.s = _linear_parts(lin)

    def fwd(self, x):
        if self.A is None:
            return ops.gemm(x, self.W, bias=self.b), None
        u, su = ops.lora_down(x, self.A, split=True)
        y = ops.gemm(x, self.W, bias=self.b, ext=(su, ops.lora_split(self.Bw, "weight", self.s)))
        return y, u

    def bwd(self, dy, x, u, acc=None):
        """-> (dx, dW, db, dA, dB); dx added into `acc` (bf16) when given."""
        dA = dB = ext = None
        if self.A is not None:
            dB = ops.lora_wgrad(dy, u, alpha=self.s)                          # s dY^T (x A^T)
            w, sw = ops.lora_down(dy, self.Bw, alpha=self.s, transposed=True, split=True)  # s dY B
            dA = ops.lora_wgrad(x, w, transpose_out=True)                     # (s dY B)^T x
            ext = (sw, ops.lora_split(self.A, "weight", transposed=True))
        dx = ops.gemm(dy, ops.transpose(self.W), epilogue="accum" if acc is not None else "store",
                      aux0=acc, out=acc, ext=ext)
        dW = ops.wgrad(dy, x) if self.W.requires_grad else None
        db = ops.colsum(dy) if (self.b is not None and self.b.requires_grad) else None
        return dx, dW, db, dA, dB


class _AttnCall(torch.autograd.Function):
    """attention.py:996-1114 for one Attention call; see the module docstring."""

    @staticmethod
    def forward(ctx, st, x, enc, bias, gq, gk, *params):
        B, N, L, H, d = st["B"], st["N"], st["L"], st["H"], st["d"]
        pq, pk, pv, po = st["proj"]
        x2 = x.reshape(B * N, x.shape[-1]).contiguous()
        e2 = x2 if enc is None else enc.reshape(B * L, enc.shape[-1]).contiguous()
        q_raw, u_q = pq.fwd(x2)
        k_raw, u_k = pk.fwd(e2)
        v, u_v = pv.fwd(e2)
        rope = st["rope"]
        if rope is not None and st["eps"] == st["k_eps"]:  # one launch for q and k
            q, k, rq, rk = ops.qk_norm_rope_fwd(q_raw, k_raw, gq, gk, rope, eps=st["eps"])
        elif rope is not None:  # q_norm / k_norm with different eps: each its own
            q, _, rq, _ = ops.qk_norm_rope_fwd(q_raw, None, gq, None, rope, eps=st["eps"])
            k, _, rk, _ = ops.qk_norm_rope_fwd(k_raw, None, gk, None, rope, eps=st["k_eps"])
        else:
            q, _, rq, _ = ops.qk_norm_rope_fwd(q_raw, None, gq, None, None, B=B, N=N, eps=st["eps"])
            k, _, rk, _ = ops.qk_norm_rope_fwd(k_raw, None, gk, None, None, B=B, N=L, eps=st["k_eps"])
        o, lse = ops.attn_fwd(q, k, v, B, H, d, st["scale"], key_bias=bias)
        skip = st["skip"]
        if skip is not None:  # attention.py:1071-1085 (inference only)
            m, name = skip
            if name == "AttentionSkip":
                o = ops.skip_blend(o, x2, m, N)
            elif name == "AttentionValues":
                o = ops.skip_blend(o, v, m, N)
        out, u_o = po.fwd(o)
        ctx.st = st
        ctx.save_for_backward(x2, e2 if enc is not None else None, bias, gq, gk, q_raw, k_raw, v, q, k,
                              rq, rk, o, lse, u_q, u_k, u_v, u_o)
        ctx.has_enc = enc is not None
        return out.view(B, N, -1)

    @staticmethod
    def backward(ctx, dout):
        st = ctx.st
        B, N, L, H, d = st["B"], st["N"], st["L"], st["H"], st["d"]
        pq, pk, pv, po = st["proj"]
        (x2, e2, bias, gq, gk, q_raw, k_raw, v, q, k, rq, rk, o, lse, u_q, u_k, u_v,
         u_o) = ctx.saved_tensors
        self_attn = not ctx.has_enc
        if self_attn:
            e2 = x2
        dy = dout.reshape(B * N, -1).contiguous()
        do, dWo, dbo, dAo, dBo = po.bwd(dy, o, u_o)
        dq, dk, dv = ops.attn_bwd(q, k, v, o, do, lse, B, H, d, st["scale"], key_bias=bias)
        rope = st["rope"]
        if rope is not None:
            dq_raw, dk_raw = ops.qk_norm_rope_bwd(dq, q_raw, gq, rq, dk, k_raw, gk, rk, rope)
        else:
            dq_raw, _ = ops.qk_norm_rope_bwd(dq, q_raw, gq, rq, B=B, N=N)
            dk_raw, _ = ops.qk_norm_rope_bwd(dk, k_raw, gk, rk, B=B, N=L)
        dgq = dgk = None
        if gq.requires_grad or gk.requires_grad:
            dgq = torch.zeros_like(gq)
            dgk = torch.zeros_like(gk)
            if rope is not None:
                ops.qk_norm_wgrad_into(dq, q_raw, rq, dgq, dk, k_raw, rk, dgk, rope=rope)
            else:
                ops.qk_norm_wgrad_into(dq, q_raw, rq, dgq, B=B, N=N)
                ops.qk_norm_wgrad_into(dk, k_raw, rk, dgk, B=B, N=L)
        dx, dWq, dbq, dAq, dBq = pq.bwd(dq_raw, x2, u_q)
        if self_attn:  # k and v read the same rows: their input grads add into dx
            _, dWk, dbk, dAk, dBk = pk.bwd(dk_raw, e2, u_k, acc=dx)
            _, dWv, dbv, dAv, dBv = pv.bwd(dv, e2, u_v, acc=dx)
            denc = None
        else:
            denc, dWk, dbk, dAk, dBk = pk.bwd(dk_raw, e2, u_k)
            _, dWv, dbv, dAv, dBv = pv.bwd(dv, e2, u_v, acc=denc)
            denc = denc.view(B, L, -1)
        grads = []
        for p_, dW, db, dA, dB in ((pq, dWq, dbq, dAq, dBq), (pk, dWk, dbk, dAk, dBk),
                                   (pv, dWv, dbv, dAv, dBv), (po, dWo, dbo, dAo, dBo)):
            grads += [dW, db, dA, dB]
        return (None, dx.view(B, N, -1), denc, None, dgq, dgk, *grads)


class HipAttnProcessor:
    """Attention.set_processor plug-in (attention.py:532-552) with AttnProcessor2_0's call
    signature (attention.py:943-955); see the module docstring."""

    def __call__(self, attn, hidden_states, freqs_cis=None, encoder_hidden_states=None,
                 attention_mask=None, temb=None, skip_layer_mask=None, skip_layer_strategy=None,
                 *args, **kwargs):
        for name in ("spatial_norm", "group_norm", "norm_cross"):
            if getattr(attn, name, None):
                raise NotImplementedError(f"HipAttnProcessor: attn.{name} is not used by LTX-Video")
        if getattr(attn, "residual_connection", False) or getattr(attn, "rescale_output_factor", 1.0) != 1.0:
            raise NotImplementedError("HipAttnProcessor: residual_connection / rescale_output_factor "
                                      "are not used by LTX-Video (attention.py:1103-1112)")
        if hidden_states.dim() != 3:
            raise NotImplementedError("HipAttnProcessor: [B, N, C] hidden states (LTX-Video)")
        if hidden_states.dtype != torch.bfloat16:
            raise TypeError("HipAttnProcessor computes in bf16: call model.to(torch.bfloat16)")
        B, N, _ = hidden_states.shape
        enc = encoder_hidden_states
        L = N if enc is None else enc.shape[1]
        proj = tuple(_Proj(m) for m in (attn.to_q, attn.to_k, attn.to_v, attn.to_out[0]))
        H = attn.heads
        inner = proj[0].W.shape[0]
        d = inner // H  # attention.py:1017-1018 (the reference Attention has no dim_head attribute)
        rope = None
        if enc is None and attn.use_rope:
            if isinstance(freqs_cis, (tuple, list)):
                rope = ops.RopePair(freqs_cis[0], freqs_cis[1])
            elif isinstance(freqs_cis, ops.RopeSpec):
                rope = freqs_cis
            else:
                raise TypeError("freqs_cis: the (cos, sin) pair of precompute_freqs_cis or an ops.RopeSpec")
            if (rope.B, rope.N, rope.D) != (B, N, inner):
                raise ValueError(f"freqs_cis covers {(rope.B, rope.N, rope.D)}, hidden states {(B, N, inner)}")
        skip = None
        if skip_layer_mask is not None and skip_layer_strategy is not None:
            if torch.is_grad_enabled():
                raise NotImplementedError("skip-layer masks are an inference (forward-only) feature")
            name = getattr(skip_layer_strategy, "name", str(skip_layer_strategy))
            skip = (skip_layer_mask.reshape(B).to(torch.bfloat16).contiguous(), name)
        st = dict(B=B, N=N, L=L, H=H, d=d, scale=float(attn.scale), rope=rope, proj=proj, skip=skip,
                  eps=float(attn.q_norm.eps), k_eps=float(attn.k_norm.eps))
        if enc is not None and enc.dtype != torch.bfloat16:
            raise TypeError("HipAttnProcessor: encoder_hidden_states must be bf16")
        params = []
        for p_ in proj:
            params += [p_.W, p_.b, p_.A, p_.Bw]
        return _AttnCall.apply(st, hidden_states, enc, _key_bias(attention_mask, B, L),
                               attn.q_norm.weight, attn.k_norm.weight, *params)
