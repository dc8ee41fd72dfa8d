"""HipAttnProcessor: the operator-level plugin for Attention.set_processor (attention.py:532-552,
935-1114). Computes one Attention call (q/k/v projections with optional LoRA, q/k RMSNorm, RoPE
for self-attention, SDPA, to_out) with the same kernels the fused block uses.

Forward only (inference / pipeline use, e.g. LTXVideoPipeline's `transformer(...)` calls),
including the skip-layer (STG) blends of attention.py:1071-1085. Training runs the fused per-block autograd Function instead; calling
this processor on tensors that require grad raises.
"""
import torch

from . import ops


class HipAttnProcessor:
    def __call__(self, attn, hidden_states, freqs_cis=None, encoder_hidden_states=None,
                 attention_mask=None, temb=None, skip_layer_mask=None, skip_layer_strategy=None,
                 *args, **kwargs):
        from .transformer3d import _lin
        if torch.is_grad_enabled() and hidden_states.requires_grad:
            raise NotImplementedError("HipAttnProcessor is forward-only; training uses the fused block")
        B, N, Dq = hidden_states.shape
        src = hidden_states if encoder_hidden_states is None else encoder_hidden_states
        L = src.shape[1]
        H, d = attn.heads, attn.dim_head
        D = H * d
        x = hidden_states.reshape(B * N, Dq).contiguous()
        e = src.reshape(B * L, src.shape[2]).contiguous()

        def proj(lin, inp):
            w, b, lora = _lin(lin)
            if lora is None:
                return ops.gemm(inp, w, bias=b)
            _, su = ops.lora_down(inp, lora.lora_A["default"].weight, split=True)
            return ops.gemm(inp, w, bias=b, ext=(su, lora.weight_split("B")))

        q_raw = proj(attn.to_q, x)
        k_raw = proj(attn.to_k, e)
        v = proj(attn.to_v, e)
        if encoder_hidden_states is None and attn.use_rope:
            if not isinstance(freqs_cis, ops.RopeSpec):
                raise TypeError("freqs_cis must be an ltx_amd.ops.RopeSpec (cos/sin are formed in-kernel)")
            q, k, _, _ = ops.qk_norm_rope_fwd(q_raw, k_raw, attn.q_norm.weight, attn.k_norm.weight,
                                              freqs_cis)
        else:
            q, _, _, _ = ops.qk_norm_rope_fwd(q_raw, None, attn.q_norm.weight, None, None, B=B, N=N)
            k, _, _, _ = ops.qk_norm_rope_fwd(k_raw, None, attn.k_norm.weight, None, None, B=B, N=L)
        bias = None
        if attention_mask is not None:
            bias = attention_mask.reshape(B, -1).float().contiguous()
        o, _ = ops.attn_fwd(q, k, v, B, H, d, attn.scale, key_bias=bias)
        if skip_layer_mask is not None and skip_layer_strategy is not None:
            # attention.py:1071-1085 (Residual needs attn.residual_connection: False in LTX)
            name = getattr(skip_layer_strategy, "name", str(skip_layer_strategy))
            m = skip_layer_mask.reshape(B).to(torch.bfloat16)
            if name == "AttentionSkip":
                o = ops.skip_blend(o, x, m, N)
            elif name == "AttentionValues":
                o = ops.skip_blend(o, v, m, N)
        out = proj(attn.to_out[0], o)
        return out.view(B, N, -1)
