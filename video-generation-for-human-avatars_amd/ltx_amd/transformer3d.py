"""Transformer3DModel for MI355X: the reference's module tree and call surface
(ltx_video/models/transformers/transformer3d.py:49-565, attention.py:38-1264) executed by fused
HIP kernels through libltxhip.so.

Module / parameter names are the reference's (and therefore PEFT-targetable and state-dict
compatible): transformer_blocks.{i}.attn1.to_q ..., attn2.to_out.0, q_norm.weight, ff.net.0.proj,
ff.net.2, scale_shift_table, adaln_single.emb.timestep_embedder.linear_1, caption_projection ...

Execution: each BasicTransformerBlock runs as ONE torch.autograd.Function (_BlockFn) whose
forward/backward are explicit sequences of C-ABI kernel launches (see DESIGN.md for the list and
for which tensors are kept for the backward). Frozen weights are packed once into the layouts the
kernels want (fused QKV [3D, D], and W^T copies for the dgrad GEMMs -- the weights never change
in lora_audio training, so no wgrad and no repacking per step). The caption projection (trainable)
and the output head are their own Functions; the AdaLN-single timestep path needs no gradient.
"""
import glob
import json
import math
import os
from dataclasses import dataclass
from enum import Enum, auto
from pathlib import Path
from typing import Any, Dict, List, Optional

import torch
from torch import nn

from . import _lib, ops
from .patchifier import SymmetricPatchifier

# LTX-Video 2B transformer config (ltx_video/utils/diffusers_config_mapping.py:74-105)
OURS_TRANSFORMER_CONFIG = {
    "_class_name": "Transformer3DModel",
    "activation_fn": "gelu-approximate",
    "attention_bias": True,
    "attention_head_dim": 64,
    "attention_type": "default",
    "caption_channels": 4096,
    "cross_attention_dim": 2048,
    "double_self_attention": False,
    "dropout": 0.0,
    "in_channels": 128,
    "norm_elementwise_affine": False,
    "norm_eps": 1e-06,
    "norm_num_groups": 32,
    "num_attention_heads": 32,
    "num_embeds_ada_norm": 1000,
    "num_layers": 28,
    "num_vector_embeds": None,
    "only_cross_attention": False,
    "out_channels": 128,
    "project_to_2d_pos": True,
    "upcast_attention": False,
    "use_linear_projection": False,
    "qk_norm": "rms_norm",
    "standardization_norm": "rms_norm",
    "positional_embedding_type": "rope",
    "positional_embedding_theta": 10000.0,
    "positional_embedding_max_pos": [20, 2048, 2048],
    "timestep_scale_multiplier": 1000,
}

# diffusers checkpoint key renames (diffusers_config_mapping.py:140-145)
TRANSFORMER_KEYS_RENAME_DICT = {"proj_in": "patchify_proj", "time_embed": "adaln_single",
                                "norm_q": "q_norm", "norm_k": "k_norm"}


class SkipLayerStrategy(Enum):
    """ltx_video/utils/skip_layer_strategy.py:4-8 (same members, same order)."""
    AttentionSkip = auto()
    AttentionValues = auto()
    Residual = auto()
    TransformerBlock = auto()


@dataclass
class Transformer3DModelOutput:
    sample: torch.Tensor

    def __getitem__(self, i):
        return (self.sample,)[i] if isinstance(i, int) else getattr(self, i)


# ===============================================================================================
# parameter holders (reference module tree)
# ===============================================================================================
class RMSNorm(nn.Module):
    """diffusers RMSNorm parameters (the math runs in the fused kernels)."""

    def __init__(self, dim, eps, elementwise_affine=True):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim)) if elementwise_affine else None


class LoraLinear(nn.Module):
    """peft 0.17.1 lora.Linear naming: base_layer, lora_A/lora_B ModuleDicts keyed 'default';
    f32 adapters on a bf16 base (autocast_adapter_dtype). The math is fused into the GEMMs."""

    def __init__(self, base_layer: nn.Linear, r: int, lora_alpha: int):
        super().__init__()
        self.base_layer = base_layer
        self.r = r
        self.lora_alpha = lora_alpha
        self.scaling = lora_alpha / r
        dev = base_layer.weight.device
        self.lora_A = nn.ModuleDict({"default": nn.Linear(base_layer.in_features, r, bias=False,
                                                          device=dev, dtype=torch.float32)})
        self.lora_B = nn.ModuleDict({"default": nn.Linear(r, base_layer.out_features, bias=False,
                                                          device=dev, dtype=torch.float32)})
        nn.init.kaiming_uniform_(self.lora_A["default"].weight, a=math.sqrt(5))
        nn.init.zeros_(self.lora_B["default"].weight)
        self._split_cache = {}

    def weight_split(self, which):
        """Cached K-extension weight operands (3-term bf16 split, ltx_lora_split_bf16):
        'B' -> s*B for the forward GEMM, 'A' -> A^T for the input-gradient GEMM. Rebuilt when
        the adapter changes: new storage, an in-place torch update (version counter) or a
        FusedAdamW step (ops.weight_generation())."""
        p = _ab(self)[1 if which == "B" else 0]
        key = (p.data_ptr(), p._version, ops.weight_generation())
        hit = self._split_cache.get(which)
        if hit is None or hit[0] != key:
            with torch.no_grad():
                t = (ops.lora_split(p, "weight", self.scaling) if which == "B"
                     else ops.lora_split(p, "weight", transposed=True))
            hit = (key, t)
            self._split_cache[which] = hit
        return hit[1]

    def weight_pieces(self, which):
        """Cached bf16 pieces (ops.lora_pieces) of 'A' (lora_A) or 'Bt' (lora_B^T): the weight
        operand of the token-sized adapter contractions (ltx_lora_rows); same keys as
        weight_split."""
        p = _ab(self)[1 if which == "Bt" else 0]
        key = (p.data_ptr(), p._version, ops.weight_generation())
        hit = self._split_cache.get("pieces_" + which)
        if hit is None or hit[0] != key:
            with torch.no_grad():
                t = ops.lora_pieces(p, transposed=(which == "Bt"))
            hit = (key, t)
            self._split_cache["pieces_" + which] = hit
        return hit[1]

    @property
    def weight(self):
        return self.base_layer.weight

    @property
    def bias(self):
        return self.base_layer.bias

    @property
    def in_features(self):
        return self.base_layer.in_features

    @property
    def out_features(self):
        return self.base_layer.out_features

    @torch.no_grad()
    def merged_weight(self):
        """W + s * B A (peft merge_and_unload), in the base dtype."""
        a = self.lora_A["default"].weight
        b = self.lora_B["default"].weight
        return (self.base_layer.weight.float() + self.scaling * (b @ a)).to(self.base_layer.weight.dtype)


def _lin(m):
    """(weight, bias, lora) of an nn.Linear or LoraLinear."""
    if isinstance(m, LoraLinear):
        return m.base_layer.weight, m.base_layer.bias, m
    return m.weight, m.bias, None


class Attention(nn.Module):
    """Attention module of attention.py:325-932 (rms_norm qk-norm across all heads, biases)."""

    def __init__(self, query_dim, cross_attention_dim=None, heads=8, dim_head=64, bias=False,
                 out_bias=True, qk_norm=None, use_rope=False, **_unused):
        super().__init__()
        self.inner_dim = dim_head * heads
        self.heads = heads
        self.dim_head = dim_head
        self.scale = dim_head ** -0.5
        self.is_cross_attention = cross_attention_dim is not None
        self.cross_attention_dim = cross_attention_dim or query_dim
        self.use_rope = use_rope
        self.use_tpu_flash_attention = False
        if qk_norm != "rms_norm":
            raise NotImplementedError("LTX-Video uses qk_norm='rms_norm'")
        self.q_norm = RMSNorm(self.inner_dim, eps=1e-5)
        self.k_norm = RMSNorm(self.inner_dim, eps=1e-5)
        self.to_q = nn.Linear(query_dim, self.inner_dim, bias=bias)
        self.to_k = nn.Linear(self.cross_attention_dim, self.inner_dim, bias=bias)
        self.to_v = nn.Linear(self.cross_attention_dim, self.inner_dim, bias=bias)
        self.to_out = nn.ModuleList([nn.Linear(self.inner_dim, query_dim, bias=out_bias),
                                     nn.Dropout(0.0)])
        self.processor = None
        from .processor import HipAttnProcessor
        self.set_processor(HipAttnProcessor())

    def set_processor(self, processor):
        """Operator plugin point (attention.py:532-552)."""
        self.processor = processor

    def get_processor(self, return_deprecated_lora=False):
        return self.processor

    def set_use_tpu_flash_attention(self):
        raise NotImplementedError("TPU flash attention is out of scope on MI355X")

    def forward(self, hidden_states, freqs_cis=None, encoder_hidden_states=None,
                attention_mask=None, skip_layer_mask=None, skip_layer_strategy=None,
                **cross_attention_kwargs):
        return self.processor(self, hidden_states, freqs_cis=freqs_cis,
                              encoder_hidden_states=encoder_hidden_states,
                              attention_mask=attention_mask, skip_layer_mask=skip_layer_mask,
                              skip_layer_strategy=skip_layer_strategy)


class GELU(nn.Module):
    """diffusers GELU(dim_in, dim_out, approximate='tanh'): Linear `proj` then tanh-GELU."""

    def __init__(self, dim_in, dim_out, approximate="tanh", bias=True):
        super().__init__()
        self.proj = nn.Linear(dim_in, dim_out, bias=bias)
        self.approximate = approximate


class FeedForward(nn.Module):
    """attention.py:1204-1264 with activation_fn='gelu-approximate' (non-gated 4x MLP)."""

    def __init__(self, dim, dim_out=None, mult=4, dropout=0.0, activation_fn="gelu-approximate",
                 inner_dim=None, bias=True, **_unused):
        super().__init__()
        inner_dim = inner_dim or int(dim * mult)
        dim_out = dim_out or dim
        if activation_fn != "gelu-approximate":
            raise NotImplementedError(f"activation_fn={activation_fn!r}: LTX-2B uses "
                                      "'gelu-approximate' (diffusers_config_mapping.py:76)")
        self.net = nn.ModuleList([GELU(dim, inner_dim, "tanh", bias), nn.Dropout(dropout),
                                  nn.Linear(inner_dim, dim_out, bias=bias)])


class BasicTransformerBlock(nn.Module):
    """attention.py:38-321, adaptive_norm='single_scale_shift', standardization rms_norm."""

    def __init__(self, dim, num_attention_heads, attention_head_dim, cross_attention_dim=None,
                 activation_fn="gelu-approximate", attention_bias=False, norm_eps=1e-5,
                 qk_norm=None, use_rope=False, adaptive_norm="single_scale_shift",
                 standardization_norm="rms_norm", norm_elementwise_affine=False, **_unused):
        super().__init__()
        if adaptive_norm != "single_scale_shift" or standardization_norm != "rms_norm":
            raise NotImplementedError("LTX-2B: adaptive_norm single_scale_shift + rms_norm")
        if norm_elementwise_affine:
            raise NotImplementedError("LTX-2B: norm_elementwise_affine=False")
        self.adaptive_norm = adaptive_norm
        self.norm_eps = norm_eps
        self.norm1 = RMSNorm(dim, eps=norm_eps, elementwise_affine=False)
        self.attn1 = Attention(dim, None, num_attention_heads, attention_head_dim,
                               bias=attention_bias, qk_norm=qk_norm, use_rope=use_rope)
        self.attn2 = Attention(dim, cross_attention_dim, num_attention_heads, attention_head_dim,
                               bias=attention_bias, qk_norm=qk_norm, use_rope=use_rope)
        self.norm2 = RMSNorm(dim, eps=norm_eps, elementwise_affine=False)
        self.ff = FeedForward(dim, activation_fn=activation_fn)
        self.scale_shift_table = nn.Parameter(torch.randn(6, dim) / dim ** 0.5)
        self._pack = None
        self._pack_key = None

    # ---- frozen-weight packing (fused QKV + W^T copies for the dgrad GEMMs) ----
    def _frozen(self):
        # direct _modules / _parameters lookups: nn.Module.__getattr__ is ~60 us per block here,
        # paid twice per step per block on the host critical path
        a1, a2 = self._modules["attn1"]._modules, self._modules["attn2"]._modules
        net = self._modules["ff"]._modules["net"]._modules
        pw = lambda m, n="weight": _base(m)._parameters[n]
        return [pw(a1["to_q"]), pw(a1["to_q"], "bias"), pw(a1["to_k"]), pw(a1["to_k"], "bias"),
                pw(a1["to_v"]), pw(a1["to_v"], "bias"), pw(a1["to_out"]._modules["0"]),
                pw(a2["to_q"]), pw(a2["to_k"]), pw(a2["to_v"]), pw(a2["to_out"]._modules["0"]),
                pw(net["0"]._modules["proj"]), pw(net["2"])]

    @torch.no_grad()
    def packed(self):
        """Fused QKV weight/bias and W^T copies for the dgrad GEMMs, rebuilt whenever a weight
        changes (new storage, an in-place torch update, or a FusedAdamW step in
        train_mode='full' -- ops.weight_generation())."""
        fz = self._frozen()
        key = (tuple((t.data_ptr(), t._version) for t in fz), ops.weight_generation()
               if any(t.requires_grad for t in fz) else 0)
        if self._pack is not None and self._pack_key == key:
            return self._pack
        a1, a2, ff = self.attn1, self.attn2, self.ff
        p = {}
        p["qkv_w"] = torch.cat([a1.to_q.weight, a1.to_k.weight, a1.to_v.weight], 0).contiguous()
        p["qkv_b"] = torch.cat([a1.to_q.bias, a1.to_k.bias, a1.to_v.bias], 0).contiguous()
        p["qkv_wT"] = ops.transpose(p["qkv_w"])
        p["out1_wT"] = ops.transpose(a1.to_out[0].weight)
        for name, lin in (("q2", a2.to_q), ("k2", a2.to_k), ("v2", a2.to_v), ("o2", a2.to_out[0])):
            p[name + "_wT"] = ops.transpose(_lin(lin)[0])
        # text K and V as one [2D, D] projection (they share enc2): one GEMM each way
        p["kv2_w"] = torch.cat([_lin(a2.to_k)[0], _lin(a2.to_v)[0]], 0).contiguous()
        p["kv2_b"] = torch.cat([_lin(a2.to_k)[1], _lin(a2.to_v)[1]], 0).contiguous()
        p["kv2_wT"] = torch.cat([p["k2_wT"], p["v2_wT"]], 1).contiguous()
        self._kv_ext = None
        p["ff1_wT"] = ops.transpose(ff.net[0].proj.weight)
        p["ff2_wT"] = ops.transpose(ff.net[2].weight)
        self._pack, self._pack_key = p, key
        return p


def _kv_ext(blk, lk, lv):
    """K-extension weights of the merged text K/V GEMMs, rebuilt with the adapters: forward
    [2D, 2 K2] block-diagonal (split(s B_k) | 0 ; 0 | split(s B_v)), backward [D, 2 K2] =
    split(A_k^T) | split(A_v^T) (both adapters add into the encoder gradient)."""
    fb, fv = lk.weight_split("B"), lv.weight_split("B")
    ba, bv = lk.weight_split("A"), lv.weight_split("A")
    key = tuple(id(t) for t in (fb, fv, ba, bv))  # the splits are replaced when an adapter changes
    hit = getattr(blk, "_kv_ext", None)
    if hit is not None and hit[0] == key:
        return hit[1], hit[2]
    D, K2 = fb.shape
    fwd = torch.zeros(2 * D, 2 * K2, dtype=fb.dtype, device=fb.device)
    fwd[:D, :K2] = fb
    fwd[D:, K2:] = fv
    bwd = torch.cat([ba, bv], 1).contiguous()
    blk._kv_ext = (key, fwd, bwd, (fb, fv, ba, bv))  # hold the splits: ids stay unique
    return fwd, bwd


class TimestepEmbedding(nn.Module):
    def __init__(self, in_channels, time_embed_dim):
        super().__init__()
        self.linear_1 = nn.Linear(in_channels, time_embed_dim)
        self.linear_2 = nn.Linear(time_embed_dim, time_embed_dim)


class _CombinedTimestepEmbeddings(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.timestep_embedder = TimestepEmbedding(256, dim)


class AdaLayerNormSingle(nn.Module):
    """diffusers AdaLayerNormSingle parameters (emb.timestep_embedder.linear_{1,2}, linear)."""

    def __init__(self, embedding_dim, use_additional_conditions=False):
        super().__init__()
        self.emb = _CombinedTimestepEmbeddings(embedding_dim)
        self.linear = nn.Linear(embedding_dim, 6 * embedding_dim, bias=True)


class PixArtAlphaTextProjection(nn.Module):
    def __init__(self, in_features, hidden_size, out_features=None, act_fn="gelu_tanh"):
        super().__init__()
        self.linear_1 = nn.Linear(in_features, hidden_size, bias=True)
        self.linear_2 = nn.Linear(hidden_size, out_features or hidden_size, bias=True)


# ===============================================================================================
# fused autograd functions
# ===============================================================================================
class _Shared:
    """Per-forward constants shared by all blocks."""

    def __init__(self, B, N, L, heads, head_dim, rope, enc_bias, eps, text_shared=False,
                 per_token=False):
        self.B, self.N, self.L = B, N, L
        # AdaLN rows: one modulation row per batch (training) or per token (inference with a
        # [B, N] timestep, transformer3d.py:488-491): kernels index mod rows by m // rpm
        self.rpm = 1 if per_token else N
        # text_shared: every sample attends to the same prompt (train_step expands one prompt
        # over the batch, training.py:415), so the text side holds one batch (Bt = 1)
        self.text_shared = text_shared
        self.Bt = 1 if text_shared else B
        self.H, self.d = heads, head_dim
        self.D = heads * head_dim
        self.rope = rope
        self.enc_bias = enc_bias
        # text K/V per block prefetched on the side stream (inference, _forward_tokens)
        self.text_pre = None
        # all blocks' text K/V computed in one launch each way (LoRA training, _TextStack)
        self.text_stack = None
        self.eps = eps
        self.full = False  # train_mode='full': attention / AdaLN weights take gradients
        # block id -> the previous block's FF gate row view (mods[:, 5]): the block's backward
        # also writes the previous block's d_ffo = gate_mul(dh, gate) from its last norm pass,
        # handed over in ffo_pre = (dh, d_ffo) (LTX_FFGATE_FUSED=0: separate gate_mul launches)
        self.ffgate = {}
        self.ffo_pre = None


_LORA_KEYS = ("q", "k", "v", "o")


def _pgrad(p):
    """p.grad (bf16), created zeroed on first use: the full-mode kernels accumulate into it
    (the reference's .grad += over micro-steps)."""
    if p.grad is None:
        p.grad = torch.zeros_like(p, memory_format=torch.contiguous_format)
    return p.grad


def _base(m):
    """The nn.Linear under a LoraLinear (or the module itself)."""
    return m._modules["base_layer"] if type(m) is LoraLinear else m


def _lora_params(blk):
    """attn2 LoRA (A, B) per target in _LORA_KEYS order, or None (no adapters)."""
    a2 = blk._modules["attn2"]._modules
    lins = (a2["to_q"], a2["to_k"], a2["to_v"], a2["to_out"]._modules["0"])
    kinds = [type(m) is LoraLinear for m in lins]
    if not all(kinds):
        if any(kinds):
            raise NotImplementedError("LoRA must wrap all four attn2 projections (training.py:52-60)")
        return None
    return lins


def _ab(m):
    """(lora_A weight, lora_B weight) of a LoraLinear, by direct lookup."""
    return (m._modules["lora_A"]._modules["default"]._parameters["weight"],
            m._modules["lora_B"]._modules["default"]._parameters["weight"])


def _grad_buf(lin, which):
    """The .grad of a LoraLinear adapter weight ('A' or 'B'), created zeroed on first use: the
    LoRA wgrad kernels add into it directly (no per-micro-step buffer, memset or add)."""
    p = _ab(lin)[0 if which == "A" else 1]
    if p.grad is None:
        p.grad = torch.zeros_like(p, memory_format=torch.contiguous_format)
    return p.grad


class _BlockFn(torch.autograd.Function):
    """One BasicTransformerBlock.forward (attention.py:198-321) + its backward."""

    @staticmethod
    def forward(ctx, blk, sh, keep, skip, h, enc2, mods, onep, *lora_ab):
        """skip = (mask row [B] bf16, SkipLayerStrategy) for STG inference (attention.py:312-319,
        1071-1085), or None."""
        B, N, L, H, d, D = sh.B, sh.N, sh.L, sh.H, sh.d, sh.D
        M = B * N
        rpm = sh.rpm
        if skip is not None and keep:
            raise NotImplementedError("skip-layer masks are an inference (forward-only) feature")
        W = blk.packed()
        a1, a2, ff = blk.attn1, blk.attn2, blk.ff
        ldm = mods.stride(0)
        has_lora = len(lora_ab) > 0
        lora = _lora_params(blk) if has_lora else None
        r = lora[0].r if has_lora else 0
        s = lora[0].scaling if has_lora else 1.0
        # ---- 1. norm1 + AdaLN(msa) -> fused QKV -> q/k RMSNorm + RoPE -> SDPA -> gated residual
        x1, rstd1 = ops.rmsnorm_modulate_fwd(h, mods[:, 0], onep[:, 1], ldm, rpm, blk.norm_eps)
        qkv = ops.gemm(x1, W["qkv_w"], bias=W["qkv_b"])
        strat = skip[1] if skip is not None else None
        full = sh.full and keep
        if has_lora and full:
            raise NotImplementedError("train_mode='full' trains the base weights without LoRA")
        if strat is not SkipLayerStrategy.AttentionSkip and not full:
            del x1
        qk = torch.empty(M, 2 * D, dtype=torch.bfloat16, device=h.device)
        _, _, rq1, rk1 = ops.qk_norm_rope_fwd(qkv[:, :D], qkv[:, D:2 * D], a1.q_norm.weight,
                                              a1.k_norm.weight, sh.rope, q_out=qk[:, :D],
                                              k_out=qk[:, D:])
        o1, lse1 = ops.attn_fwd(qk[:, :D], qk[:, D:], qkv[:, 2 * D:], B, H, d, a1.scale)
        if strat is SkipLayerStrategy.AttentionSkip:  # blend with the processor input
            o1 = ops.skip_blend(o1, x1, skip[0], N)
            if not full:
                del x1
        elif strat is SkipLayerStrategy.AttentionValues:  # blend with to_v's output
            o1 = ops.skip_blend(o1, qkv[:, 2 * D:], skip[0], N)
        y1 = torch.empty(M, D, dtype=torch.bfloat16, device=h.device) if full else None
        h1 = ops.gemm(o1, a1.to_out[0].weight, bias=a1.to_out[0].bias, epilogue="gated_residual",
                      aux0=h, aux1=mods[:, 2], aux2=y1, rows_per_batch=rpm)
        # ---- 2. attn2 on the un-normalised h1 (attention.py:273-285), LoRA fused into the GEMMs
        wq, bq, _ = _lin(a2.to_q)
        wo, bo, _ = _lin(a2.to_out[0])
        pre = sh.text_pre.pop(id(blk), None) if sh.text_pre is not None else None
        if has_lora:
            # peft LoRA fused into the K loop: [x | split(x.A^T)] . [W | split(s*B)]^T
            Aq, Bq, Ak, Bk, Av, Bv, Ao, Bo = lora_ab
            u_q, su = ops.lora_down(h1, Aq, split=True, pieces=lambda: lora[0].weight_pieces("A"))
            q2raw = ops.gemm(h1, wq, bias=bq, ext=(su, lora[0].weight_split("B")))
            del su
        else:
            u_q = None
            q2raw = ops.gemm(h1, wq, bias=bq)
        q2, _, rq2, _ = ops.qk_norm_rope_fwd(q2raw, None, a2.q_norm.weight, None, None, B=B, N=N)
        if sh.text_stack is not None:  # computed for every block at once (_TextStack.forward)
            k2raw, k2, rk2, v2, u_k, u_v = sh.text_stack.block_kv(blk, sh)
        elif pre is None:
            k2raw, k2, rk2, v2, u_k, u_v = _text_kv(blk, sh, enc2, lora_ab)
        else:  # computed on the text side stream one block ahead (_forward_tokens)
            (k2raw, k2, rk2, v2, u_k, u_v), ev = pre
            torch.cuda.current_stream().wait_event(ev)
        o2, lse2 = ops.attn_fwd(q2, k2, v2, B, H, d, a2.scale, key_bias=sh.enc_bias,
                                kv_shared=sh.text_shared)
        if has_lora:
            u_o, su = ops.lora_down(o2, Ao, split=True, pieces=lambda: lora[3].weight_pieces("A"))
            h2 = ops.gemm(o2, wo, bias=bo, epilogue="accum", aux0=h1,
                          ext=(su, lora[3].weight_split("B")))
            del su
        else:
            u_o = None
            h2 = ops.gemm(o2, wo, bias=bo, epilogue="accum", aux0=h1)
        # ---- 3. norm2 + AdaLN(mlp) -> FF (tanh-GELU fused) -> gated residual
        x2, rstd2 = ops.rmsnorm_modulate_fwd(h2, mods[:, 3], onep[:, 4], ldm, rpm, blk.norm_eps)
        # fpre: rint(32767 gelu_tanh'(pre-activation) / 2) (int16), kept by the GELU epilogue for the
        # backward's multiply (ltx_hip.h LTX_EPI_GELU)
        fpre = torch.empty(M, ff.net[0].proj.out_features, dtype=torch.int16, device=h.device)
        act = ops.gemm(x2, ff.net[0].proj.weight, bias=ff.net[0].proj.bias, epilogue="gelu",
                       aux0=fpre)
        del x2
        y3 = torch.empty(M, D, dtype=torch.bfloat16, device=h.device) if full else None
        h3 = ops.gemm(act, ff.net[2].weight, bias=ff.net[2].bias, epilogue="gated_residual",
                      aux0=h2, aux1=mods[:, 5], aux2=y3, rows_per_batch=rpm)
        del act
        if strat is SkipLayerStrategy.TransformerBlock:
            h3 = ops.skip_blend(h3, h, skip[0], N)
        if keep:
            lora_saved = (u_q, u_k, u_v, u_o) if has_lora else ()
            full_saved = (x1, y1, y3) if full else ()
            ctx.save_for_backward(h, enc2, mods, onep, rstd1, qkv, qk, rq1, rk1, o1, lse1, h1,
                                  q2raw, rq2, q2, k2raw, rk2, k2, v2, o2, lse2, h2, rstd2, fpre,
                                  *lora_ab, *lora_saved, *full_saved)
            ctx.blk, ctx.sh, ctx.has_lora, ctx.full = blk, sh, has_lora, full
        return h3

    @staticmethod
    def backward(ctx, dh3):
        blk, sh = ctx.blk, ctx.sh
        B, N, L, H, d, D = sh.B, sh.N, sh.L, sh.H, sh.d, sh.D
        has_lora = ctx.has_lora
        saved = ctx.saved_tensors
        (h, enc2, mods, onep, rstd1, qkv, qk, rq1, rk1, o1, lse1, h1, q2raw, rq2, q2, k2raw, rk2,
         k2, v2, o2, lse2, h2, rstd2, fpre) = saved[:24]
        W = blk.packed()
        a1, a2 = blk.attn1, blk.attn2
        ldm = mods.stride(0)
        dh3 = dh3.contiguous()
        grads_lora = []
        full = ctx.full
        if full:
            x1, y1, y3 = saved[24:27]
            dmods = torch.empty(B, 6, D, dtype=torch.bfloat16, device=h.device)
        if has_lora:
            Aq, Bq, Ak, Bk, Av, Bv, Ao, Bo = saved[24:32]
            u_q, u_k, u_v, u_o = saved[32:36]
            lora = _lora_params(blk)
            r, s = lora[0].r, lora[0].scaling
        # ---- FF: h3 = h2 + g_mlp * ff(x2)
        rpm = sh.rpm
        pre, sh.ffo_pre = sh.ffo_pre, None
        # accepted only for the very dh buffer the next block's norm pass wrote. Safe because
        # ffo_pre holds a reference to that dh: while it is alive autograd cannot accumulate
        # another gradient into the buffer in place, so d_ffo = bf16(dh * g_mlp) still matches it
        if pre is not None and pre[0].data_ptr() == dh3.data_ptr() and pre[0].shape == dh3.shape:
            d_ffo = pre[1]  # written by the next block's last norm pass (bitwise gate_mul)
        else:
            d_ffo = ops.gate_mul(dh3, mods[:, 5], rpm)
        del pre
        if full:  # gate_mlp: sum over the batch's rows of bf16(dh3 * y3) (attention.py:305-308)
            ops.colsum_into(dmods[:, 5], dh3, y3, mode=1, rows_per_group=rpm, sum_groups=False,
                            accumulate=False)
        d_f = ops.gemm(d_ffo, W["ff2_wT"], epilogue="gelu_bwd", aux0=fpre)
        del d_ffo
        dx2 = ops.gemm(d_f, W["ff1_wT"])
        del d_f
        dh2 = ops.rmsnorm_modulate_bwd(dx2, h2, rstd2, onep[:, 4], ldm, rpm, dres=dh3)
        if full:  # shift_mlp / scale_mlp (attention.py:287-290)
            ops.colsum_into(dmods[:, 3], dx2, rows_per_group=rpm, sum_groups=False, accumulate=False)
            ops.colsum_into(dmods[:, 4], dx2, h2, rstd2, mode=2, rows_per_group=rpm,
                            sum_groups=False, accumulate=False)
        del dx2
        # ---- attn2: h2 = h1 + to_out(o2)   (LoRA grads: peft f32 adapters)
        # dO of the cross-attention + its delta rowsum(dO*O) in the GEMM epilogue
        delta2 = torch.empty(B, H, N, dtype=torch.float32, device=h.device) if _DELTA_FUSED else None
        rd = dict(epilogue="store_rowdot", aux0=o2, aux1=delta2, rank=d, rows_per_batch=N) \
            if _DELTA_FUSED else {}
        if has_lora:
            lq, lk, lv, lo = lora
            dy_ok = ops.lora_dy_enabled() and ops.lora_dy_fits(dh2, r)
            if dy_ok and ops.lora_dy_da_fits(dh2, o2, r):
                # one pass over dY, one over o2 (dA), one finish for w / split, dB and dA
                w_o, sw = ops.lora_dy(dh2, u_o, lo.weight_pieces("Bt"), r, s, _grad_buf(lo, "B"),
                                      x=o2, dA_out=_grad_buf(lo, "A"))
            else:
                if dy_ok:  # one pass over dY
                    w_o, sw = ops.lora_dy(dh2, u_o, lo.weight_pieces("Bt"), r, s, _grad_buf(lo, "B"))
                else:
                    ops.lora_wgrad(dh2, u_o, alpha=s, out=_grad_buf(lo, "B"), accumulate=True)
                    w_o, sw = ops.lora_down(dh2, Bo, alpha=s, transposed=True, split=True,
                                             pieces=lambda: lo.weight_pieces("Bt"))
                ops.lora_wgrad(o2, w_o, transpose_out=True, out=_grad_buf(lo, "A"), accumulate=True)
            do2 = ops.gemm(dh2, W["o2_wT"], ext=(sw, lo.weight_split("A")), **rd)
        else:
            do2 = ops.gemm(dh2, W["o2_wT"], **rd)
        if full:  # attn2.to_out.0
            lin = a2.to_out[0]
            ops.wgrad_into(_pgrad(lin.weight), dh2, o2)
            ops.colsum_into(_pgrad(lin.bias), dh2)
        # [dK_raw | dV] of the text rows side by side: the merged encoder-gradient GEMM's operand
        # (with the text stack: this block's slice of the all-blocks operand, reduced at the end)
        tx = sh.text_stack
        if tx is not None:
            dkv = tx.block_dkv(blk)
        else:
            dkv = torch.empty(k2raw.shape[0], 2 * D, dtype=torch.bfloat16, device=h.device)
        dk2b = dv2b = None
        # with the grouped text k_norm the stack keeps this block's dK (the norm's backward runs
        # for every block at once in _TextStack.backward)
        dk2_keep = tx.block_dk2(blk) if tx is not None and tx.grouped_norm else None
        if sh.text_shared and dk2_keep is not None and _TEXT_BSUM_GROUPED:
            # the batch sums of every block run in _TextStack.backward (one launch)
            dkb, dvb = tx.block_dkvb(blk, B)
            dq2, _, _ = ops.attn_bwd(q2, k2, v2, o2, do2, lse2, B, H, d, a2.scale, key_bias=sh.enc_bias,
                                     kv_shared=True, dk=dkb, dv=dvb, delta=delta2)
            dk2 = dv2 = None
        elif sh.text_shared:  # gradient of the shared text rows = sum over the query batches
            dq2, dk2b, dv2b = ops.attn_bwd(q2, k2, v2, o2, do2, lse2, B, H, d, a2.scale,
                                           key_bias=sh.enc_bias, kv_shared=True, delta=delta2)
            dk2 = ops.batch_sum(dk2b, B, out=dk2_keep)
            dv2 = ops.batch_sum(dv2b, B, out=dkv[:, D:])
            if not full:
                dk2b = dv2b = None
        else:
            dq2, dk2, dv2 = ops.attn_bwd(q2, k2, v2, o2, do2, lse2, B, H, d, a2.scale,
                                         key_bias=sh.enc_bias, dk=dk2_keep, dv=dkv[:, D:], delta=delta2)
        del do2
        dq2raw, _ = ops.qk_norm_rope_bwd(dq2, q2raw, a2.q_norm.weight, rq2, B=B, N=N)
        if dk2_keep is None:
            dk2raw, _ = ops.qk_norm_rope_bwd(dk2, k2raw, a2.k_norm.weight, rk2, B=sh.Bt, N=L,
                                             dq_out=dkv[:, :D])
        else:
            dk2raw = None
        if full:  # attn2 q/k norm weights, to_q / to_k / to_v
            ops.qk_norm_wgrad_into(dq2, q2raw, rq2, _pgrad(a2.q_norm.weight), B=B, N=N)
            ops.wgrad_into(_pgrad(a2.to_q.weight), dq2raw, h1)
            ops.colsum_into(_pgrad(a2.to_q.bias), dq2raw)
            if dk2b is not None:
                # one prompt expanded over the batch: the reference runs to_k / k_norm / to_v on B
                # identical copies of the text rows (training.py:113-117), so its k / v parameter
                # grads sum B per-sample bf16 SDPA / k-norm gradients in f32. Summing the batch
                # first (one bf16 rounding of the sum, as the K/V input gradient above does) loses
                # the small, cancelling to_k.bias gradient (measured 2.3x the reference's bf16
                # noise at 2B widths): these grads take the per-sample rows instead.
                krep, erep, rrep = k2raw.repeat(B, 1), enc2.repeat(B, 1), rk2.repeat(B)
                dk2raw_b, _ = ops.qk_norm_rope_bwd(dk2b, krep, a2.k_norm.weight, rrep, B=B, N=L)
                ops.qk_norm_wgrad_into(dk2b, krep, rrep, _pgrad(a2.k_norm.weight), B=B, N=L)
                ops.wgrad_into(_pgrad(a2.to_k.weight), dk2raw_b, erep)
                ops.colsum_into(_pgrad(a2.to_k.bias), dk2raw_b)
                ops.wgrad_into(_pgrad(a2.to_v.weight), dv2b, erep)
                ops.colsum_into(_pgrad(a2.to_v.bias), dv2b)
                del krep, erep, rrep, dk2raw_b, dk2b, dv2b
            else:
                ops.qk_norm_wgrad_into(dk2, k2raw, rk2, _pgrad(a2.k_norm.weight), B=sh.Bt, N=L)
                ops.wgrad_into(_pgrad(a2.to_k.weight), dk2raw, enc2)
                ops.colsum_into(_pgrad(a2.to_k.bias), dk2raw)
                ops.wgrad_into(_pgrad(a2.to_v.weight), dv2, enc2)
                ops.colsum_into(_pgrad(a2.to_v.bias), dv2)
        del dq2, dk2
        denc = None
        # dh1 = dh2 + dq2raw . W_q2 (+ LoRA) and, from the same epilogue, d_y1 = bf16(dh1 * g_msa)
        d_y1 = torch.empty_like(dh2)
        gated = dict(aux1=mods[:, 2], aux2=d_y1, rows_per_batch=rpm)
        if has_lora:
            dy_ok = ops.lora_dy_enabled() and ops.lora_dy_fits(dq2raw, r)
            if dy_ok and ops.lora_dy_da_fits(dq2raw, h1, r):
                w_q, sw = ops.lora_dy(dq2raw, u_q, lq.weight_pieces("Bt"), r, s, _grad_buf(lq, "B"),
                                      x=h1, dA_out=_grad_buf(lq, "A"))
            else:
                if dy_ok:
                    w_q, sw = ops.lora_dy(dq2raw, u_q, lq.weight_pieces("Bt"), r, s, _grad_buf(lq, "B"))
                else:
                    ops.lora_wgrad(dq2raw, u_q, alpha=s, out=_grad_buf(lq, "B"), accumulate=True)
                    w_q, sw = ops.lora_down(dq2raw, Bq, alpha=s, transposed=True, split=True,
                                             pieces=lambda: lq.weight_pieces("Bt"))
                ops.lora_wgrad(h1, w_q, transpose_out=True, out=_grad_buf(lq, "A"), accumulate=True)
            dh1 = ops.gemm(dq2raw, W["q2_wT"], epilogue="accum", aux0=dh2,
                           ext=(sw, lq.weight_split("A")), **gated)
            if tx is None:
                K2 = ops.lora_k2(r)
                swkv = torch.empty(dkv.shape[0], 2 * K2, dtype=torch.bfloat16, device=h.device)
                ops.lora_wgrad(dk2raw, u_k, alpha=s, out=_grad_buf(lk, "B"), accumulate=True)
                w_k, _ = ops.lora_down(dk2raw, Bk, alpha=s, transposed=True, split=True,
                                       split_out=swkv[:, :K2])
                ops.lora_wgrad(enc2, w_k, transpose_out=True, out=_grad_buf(lk, "A"),
                               accumulate=True)
                ops.lora_wgrad(dv2, u_v, alpha=s, out=_grad_buf(lv, "B"), accumulate=True)
                w_v, _ = ops.lora_down(dv2, Bv, alpha=s, transposed=True, split=True,
                                       split_out=swkv[:, K2:])
                ops.lora_wgrad(enc2, w_v, transpose_out=True, out=_grad_buf(lv, "A"),
                               accumulate=True)
                # denc = dK_raw.W_k + dV.W_v + both adapters' input-gradient terms, one GEMM
                denc = ops.gemm(dkv, W["kv2_wT"], ext=(swkv, _kv_ext(blk, lk, lv)[1]))
                del swkv
            # the adapter gradients went straight into .grad (accumulated across micro-steps by
            # the kernels' atomics); autograd gets None for them
            grads_lora = [None] * 8
        else:
            dh1 = ops.gemm(dq2raw, W["q2_wT"], epilogue="accum", aux0=dh2, **gated)
            if tx is None:
                denc = ops.gemm(dkv, W["kv2_wT"])
        del dq2raw, dk2raw, dv2, dh2, dkv
        # ---- attn1: h1 = h + g_msa * to_out(sdpa(rope(qn(q)), rope(kn(k)), v))
        # (d_y1 = bf16(dh1 * g_msa) came out of the dh1 GEMM's epilogue: `gated` above)
        delta1 = torch.empty(B, H, N, dtype=torch.float32, device=h.device) if _DELTA_FUSED else None
        rd = dict(epilogue="store_rowdot", aux0=o1, aux1=delta1, rank=d, rows_per_batch=N) \
            if _DELTA_FUSED else {}
        do1 = ops.gemm(d_y1, W["out1_wT"], **rd)
        if full:  # gate_msa, attn1.to_out.0
            ops.colsum_into(dmods[:, 2], dh1, y1, mode=1, rows_per_group=rpm, sum_groups=False,
                            accumulate=False)
            lin = a1.to_out[0]
            ops.wgrad_into(_pgrad(lin.weight), d_y1, o1)
            ops.colsum_into(_pgrad(lin.bias), d_y1)
        del d_y1
        M = B * N
        dqkv = torch.empty(M, 3 * D, dtype=torch.bfloat16, device=h.device)
        dq1, dk1, _ = ops.attn_bwd(qk[:, :D], qk[:, D:], qkv[:, 2 * D:], o1, do1, lse1, B, H, d,
                                   a1.scale, dv=dqkv[:, 2 * D:], delta=delta1)
        del do1
        ops.qk_norm_rope_bwd(dq1, qkv[:, :D], a1.q_norm.weight, rq1, dk1, qkv[:, D:2 * D],
                             a1.k_norm.weight, rk1, sh.rope, dq_out=dqkv[:, :D],
                             dk_out=dqkv[:, D:2 * D])
        if full:  # attn1 q/k norm weights, to_q / to_k / to_v (fused dQKV^T . x1)
            ops.qk_norm_wgrad_into(dq1, qkv[:, :D], rq1, _pgrad(a1.q_norm.weight), dk1,
                                   qkv[:, D:2 * D], rk1, _pgrad(a1.k_norm.weight), rope=sh.rope)
            # one [3D, D] weight-gradient GEMM for q/k/v (they share x1), rounded to bf16 and
            # then added to each .grad: autograd's new_grad + AccumulateGrad roundings
            dwqkv = ops.wgrad(dqkv, x1)
            for i, lin in enumerate((a1.to_q, a1.to_k, a1.to_v)):
                ops.add_into(_pgrad(lin.weight), dwqkv[i * D:(i + 1) * D])
                ops.colsum_into(_pgrad(lin.bias), dqkv[:, i * D:(i + 1) * D])
            del dwqkv
        del dq1, dk1
        dh = None
        if ctx.needs_input_grad[4] or full:  # (blk, sh, keep, skip, h, ...)
            dx1 = ops.gemm(dqkv, W["qkv_wT"])
            g_prev = None if full else sh.ffgate.get(id(blk))
            if g_prev is not None:
                dh, d_ffo_prev = ops.rmsnorm_modulate_bwd(dx1, h, rstd1, onep[:, 1], ldm, rpm,
                                                          dres=dh1, gate=g_prev)
                sh.ffo_pre = (dh, d_ffo_prev)
                del d_ffo_prev
            else:
                dh = ops.rmsnorm_modulate_bwd(dx1, h, rstd1, onep[:, 1], ldm, rpm, dres=dh1)
            if full:  # shift_msa / scale_msa (attention.py:229-236)
                ops.colsum_into(dmods[:, 0], dx1, rows_per_group=rpm, sum_groups=False,
                                accumulate=False)
                ops.colsum_into(dmods[:, 1], dx1, h, rstd1, mode=2, rows_per_group=rpm,
                                sum_groups=False, accumulate=False)
        dm = dmods if full else None
        # every grad this block's backward writes straight into .grad (the LoRA adapters) is
        # enqueued now: tell the DP reducer (training.GradAllReduce), which can start their
        # bucket's all-reduce beside the remaining blocks' backward. With the text stack the
        # to_k / to_v adapters are finished later, by _TextStackFn.backward.
        done = None if tx is None else tx.token_params[tx.index[id(blk)]]
        for cb in getattr(blk, "_grad_ready_hooks", ()):
            cb(blk, done)
        return (None, None, None, None, dh, denc, dm, None, *grads_lora)


class _CaptionProjFn(torch.autograd.Function):
    """PixArtAlphaTextProjection (transformer3d.py:167-172, 494-499): Linear -> tanh-GELU ->
    Linear, trainable in lora_audio (training.py:69-73). Weight grads via transposed GEMMs."""

    @staticmethod
    def forward(ctx, enc, w1, b1, w2, b2):
        pre = torch.empty(enc.shape[0], w1.shape[0], dtype=torch.int16, device=enc.device)  # gelu' / 2 as int16 snorm
        act = ops.gemm(enc, w1, bias=b1, epilogue="gelu", aux0=pre)
        out = ops.gemm(act, w2, bias=b2)
        ctx.save_for_backward(enc, pre, act, w2)
        return out

    @staticmethod
    def backward(ctx, dout):
        enc, pre, act, w2 = ctx.saved_tensors
        dout = dout.contiguous()
        dw2 = ops.wgrad(dout, act)  # token-major operands, no transpose pass
        db2 = ops.colsum(dout)
        dpre = ops.gemm(dout, ops.transpose(w2), epilogue="gelu_bwd", aux0=pre)
        dw1 = ops.wgrad(dpre, enc)
        db1 = ops.colsum(dpre)
        return None, dw1, db1, dw2, db2


def _lora_ab(blk):
    """[A_q, B_q, A_k, B_k, A_v, B_v, A_o, B_o] adapter weights of attn2 (or [])."""
    lora = _lora_params(blk)
    ab = []
    if lora is not None:
        for m in lora:
            ab += _ab(m)
    return ab


def _text_kv(blk, sh, enc2, lora_ab):
    """attn2 K / V of the text tokens (attention.py:1004-1014 with the peft adapters of
    training.py:50-68, then the k RMSNorm): they depend only on enc2 and the block's weights, so
    _forward_tokens can compute them on a side stream one block ahead."""
    a2 = blk.attn2
    W = blk.packed()
    D = sh.D
    if lora_ab:
        lora = _lora_params(blk)
        _, _, Ak, _, Av, _, _, _ = lora_ab
        K2 = ops.lora_k2(lora[1].r)
        su = torch.empty(enc2.shape[0], 2 * K2, dtype=torch.bfloat16, device=enc2.device)
        u_k, _ = ops.lora_down(enc2, Ak, split=True, split_out=su[:, :K2])
        u_v, _ = ops.lora_down(enc2, Av, split=True, split_out=su[:, K2:])
        kv = ops.gemm(enc2, W["kv2_w"], bias=W["kv2_b"], ext=(su, _kv_ext(blk, lora[1], lora[2])[0]))
    else:
        u_k = u_v = None
        kv = ops.gemm(enc2, W["kv2_w"], bias=W["kv2_b"])
    k2raw, v2 = kv[:, :D], kv[:, D:]
    k2, _, rk2, _ = ops.qk_norm_rope_fwd(k2raw, None, a2.k_norm.weight, None, None, B=sh.Bt, N=sh.L)
    return k2raw, k2, rk2, v2, u_k, u_v


# training with LoRA: every block's attn2 text K/V (attention.py:1004-1014 + the to_k / to_v
# adapters, training.py:50-68) depends only on enc2, so all 28 are one launch each way instead of
# ~10 small M = L launches per block (LTX_TEXT_BATCH=0: per block, as before)
_TEXT_BATCH = os.environ.get("LTX_TEXT_BATCH", "1") != "0"
# the attention backward's delta = rowsum(dO*O) written by the dO GEMM's epilogue
# (LTX_EPI_STORE_ROWDOT) instead of a separate pass over dO and O (LTX_DELTA_FUSED=0: separate)
_DELTA_FUSED = os.environ.get("LTX_DELTA_FUSED", "1") != "0"
# LTX_TEXT_KNORM_GROUPED=0: the batched text side runs its attn2 k_norm per block (fwd and bwd)
_TEXT_KNORM_GROUPED = os.environ.get("LTX_TEXT_KNORM_GROUPED", "1") != "0"
# LTX_TEXT_BSUM_GROUPED=0: with the grouped k_norm and a shared prompt, the query-batch sums of the
# text-key gradients run per block (two launches each) instead of once for every block
_TEXT_BSUM_GROUPED = os.environ.get("LTX_TEXT_BSUM_GROUPED", "1") != "0"


class _TextStack:
    """The text side of every block's attn2 in one launch per kernel (LoRA training).

    Forward: the K/V projections of all blocks are ONE GEMM over the blocks' stacked [2D, D]
    weights, enc2 . [W_k1; W_v1; ...; W_kn; W_vn]^T + b, with each block's LoRA fused as its own
    K-extension (ltx_gemm_bf16_nt_gext: output columns of block i read the adapter operand
    columns of block i); the 2n lora_A products u = enc2 . A^T are one grouped lora_down.
    Backward: the blocks write their [dK_raw | dV] into one [Lt, n*2D] operand; after the last
    block (_TextStackFn.backward) the 2n lora_B grads, the 2n dgrads w = s*dY.B and the 2n lora_A
    grads are one grouped launch each, and the encoder gradient of all blocks is one GEMM with
    K = n*2D (plus every adapter's input-gradient term as K-extension): the f32 sum of the
    reference's per-block dX terms, rounded once."""

    def __init__(self, model, enc2):
        # built lazily by the first block_kv call (block 0's attn2): the cache validation and the
        # three launches then run on the host while block 0's attn1 keeps the device busy
        self.model, self.enc2 = model, enc2
        self.kv = None

    def _build(self):
        c = self.model._text_stack_cache()
        self.blocks, self.index = c["blocks"], c["index"]
        self.block_params, self.token_params = c["block_params"], c["token_params"]
        self.r, self.s, self.D = c["r"], c["s"], c["D"]
        self.w_all, self.b_all, self.wT_all = c["w"], c["b"], c["wT"]
        self.ext_f, self.ext_b, self.A_all, self.B_all = c["ext_f"], c["ext_b"], c["A"], c["B"]
        self.adapters = c["adapters"]
        enc2 = self.enc2
        n, D, r = len(self.blocks), self.D, self.r
        K2 = ops.lora_k2(r)
        self.K2 = K2
        Lt = enc2.shape[0]
        dev = enc2.device
        # u = enc2 . A^T of the 2n adapters (k of block i = adapter 2i, v = 2i+1) + their splits
        self.u = torch.empty(Lt, 2 * n * r, dtype=torch.float32, device=dev)
        su = torch.empty(Lt, 2 * n * K2, dtype=torch.bfloat16, device=dev)
        ops.lora_down(enc2, self.A_all[0], split=True, out=self.u[:, :r], split_out=su[:, :K2],
                      groups=2 * n, group_strides=(0, r * D, r, K2))
        self.kv = ops.gemm(enc2, self.w_all, bias=self.b_all, ext=(su, self.ext_f),
                           ext_group=(2 * D, 2 * K2))
        del su
        self.dkv = torch.empty(Lt, 2 * n * D, dtype=torch.bfloat16, device=dev)
        # the k_norm of every block's text keys: one grouped launch (bitwise the per-block calls)
        self.knw = self.model._text_knorm_weights(self.blocks, D)
        self.grouped_norm = self.knw is not None and _TEXT_KNORM_GROUPED
        self.dkvb = None  # [B*Lt, 2nD] per-query-batch [dK | dV] of every block (block_dkvb)
        if self.grouped_norm:
            self.k2_all, self.rk2_all = ops.qk_norm_fwd_grouped(self.kv, 2 * D, self.knw)
            self.dk2_all = torch.empty(n, Lt, D, dtype=torch.bfloat16, device=dev)

    def block_kv(self, blk, sh):
        """(k2raw, k2, rk2, v2, u_k, u_v) of one block: views of the stacked results + the k
        RMSNorm (per block: its weight)."""
        if self.kv is None:
            self._build()
        i, D, r = self.index[id(blk)], self.D, self.r
        k2raw = self.kv[:, 2 * i * D:(2 * i + 1) * D]
        v2 = self.kv[:, (2 * i + 1) * D:(2 * i + 2) * D]
        if self.grouped_norm:
            k2, rk2 = self.k2_all[i], self.rk2_all[i]
        else:
            k2, _, rk2, _ = ops.qk_norm_rope_fwd(k2raw, None, blk.attn2.k_norm.weight, None, None,
                                                 B=sh.Bt, N=sh.L)
        return (k2raw, k2, rk2, v2, self.u[:, 2 * i * r:(2 * i + 1) * r],
                self.u[:, (2 * i + 1) * r:(2 * i + 2) * r])

    def block_dkv(self, blk):
        i, D = self.index[id(blk)], self.D
        return self.dkv[:, 2 * i * D:2 * (i + 1) * D]

    def block_dkvb(self, blk, B):
        """(dK, dV) column views of this block in the [B*Lt, 2nD] stack of the per-query-batch
        text-key gradients (shared prompt, grouped_norm): _TextStack.backward sums the batches of
        every block in one launch instead of two per block"""
        n, D = len(self.blocks), self.D
        if self.dkvb is None:
            self.dkvb = torch.empty(B * self.kv.shape[0], 2 * n * D, dtype=torch.bfloat16,
                                    device=self.kv.device)
        i = self.index[id(blk)]
        return self.dkvb[:, 2 * i * D:(2 * i + 1) * D], self.dkvb[:, (2 * i + 1) * D:(2 * i + 2) * D]

    def block_dk2(self, blk):
        """this block's dK of the normalised text keys (grouped_norm: the input of the grouped
        k_norm backward)"""
        return self.dk2_all[self.index[id(blk)]]

    def backward(self):
        """Adapter grads of every block's to_k / to_v (into .grad) and the encoder gradient."""
        n, D, r, K2, s = len(self.blocks), self.D, self.r, self.K2, self.s
        enc2, dkv = self.enc2, self.dkv
        Lt = enc2.shape[0]
        dev = enc2.device
        if self.grouped_norm:  # every block's k_norm backward -> its dK_raw columns of dkv
            if self.dkvb is not None:
                # the query batches' [dK | dV] of every block in one sum: dkv's k columns then
                # hold each block's dK at the normalised keys, normalised in place below
                ops.batch_sum(self.dkvb, self.dkvb.shape[0] // Lt, out=dkv)
                ops.qk_norm_bwd_grouped(dkv, 2 * D, self.kv, 2 * D, self.knw, self.rk2_all, dkv, 2 * D)
            else:
                ops.qk_norm_bwd_grouped(self.dk2_all.view(n * Lt, D), Lt * D, self.kv, 2 * D, self.knw,
                                        self.rk2_all, dkv, 2 * D)
            # the stacked per-batch gradients are consumed: release them now (the [B*Lt, 2nD]
            # stack is ~470 MB at config A) instead of holding them until the next micro-step
            self.dkvb = None
            self.dk2_all = None
        # lora_B grads: dB_j = s * dY_j^T . u_j  (dY of adapter j = columns j*D .. of dkv)
        dB = ops.lora_wgrad(dkv[:, :D], self.u[:, :r], alpha=s, groups=2 * n,
                            group_strides=(D, r))
        # dgrads w_j = s * dY_j . B_j (+ their K-extension split)
        w = torch.empty(Lt, 2 * n * r, dtype=torch.float32, device=dev)
        sw = torch.empty(Lt, 2 * n * K2, dtype=torch.bfloat16, device=dev)
        ops.lora_down(dkv[:, :D], self.B_all[0], alpha=s, transposed=True, split=True,
                      out=w[:, :r], split_out=sw[:, :K2], groups=2 * n,
                      group_strides=(D, D * r, r, K2))
        # lora_A grads: dA_j = w_j^T . enc2
        dA = ops.lora_wgrad(enc2, w[:, :r], transpose_out=True, groups=2 * n, group_strides=(0, r))
        # into .grad (one multi-tensor add each; bitwise the per-block kernels' single-split adds)
        gB, gA = [], []
        for m in self.adapters:
            gB.append(_grad_buf(m, "B"))
            gA.append(_grad_buf(m, "A"))
        torch._foreach_add_(gB, list(dB.unbind(0)))
        torch._foreach_add_(gA, list(dA.unbind(0)))
        # encoder gradient of all blocks: sum_i [dK_raw_i | dV_i] . [W_k_i ; W_v_i] + adapters
        denc = ops.gemm(dkv, self.wT_all, ext=(sw, self.ext_b))
        for blk, ps in zip(self.blocks, self.block_params):
            for cb in getattr(blk, "_grad_ready_hooks", ()):
                cb(blk, ps)
        return denc


class _TextStackFn(torch.autograd.Function):
    """enc2 -> enc2 (an alias the blocks consume): autograd runs its backward once every block's
    backward has written its [dK_raw | dV] slice, and it returns the encoder gradient."""

    @staticmethod
    def forward(ctx, enc2, tx):
        ctx.tx = tx
        return enc2.view_as(enc2)

    @staticmethod
    def backward(ctx, denc_blocks):
        denc = ctx.tx.backward()
        ctx.tx = None
        return denc, None


# inference forwards compute the text K/V one block ahead on a side stream (LTX_TEXT_STREAM=0:
# inline). Measured: -2.5 % per denoising step; no gain in training (fwd or bwd), where the big
# GEMMs hold every CU and the main stream ends up waiting for the side stream.
_TEXT_STREAM = os.environ.get("LTX_TEXT_STREAM", "1") != "0"
_SIDE_STREAMS = {}


def _side_stream(device):
    key = str(device)
    if key not in _SIDE_STREAMS:
        _SIDE_STREAMS[key] = torch.cuda.Stream(device=device)
    return _SIDE_STREAMS[key]


def _lin_wgrad(dy, x):
    """nn.Linear weight grad dy^T . x over the rows (bf16, f32 accumulation)."""
    return ops.wgrad(dy.contiguous(), x.contiguous())


class _AdaModFn(torch.autograd.Function):
    """ada_values = scale_shift_table + tmod (attention.py:225-231; head: transformer3d.py:554-556,
    tmod broadcast over the P rows) -> (mods, 1 + mods on the scale rows). Differentiable for
    train_mode='full': d sst = sum over the batch, d tmod = d ada (or its sum over the P rows)."""

    @staticmethod
    def forward(ctx, sst, tmod, scale_mask, broadcast):
        mods, onep = ops.ada_modulation(sst, tmod, scale_mask, broadcast=broadcast)
        ctx.broadcast, ctx.P = broadcast, sst.shape[0]
        ctx.mark_non_differentiable(onep)
        return mods, onep

    @staticmethod
    def backward(ctx, dmods, donep):
        B, P, D = dmods.shape
        d = dmods.contiguous().view(B, P * D)
        dsst = ops.group_colsum(d).view(P, D)
        dtmod = ops.group_colsum(d.view(B * P, D), rows_per_group=P) if ctx.broadcast else d
        return dsst, dtmod, None, None


class _AdaLNFn(torch.autograd.Function):
    """AdaLayerNormSingle (transformer3d.py:473-491) with trainable weights (train_mode='full'):
    te -> linear_1 -> SiLU -> linear_2 = emb; SiLU(emb) -> linear = tmod. Backward: the small
    [B, *] GEMMs, SiLU backward kernels, weight grads over the B rows (zero-padded K)."""

    @staticmethod
    def forward(ctx, te, w1, b1, w2, b2, w, b):
        e1 = ops.gemm(te, w1, bias=b1)
        s1 = ops.silu(e1)
        emb = ops.gemm(s1, w2, bias=b2)
        s2 = ops.silu(emb)
        tmod = ops.gemm(s2, w, bias=b)
        ctx.save_for_backward(te, e1, s1, emb, s2, w2, w)
        return tmod, emb

    @staticmethod
    def backward(ctx, dtmod, demb):
        te, e1, s1, emb, s2, w2, w = ctx.saved_tensors
        dtmod = dtmod.contiguous()
        ds2 = ops.gemm(dtmod, ops.transpose(w))
        dw, db = _lin_wgrad(dtmod, s2), ops.colsum(dtmod)
        demb_t = ops.silu_bwd(emb, ds2, dres=None if demb is None else demb.contiguous())
        ds1 = ops.gemm(demb_t, ops.transpose(w2))
        dw2, db2 = _lin_wgrad(demb_t, s1), ops.colsum(demb_t)
        de1 = ops.silu_bwd(e1, ds1)
        dw1, db1 = _lin_wgrad(de1, te), ops.colsum(de1)
        return None, dw1, db1, dw2, db2, dw, db


class _HeadFn(torch.autograd.Function):
    """Output modulation + projection (transformer3d.py:553-561): LayerNorm (no affine,
    eps 1e-6) * (1 + scale) + shift, then proj_out. In train_mode='full' also the grads of the
    head's shift/scale rows (per batch) and of proj_out."""

    @staticmethod
    def forward(ctx, h, mod, onep, w, b, N, eps):
        ldm = mod.stride(0)
        y, mean, rstd = ops.layernorm_modulate_fwd(h, mod[:, 0], onep[:, 1], ldm, N, eps)
        out = ops.gemm(y, w, bias=b)
        ctx.save_for_backward(h, mean, rstd, mod, onep, w)
        ctx.N, ctx.eps = N, eps
        return out

    @staticmethod
    def backward(ctx, dout):
        h, mean, rstd, mod, onep, w = ctx.saved_tensors
        dout = dout.contiguous()
        wT = ops.transpose(w)
        dy = ops.gemm(dout, wT)
        dh = ops.layernorm_modulate_bwd(dy, h, mean, rstd, onep[:, 1], onep.stride(0), ctx.N)
        dmod = dw = db = None
        if ctx.needs_input_grad[1]:
            B = mod.shape[0]
            dmod = torch.empty(B, 2, h.shape[1], dtype=torch.bfloat16, device=h.device)
            ops.colsum_into(dmod[:, 0], dy, rows_per_group=ctx.N, sum_groups=False,
                            accumulate=False)
            ops.colsum_into(dmod[:, 1], dy, h, rstd, mean, mode=3, rows_per_group=ctx.N,
                            sum_groups=False, accumulate=False)
        if ctx.needs_input_grad[3]:
            y, _, _ = ops.layernorm_modulate_fwd(h, mod[:, 0], onep[:, 1], mod.stride(0), ctx.N,
                                                 ctx.eps)
            dw, db = _lin_wgrad(dout, y), ops.colsum(dout)
        return dh, dmod, None, dw, db, None, None


# ===============================================================================================
# the model
# ===============================================================================================
class Transformer3DModel(nn.Module):
    _supports_gradient_checkpointing = True

    def __init__(self, num_attention_heads: int = 16, attention_head_dim: int = 88,
                 in_channels: Optional[int] = None, out_channels: Optional[int] = None,
                 num_layers: int = 1, dropout: float = 0.0, norm_num_groups: int = 32,
                 cross_attention_dim: Optional[int] = None, attention_bias: bool = False,
                 num_vector_embeds: Optional[int] = None, activation_fn: str = "geglu",
                 num_embeds_ada_norm: Optional[int] = None, use_linear_projection: bool = False,
                 only_cross_attention: bool = False, double_self_attention: bool = False,
                 upcast_attention: bool = False, adaptive_norm: str = "single_scale_shift",
                 standardization_norm: str = "layer_norm", norm_elementwise_affine: bool = True,
                 norm_eps: float = 1e-5, attention_type: str = "default",
                 caption_channels: int = None, use_tpu_flash_attention: bool = False,
                 qk_norm: Optional[str] = None, positional_embedding_type: str = "rope",
                 positional_embedding_theta: Optional[float] = None,
                 positional_embedding_max_pos: Optional[List[int]] = None,
                 timestep_scale_multiplier: Optional[float] = None,
                 causal_temporal_positioning: bool = False,
                 patchifier: Optional[SymmetricPatchifier] = None):
        super().__init__()
        self.config = dict(
            num_attention_heads=num_attention_heads, attention_head_dim=attention_head_dim,
            in_channels=in_channels, out_channels=out_channels, num_layers=num_layers,
            dropout=dropout, norm_num_groups=norm_num_groups,
            cross_attention_dim=cross_attention_dim, attention_bias=attention_bias,
            num_vector_embeds=num_vector_embeds, activation_fn=activation_fn,
            num_embeds_ada_norm=num_embeds_ada_norm, use_linear_projection=use_linear_projection,
            only_cross_attention=only_cross_attention,
            double_self_attention=double_self_attention, upcast_attention=upcast_attention,
            adaptive_norm=adaptive_norm, standardization_norm=standardization_norm,
            norm_elementwise_affine=norm_elementwise_affine, norm_eps=norm_eps,
            attention_type=attention_type, caption_channels=caption_channels,
            use_tpu_flash_attention=use_tpu_flash_attention, qk_norm=qk_norm,
            positional_embedding_type=positional_embedding_type,
            positional_embedding_theta=positional_embedding_theta,
            positional_embedding_max_pos=positional_embedding_max_pos,
            timestep_scale_multiplier=timestep_scale_multiplier,
            causal_temporal_positioning=causal_temporal_positioning)
        if positional_embedding_type != "rope":
            raise ValueError("Absolute positional embedding is no longer supported")
        if positional_embedding_theta is None or positional_embedding_max_pos is None:
            raise ValueError("rope needs positional_embedding_theta and _max_pos")
        if use_tpu_flash_attention:
            raise NotImplementedError("TPU flash attention is out of scope on MI355X")
        self.use_tpu_flash_attention = False
        self.num_attention_heads = num_attention_heads
        self.attention_head_dim = attention_head_dim
        inner_dim = num_attention_heads * attention_head_dim
        self.inner_dim = inner_dim
        self.patchify_proj = nn.Linear(in_channels, inner_dim, bias=True)
        self.positional_embedding_type = positional_embedding_type
        self.positional_embedding_theta = positional_embedding_theta
        self.positional_embedding_max_pos = positional_embedding_max_pos
        self.use_rope = True
        self.timestep_scale_multiplier = timestep_scale_multiplier
        self.patchifier = patchifier
        self.transformer_blocks = nn.ModuleList([
            BasicTransformerBlock(inner_dim, num_attention_heads, attention_head_dim,
                                  cross_attention_dim=cross_attention_dim,
                                  activation_fn=activation_fn, attention_bias=attention_bias,
                                  norm_eps=norm_eps, qk_norm=qk_norm, use_rope=True,
                                  adaptive_norm=adaptive_norm,
                                  standardization_norm=standardization_norm,
                                  norm_elementwise_affine=norm_elementwise_affine)
            for _ in range(num_layers)])
        self.out_channels = in_channels if out_channels is None else out_channels
        self.norm_out = nn.LayerNorm(inner_dim, elementwise_affine=False, eps=1e-6)
        self.scale_shift_table = nn.Parameter(torch.randn(2, inner_dim) / inner_dim ** 0.5)
        self.proj_out = nn.Linear(inner_dim, self.out_channels)
        self.adaln_single = AdaLayerNormSingle(inner_dim)
        self.caption_projection = None
        if caption_channels is not None:
            self.caption_projection = PixArtAlphaTextProjection(caption_channels, inner_dim)
        self.gradient_checkpointing = False

    # ---- construction ----------------------------------------------------------------------
    @classmethod
    def from_config(cls, config: Dict[str, Any], **kwargs):
        import inspect
        merged = dict(config)
        merged.update(kwargs)
        accepted = inspect.signature(cls.__init__).parameters
        return cls(**{k: v for k, v in merged.items() if k in accepted and k != "self"})

    def load_state_dict(self, state_dict, *args, **kwargs):
        """Strips the ComfyUI 'model.diffusion_model.' prefix (transformer3d.py:279-292)."""
        if any(k.startswith("model.diffusion_model.") for k in state_dict):
            state_dict = {k.replace("model.diffusion_model.", ""): v for k, v in state_dict.items()
                          if k.startswith("model.diffusion_model.")}
        return super().load_state_dict(state_dict, *args, **kwargs)

    @classmethod
    def from_pretrained(cls, pretrained_model_path, *args, **kwargs):
        """Single-file safetensors with metadata['config'] = {"transformer": {...}}, or a
        diffusers-style directory with transformer/config.json (transformer3d.py:294-359)."""
        from safetensors import safe_open
        path = Path(pretrained_model_path)
        if path.is_dir():
            with open(path / "transformer" / "config.json") as f:
                config = json.load(f)
            if "positional_embedding_theta" not in config:
                config = OURS_TRANSFORMER_CONFIG  # the only diffusers config LTX maps
            state = {}
            for part in glob.glob(str(path / "transformer" / "diffusion_pytorch_model*.safetensors")):
                with safe_open(part, framework="pt", device="cpu") as f:
                    for k in f.keys():
                        state[k] = f.get_tensor(k)
            renamed = {}
            for k, v in state.items():
                nk = k
                for a, b in TRANSFORMER_KEYS_RENAME_DICT.items():
                    nk = nk.replace(a, b)
                renamed[nk] = v
            state = renamed
        elif path.is_file() and str(path).endswith(".safetensors"):
            state = {}
            with safe_open(str(path), framework="pt", device="cpu") as f:
                metadata = f.metadata()
                for k in f.keys():
                    state[k] = f.get_tensor(k)
            config = json.loads(metadata["config"])["transformer"]
        else:
            raise FileNotFoundError(str(path))
        with torch.device("meta"):
            model = cls.from_config(config)
        model.load_state_dict(state, assign=True, strict=True)
        patchifier = kwargs.get("patchifier")
        if patchifier is not None:
            model.patchifier = patchifier
        return model

    def _text_knorm_weights(self, blocks, D):
        """[n, D] stack of the blocks' attn2 k_norm weights for the grouped text k_norm (frozen in
        LoRA training: rebuilt only when one of them changes), or None when one is missing."""
        knws = [b.attn2.k_norm.weight for b in blocks]
        if not all(w is not None and w.dtype == torch.bfloat16 and w.numel() == D for w in knws):
            return None
        key = tuple((w.data_ptr(), w._version) for w in knws)
        c = getattr(self, "_knw_cache", None)
        if c is None or c[0] != key:
            c = (key, torch.stack([w.detach() for w in knws]).contiguous())
            self._knw_cache = c
        return c[1]

    def _text_structure(self):
        """Module-structure facts of the batched text side, cached on the identity of every
        block's attn2 projections and the trainability of the K/V base weights (cheap to check;
        the per-block lists below cost ~3 ms of host time to rebuild): None when the text side
        cannot be batched, else the blocks, their (k, v) adapters and parameter lists."""
        blocks = list(self.transformer_blocks)
        if not (_TEXT_BATCH and blocks):
            return None
        lins = [_lora_params(b) for b in blocks]
        if any(l is None for l in lins):
            return None
        key = tuple((id(l[1]), id(l[2]), _base(l[1])._parameters["weight"].requires_grad,
                     _base(l[2])._parameters["weight"].requires_grad) for l in lins)
        c = getattr(self, "_tx_struct", None)
        if c is not None and c[0] == key:
            return c[1]
        r, sc = lins[0][1].r, lins[0][1].scaling
        # grouped K-extension columns: one block's [k | v] outputs = 2D, a multiple of 256
        ok = (2 * blocks[0].attn2.inner_dim) % 256 == 0 and all(
            l[1].r == r and l[2].r == r and l[1].scaling == sc and l[2].scaling == sc
            and not k[2] and not k[3] for l, k in zip(lins, key))
        st = None
        if ok:
            # per block: the to_k / to_v adapter weights (finished by _TextStack.backward) and
            # the rest of its trainable parameters (finished by its own backward)
            block_params = [list(_ab(l[1]) + _ab(l[2])) for l in lins]
            text_ids = {id(p) for ps in block_params for p in ps}
            st = {"blocks": blocks, "lins": lins, "adapters": [m for l in lins for m in (l[1], l[2])],
                  "index": {id(b): i for i, b in enumerate(blocks)}, "block_params": block_params,
                  "token_params": [[p for p in b.parameters() if id(p) not in text_ids]
                                   for b in blocks],
                  "text_ids": text_ids, "r": r, "s": sc, "D": blocks[0].attn2.inner_dim}
        self._tx_struct = (key, st)
        return st

    def _text_batchable(self):
        """The batched text side (_TextStack) applies with LoRA on every block's attn2 and frozen
        K/V base weights (lora_audio training)."""
        return self._text_structure() is not None

    @torch.no_grad()
    def _text_stack_cache(self):
        """Stacked operands of _TextStack, rebuilt when a block's packed weights or an adapter
        change: [2nD, D] K/V weights, bias, their [D, 2nD] transpose, the forward K-extension
        weights [2nD, 2 K2] (each block's block-diagonal split(s B_k) | split(s B_v)), the
        backward ones [D, 2n K2], and the f32 adapters A [2n, r, D], B [2n, D, r]."""
        st = self._text_structure()
        blocks, lins, adapters = st["blocks"], st["lins"], st["adapters"]
        packs = [b.packed() for b in blocks]
        exts = [_kv_ext(b, l[1], l[2]) for b, l in zip(blocks, lins)]
        abs_ = [t for m in adapters for t in _ab(m)]
        key = (tuple(id(pk) for pk in packs), tuple(id(e[0]) for e in exts),
               tuple((t.data_ptr(), t._version) for t in abs_), ops.weight_generation())
        c = getattr(self, "_tx_cache", None)
        if c is not None and c["key"] == key:
            return c
        base_key = tuple(id(pk) for pk in packs)
        if c is not None and c["base_key"] == base_key:
            w, b, wT = c["w"], c["b"], c["wT"]
        else:
            self._tx_cache = None  # drop the old stacks before building new ones
            w = torch.cat([pk["kv2_w"] for pk in packs], 0)
            b = torch.cat([pk["kv2_b"] for pk in packs], 0)
            wT = torch.cat([pk["kv2_wT"] for pk in packs], 1)
        c = dict(st)
        c.update({"key": key, "base_key": base_key, "w": w, "b": b, "wT": wT,
                  "ext_f": torch.cat([e[0] for e in exts], 0),
                  "ext_b": torch.cat([e[1] for e in exts], 1),
                  "A": torch.stack([_ab(m)[0] for m in adapters]),
                  "B": torch.stack([_ab(m)[1] for m in adapters])})
        self._tx_cache = c
        return c

    def grad_ready_order(self):
        """The trainable parameters in the order the backward finishes their gradients: the
        blocks' own parameters from the last block to the first (their grads are complete when
        that block's backward returns), then everything upstream of the blocks (caption
        projection, AdaLN-single, patchify_proj) and the head. training.GradAllReduce buckets in
        this order so the first buckets can be reduced while the backward still runs."""
        seen, order = set(), []
        # with the batched text side the to_k / to_v adapters finish after the last block
        st = self._text_structure()
        late = st["text_ids"] if st is not None else set()
        for blk in reversed(self.transformer_blocks):
            for p in blk.parameters():
                if p.requires_grad and id(p) not in seen and id(p) not in late:
                    seen.add(id(p))
                    order.append(p)
        for blk in reversed(self.transformer_blocks):
            for p in blk.parameters():
                if p.requires_grad and id(p) not in seen:
                    seen.add(id(p))
                    order.append(p)
        for p in self.parameters():
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                order.append(p)
        return order

    @property
    def dtype(self):
        return self.patchify_proj.weight.dtype

    @property
    def device(self):
        return self.patchify_proj.weight.device

    def _set_gradient_checkpointing(self, module, value=False):
        if hasattr(module, "gradient_checkpointing"):
            module.gradient_checkpointing = value

    def create_skip_layer_mask(self, batch_size, num_conds, ptb_index, skip_block_list=None):
        """transformer3d.py:187-203 (used by the inference pipeline's STG)."""
        if skip_block_list is None or len(skip_block_list) == 0:
            return None
        mask = torch.ones((len(self.transformer_blocks), batch_size * num_conds),
                          device=self.device, dtype=self.dtype)
        for block_idx in skip_block_list:
            mask[block_idx, ptb_index::num_conds] = 0
        return mask

    def get_fractional_positions(self, indices_grid):
        return torch.stack([indices_grid[:, i] / self.positional_embedding_max_pos[i]
                            for i in range(3)], dim=-1)

    # ---- forward ---------------------------------------------------------------------------
    def forward(self, hidden_states, indices_grid, ref_image_hidden_states=None,
                pose_hidden_states=None, encoder_hidden_states=None, timestep=None,
                class_labels=None, cross_attention_kwargs=None, attention_mask=None,
                encoder_attention_mask=None, skip_layer_mask=None, skip_layer_strategy=None,
                return_dict=True):
        """transformer3d.py:361-565: the training call and the inference call (timestep [B],
        [B,1] or per token [B,N]; float pixel-coordinate indices_grid; skip_layer_mask
        [num_layers, B] with a SkipLayerStrategy -- forward only). Does not mutate
        `hidden_states` (the reference lerps into it in place, transformer3d.py:447-466)."""
        _lib.ensure_device(hidden_states.device)
        if attention_mask is not None:
            raise NotImplementedError("self-attention masks are not used on the LTX paths")
        dt = torch.bfloat16
        if ref_image_hidden_states is None or pose_hidden_states is None:
            raise ValueError("the avatar model conditions on ref_image_hidden_states and pose_hidden_states")
        # conditioning lerp (transformer3d.py:447-466), out of place
        x_in = ops.condition_lerp(hidden_states.to(dt), ref_image_hidden_states.to(dt),
                                  pose_hidden_states.to(dt))
        out = self._forward_tokens(x_in, indices_grid, encoder_hidden_states, timestep,
                                   encoder_attention_mask, skip_layer_mask, skip_layer_strategy)
        if not return_dict:
            return (out,)
        return Transformer3DModelOutput(sample=out)

    def _forward_tokens(self, x_in, indices_grid, encoder_hidden_states, timestep,
                        encoder_attention_mask=None, skip_layer_mask=None,
                        skip_layer_strategy=None):
        """Everything after the conditioning lerp: patchify_proj, AdaLN-single, RoPE, caption
        projection, the block stack and the output head. x_in [B, N, C] bf16 -> [B, N, C_out]."""
        B, N, C = x_in.shape
        D = self.inner_dim
        H = self.num_attention_heads
        dt = torch.bfloat16
        if self.dtype != dt:
            raise TypeError("the MI355X path computes in bf16: call model.to(torch.bfloat16)")
        # one prompt expanded over the batch (stride-0 views, as train_step passes it): run the
        # text side once; the cross-attention reads the shared K/V for every sample
        m = encoder_attention_mask
        text_shared = (B > 1 and encoder_hidden_states.stride(0) == 0
                       and (m is None or m.shape[0] == 1 or m.stride(0) == 0))
        if text_shared:
            encoder_hidden_states = encoder_hidden_states[:1]
            m = None if m is None else m[:1]
        Bt = 1 if text_shared else B
        # encoder mask -> additive bias (transformer3d.py:441-445): (1 - m) * -10000 in bf16
        enc_bias = None
        if m is not None:
            if m.ndim == 2:
                enc_bias = ((1 - m.to(dt)) * -10000.0).float().contiguous()
            else:
                enc_bias = m.reshape(Bt, -1).float().contiguous()
        # per-token timesteps (inference with conditioning latents, pipeline_ltx_video.py:1190-1195)
        per_token = timestep.numel() != B
        if per_token and timestep.numel() != B * N:
            raise ValueError(f"timestep has {timestep.numel()} values for batch {B} x {N} tokens")
        keep = torch.is_grad_enabled()
        # train_mode='full' (training.py:75-91): AdaLN-single, every scale_shift_table, the
        # attention weights and proj_out train
        full = keep and self.adaln_single.linear.weight.requires_grad
        with torch.no_grad():
            h = ops.gemm(x_in.reshape(B * N, C), self.patchify_proj.weight,
                         bias=self.patchify_proj.bias)
        if full:
            ad = self.adaln_single
            mult = float(self.timestep_scale_multiplier or 1.0)
            te = ops.timestep_embedding(timestep.reshape(-1).float().contiguous(), mult)
            tmod, emb = _AdaLNFn.apply(te, ad.emb.timestep_embedder.linear_1.weight,
                                       ad.emb.timestep_embedder.linear_1.bias,
                                       ad.emb.timestep_embedder.linear_2.weight,
                                       ad.emb.timestep_embedder.linear_2.bias, ad.linear.weight,
                                       ad.linear.bias)
        else:
            with torch.no_grad():
                tmod, emb = self._adaln(timestep)
        rope = ops.RopeSpec(indices_grid, D, self.positional_embedding_theta,
                            self.positional_embedding_max_pos)
        enc = encoder_hidden_states.to(dt)
        L = enc.shape[1]
        enc2d = enc.reshape(Bt * L, enc.shape[2]).contiguous()
        cp = self.caption_projection
        enc2 = _CaptionProjFn.apply(enc2d, cp.linear_1.weight, cp.linear_1.bias,
                                    cp.linear_2.weight, cp.linear_2.bias)
        eps = self.transformer_blocks[0].norm_eps if len(self.transformer_blocks) else 1e-6
        sh = _Shared(B, N, L, H, self.attention_head_dim, rope, enc_bias, eps, text_shared,
                     per_token)
        sh.full = full
        ckpt = self.training and self.gradient_checkpointing and keep
        # the stack's backward (adapter grads of every to_k / to_v) runs as the backward of enc2,
        # so it needs enc2 in the graph: with a frozen caption_projection the per-block text path
        # computes those adapter grads instead
        if keep and not full and enc2.requires_grad and self._text_batchable():
            sh.text_stack = _TextStack(self, enc2)
            enc2 = _TextStackFn.apply(enc2, sh.text_stack)
        strat = None
        if skip_layer_mask is not None and skip_layer_strategy is not None:
            strat = SkipLayerStrategy[skip_layer_strategy.name] if isinstance(
                skip_layer_strategy, Enum) else SkipLayerStrategy[str(skip_layer_strategy)]
            if strat is SkipLayerStrategy.Residual:  # acts only with residual_connection (False)
                strat = None
        blocks = list(self.transformer_blocks)
        if _TEXT_STREAM and not keep and h.is_cuda and len(blocks) > 1:
            # inference: text K/V of block i+1 on a side stream while block i runs (the small
            # M = L GEMM, LoRA and norm launches fill CUs the main stream leaves idle)
            side = _side_stream(h.device)
            main = torch.cuda.current_stream()
            sh.text_pre = {}

            def prep(j):
                bj = blocks[j]
                with torch.no_grad():  # weight caches are built on the main stream
                    bj.packed()
                    lj = _lora_params(bj)
                    if lj is not None:
                        _kv_ext(bj, lj[1], lj[2])
                # the side stream starts only after everything main has enqueued so far: enc2 and
                # the caches just (re)built above (cold cache, or after an optimizer step)
                ready = torch.cuda.Event()
                ready.record(main)
                with torch.no_grad(), torch.cuda.stream(side):
                    side.wait_event(ready)
                    vals = _text_kv(bj, sh, enc2, _lora_ab(bj))
                    ev = torch.cuda.Event()
                    ev.record(side)
                for t in vals:
                    if t is not None:
                        t.record_stream(main)
                sh.text_pre[id(bj)] = (vals, ev)
            prep(0)
        else:
            prep = None
        fuse_gate = keep and not ckpt and not full and strat is None and \
            os.environ.get("LTX_FFGATE_FUSED", "1") != "0"
        prev_gate = None
        for i, blk in enumerate(self.transformer_blocks):
            if prep is not None and i + 1 < len(blocks):
                prep(i + 1)
            skip = None if strat is None else (skip_layer_mask[i].to(dt).contiguous(), strat)
            if full:
                mods, onep = _AdaModFn.apply(blk.scale_shift_table, tmod, (1 << 1) | (1 << 4),
                                             False)
            else:
                with torch.no_grad():
                    mods, onep = ops.ada_modulation(blk.scale_shift_table, tmod,
                                                    (1 << 1) | (1 << 4))
            ab = _lora_ab(blk)
            if fuse_gate:
                if prev_gate is not None:
                    sh.ffgate[id(blk)] = prev_gate
                prev_gate = mods[:, 5]
            if ckpt:
                h = torch.utils.checkpoint.checkpoint(
                    lambda *a, _b=blk, _s=skip: _BlockFn.apply(_b, sh, True, _s, *a),
                    h, enc2, mods, onep, *ab, use_reentrant=False)
            else:
                h = _BlockFn.apply(blk, sh, keep, skip, h, enc2, mods, onep, *ab)
        if full:
            hmod, honep = _AdaModFn.apply(self.scale_shift_table, emb, 1 << 1, True)
        else:
            with torch.no_grad():
                hmod, honep = ops.ada_modulation(self.scale_shift_table, emb, 1 << 1,
                                                 broadcast=True)
        out = _HeadFn.apply(h, hmod, honep, self.proj_out.weight, self.proj_out.bias, sh.rpm, 1e-6)
        return out.view(B, N, self.out_channels)

    def _adaln(self, timestep):
        """AdaLayerNormSingle (transformer3d.py:473-491) of timestep.flatten(): returns
        (tmod [T,6D], emb [T,D]), T = B (one timestep per sample) or B*N (per token)."""
        mult = float(self.timestep_scale_multiplier or 1.0)
        ad = self.adaln_single
        te = ops.timestep_embedding(timestep.reshape(-1).float().contiguous(), mult)
        e1 = ops.gemm(te, ad.emb.timestep_embedder.linear_1.weight,
                      bias=ad.emb.timestep_embedder.linear_1.bias)
        emb = ops.gemm(ops.silu(e1), ad.emb.timestep_embedder.linear_2.weight,
                       bias=ad.emb.timestep_embedder.linear_2.bias)
        tmod = ops.gemm(ops.silu(emb), ad.linear.weight, bias=ad.linear.bias)
        return tmod, emb
