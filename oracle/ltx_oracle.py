"""CPU restatement of the reference training hot path -- TEST INFRASTRUCTURE / CPU BASELINE ONLY.

Header (read me): this module is the parity ORACLE for the MI355X build. Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it, and only as the
checker (or as the timed CPU "port" baseline) -- never as the thing measured or shipped. The
product package (video-generation-for-human-avatars_amd/ltx_amd) never imports it and fails
loudly when its HIP library is missing.

It restates, op for op and in the reference's eager dtypes, the path that
``ltx_video/training.py:94-166`` (train_step) drives through
``Transformer3DModel.forward`` (transformer3d.py:361-565) and ``BasicTransformerBlock.forward``
(attention.py:198-321), including the third-party pieces the reference imports (diffusers 0.35.1
RMSNorm / AdaLayerNormSingle / PixArtAlphaTextProjection / GELU, peft 0.17.1 LoRA Linear).
Parity of THIS module with the reference is pinned by tests/test_oracle_golden.py against the
golden vectors generated from the reference itself (oracle/gen_golden.py).

Everything is functional over a flat ``params`` dict keyed by the reference's parameter names
(peft's ``base_layer`` level removed: ``transformer_blocks.0.attn2.to_q.weight``,
``transformer_blocks.0.attn2.to_q.lora_A.default.weight`` ...). Device-agnostic: the GPU tests
also run it on ``cuda`` in fp32 / bf16 as the torch reference for the HIP kernels.
"""
import math

import torch
import torch.nn.functional as F


# ----------------------------------------------------------------------------------------------
# patchifier  (symmetric_patchifier.py:33-84, patch size 1)
# ----------------------------------------------------------------------------------------------
def latent_coords(f, h, w, b, device="cpu"):
    """[b, 3, f*h*w] int64 (t, h, w), w fastest (symmetric_patchifier.py:33-51)."""
    grid = torch.meshgrid(torch.arange(f, device=device), torch.arange(h, device=device),
                          torch.arange(w, device=device), indexing="ij")
    coords = torch.stack(grid, dim=0).reshape(3, f * h * w)
    return coords.unsqueeze(0).repeat(b, 1, 1)


def patchify(latents):
    """[B,C,F,H,W] -> ([B,F*H*W,C], coords) (symmetric_patchifier.py:55-65)."""
    b, c, f, h, w = latents.shape
    tokens = latents.permute(0, 2, 3, 4, 1).reshape(b, f * h * w, c)
    return tokens, latent_coords(f, h, w, b, latents.device)


def unpatchify(tokens, h, w, c):
    """[B,N,C] -> [B,C,F,H,W] (symmetric_patchifier.py:67-84)."""
    b, n, _ = tokens.shape
    f = n // (h * w)
    return tokens.reshape(b, f, h, w, c).permute(0, 4, 1, 2, 3)


# ----------------------------------------------------------------------------------------------
# rectified flow (rf.py:376-426, training.py:124-146)
# ----------------------------------------------------------------------------------------------
def sample_timesteps(batch, mu=-0.5, sigma=1.0, qmin=0.005, qmax=0.999, device="cpu"):
    """training.py:124-132: LogNormal draw, r/(1+r), clamp to the batch quantiles."""
    logn = torch.distributions.LogNormal(torch.tensor(mu, device=device),
                                         torch.tensor(sigma, device=device))
    raw = logn.sample((batch,))
    t_raw = raw / (1 + raw)
    lo = torch.quantile(t_raw, qmin)
    hi = torch.quantile(t_raw, qmax)
    return t_raw.clamp(min=float(lo), max=float(hi))


def add_noise(x0, noise, t):
    """rf.py:376-386 (append_dims, torch_utils.py:16-25): fp32 via type promotion."""
    s = t.reshape(t.shape + (1,) * (x0.ndim - t.ndim))
    return (1 - s) * x0 + s * noise


def velocity_target(x0, noise, t):
    """rf.py:400-426: alpha_dot = -1, sigma_dot = +1 (fp32 tensors -> promotion)."""
    a_dot = torch.full_like(t, -1.0)
    s_dot = torch.full_like(t, 1.0)
    while a_dot.dim() < x0.dim():
        a_dot = a_dot.unsqueeze(-1)
        s_dot = s_dot.unsqueeze(-1)
    return a_dot * x0 + s_dot * noise


# ----------------------------------------------------------------------------------------------
# primitive ops in the reference's dtypes
# ----------------------------------------------------------------------------------------------
def rmsnorm(x, eps, weight=None):
    """diffusers 0.35.1 RMSNorm (attention.py:117-119, 434-436)."""
    var = x.to(torch.float32).pow(2).mean(-1, keepdim=True)
    y = x * torch.rsqrt(var + eps)
    if weight is not None:
        if weight.dtype in (torch.float16, torch.bfloat16):
            y = y.to(weight.dtype)
        return y * weight
    return y.to(x.dtype)


def linear(x, p, name):
    return F.linear(x, p[name + ".weight"], p.get(name + ".bias"))


def lora_linear(x, p, name, scaling):
    """peft 0.17.1 lora.Linear.forward with fp32 adapters (training.py:50-68)."""
    result = linear(x, p, name)
    a = p.get(name + ".lora_A.default.weight")
    if a is None:
        return result
    b = p[name + ".lora_B.default.weight"]
    result_dtype = result.dtype
    xa = x.to(a.dtype)
    result = result + F.linear(F.linear(xa, a), b) * scaling
    return result.to(result_dtype)


def rope_freqs(indices_grid, dim, theta, max_pos, out_dtype):
    """Transformer3DModel.precompute_freqs_cis, spacing='exp' (transformer3d.py:209-277)."""
    frac = torch.stack([indices_grid[:, i] / max_pos[i] for i in range(3)], dim=-1)
    dtype = torch.float32
    idx = theta ** torch.linspace(math.log(1, theta), math.log(theta, theta), dim // 6,
                                  device=frac.device, dtype=dtype)
    idx = idx.to(dtype)
    idx = idx * math.pi / 2
    freqs = (idx * (frac.unsqueeze(-1) * 2 - 1)).transpose(-1, -2).flatten(2)
    cos = freqs.cos().repeat_interleave(2, dim=-1)
    sin = freqs.sin().repeat_interleave(2, dim=-1)
    if dim % 6 != 0:
        cos = torch.cat([torch.ones_like(cos[:, :, : dim % 6]), cos], dim=-1)
        sin = torch.cat([torch.zeros_like(cos[:, :, : dim % 6]), sin], dim=-1)
    return cos.to(out_dtype), sin.to(out_dtype)


def apply_rotary_emb(x, cos, sin):
    """attention.py:917-932: interleaved pairs (2i, 2i+1) -> (-x[2i+1], x[2i])."""
    x2 = x.unflatten(-1, (-1, 2))
    t1, t2 = x2.unbind(-1)
    rot = torch.stack((-t2, t1), dim=-1).flatten(-2)
    return x * cos + rot * sin


def timestep_embedding(t, dim=256, max_period=10000):
    """diffusers get_timestep_embedding(flip_sin_to_cos=True, downscale_freq_shift=0)
    (same formula as ltx_video/models/transformers/embeddings.py:10-50)."""
    half = dim // 2
    exponent = -math.log(max_period) * torch.arange(0, half, dtype=torch.float32, device=t.device)
    exponent = exponent / half
    emb = t[:, None].float() * torch.exp(exponent)[None, :]
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=-1)
    return torch.cat([emb[:, half:], emb[:, :half]], dim=-1)


def adaln_single(p, t, dtype):
    """diffusers AdaLayerNormSingle (transformer3d.py:160-165, 481-491)."""
    proj = timestep_embedding(t).to(dtype)
    e = linear(proj, p, "adaln_single.emb.timestep_embedder.linear_1")
    e = linear(F.silu(e), p, "adaln_single.emb.timestep_embedder.linear_2")
    return linear(F.silu(e), p, "adaln_single.linear"), e


def caption_projection(p, enc):
    """diffusers PixArtAlphaTextProjection (transformer3d.py:167-172, 494-499)."""
    h = linear(enc, p, "caption_projection.linear_1")
    h = F.gelu(h, approximate="tanh")
    return linear(h, p, "caption_projection.linear_2")


# ----------------------------------------------------------------------------------------------
# attention + block
# ----------------------------------------------------------------------------------------------
SKIP_STRATEGIES = ("AttentionSkip", "AttentionValues", "Residual", "TransformerBlock")


def attention(p, name, x, heads, freqs=None, enc=None, mask_bias=None, lora_scaling=1.0,
              skip_mask=None, skip_strategy=None):
    """Attention + AttnProcessor2_0.__call__ (attention.py:935-1114). skip_mask [B] (this block's
    row of the skip-layer mask) blends the SDPA output before to_out (attention.py:1071-1085):
    AttentionSkip with the processor input, AttentionValues with to_v's output. Residual only
    acts when attn.residual_connection (False in LTX: a no-op, attention.py:1103-1110)."""
    B = x.shape[0]
    q = lora_linear(x, p, name + ".to_q", lora_scaling)
    q = rmsnorm(q, 1e-5, p[name + ".q_norm.weight"])
    src = x if enc is None else enc
    k = lora_linear(src, p, name + ".to_k", lora_scaling)
    k = rmsnorm(k, 1e-5, p[name + ".k_norm.weight"])
    if enc is None and freqs is not None:
        k = apply_rotary_emb(k, *freqs)
        q = apply_rotary_emb(q, *freqs)
    v = lora_linear(src, p, name + ".to_v", lora_scaling)
    value_for_stg = v
    hd = k.shape[-1] // heads
    q = q.view(B, -1, heads, hd).transpose(1, 2)
    k = k.view(B, -1, heads, hd).transpose(1, 2)
    v = v.view(B, -1, heads, hd).transpose(1, 2)
    mask = None
    if mask_bias is not None:  # prepare_attention_mask (attention.py:836-877) -> [B,H,1,L]
        mask = mask_bias.repeat_interleave(heads, dim=0).view(B, heads, -1, mask_bias.shape[-1])
    o = F.scaled_dot_product_attention(q, k, v, attn_mask=mask, dropout_p=0.0, is_causal=False)
    o = o.transpose(1, 2).reshape(B, -1, heads * hd).to(q.dtype)
    if skip_mask is not None:
        m = skip_mask.reshape(B, 1, 1)
        if skip_strategy == "AttentionSkip":
            o = o * m + x * (1.0 - m)
        elif skip_strategy == "AttentionValues":
            o = o * m + value_for_stg * (1.0 - m)
    return lora_linear(o, p, name + ".to_out.0", lora_scaling)


def block(p, i, h, freqs, enc, enc_bias, tmod, heads, lora_scaling=1.0, eps=1e-6,
          skip_mask=None, skip_strategy=None):
    """BasicTransformerBlock.forward (attention.py:198-321), single_scale_shift, rms_norm;
    skip_mask [B] is passed to attn1 only, TransformerBlock blends the block output with its
    input (attention.py:312-319)."""
    pre = f"transformer_blocks.{i}"
    B = h.shape[0]
    original = h
    n = rmsnorm(h, eps)
    sst = p[pre + ".scale_shift_table"]
    ada = sst[None, None] + tmod.reshape(B, tmod.shape[1], 6, -1)
    sh_msa, sc_msa, g_msa, sh_mlp, sc_mlp, g_mlp = ada.unbind(dim=2)
    n = n * (1 + sc_msa) + sh_msa
    n = n.squeeze(1)
    a = attention(p, pre + ".attn1", n, heads, freqs=freqs, lora_scaling=lora_scaling,
                  skip_mask=skip_mask, skip_strategy=skip_strategy)
    h = g_msa * a + h
    a = attention(p, pre + ".attn2", h, heads, enc=enc, mask_bias=enc_bias,
                  lora_scaling=lora_scaling)
    h = a + h
    n = rmsnorm(h, eps)
    n = n * (1 + sc_mlp) + sh_mlp
    f = linear(n, p, pre + ".ff.net.0.proj")
    f = F.gelu(f, approximate="tanh")
    f = linear(f, p, pre + ".ff.net.2")
    h = g_mlp * f + h
    if skip_mask is not None and skip_strategy == "TransformerBlock":
        m = skip_mask.view(-1, 1, 1)
        h = h * m + original * (1.0 - m)
    return h


def forward(p, cfg, hidden_states, indices_grid, ref_image_hidden_states, pose_hidden_states,
            encoder_hidden_states, timestep, encoder_attention_mask=None, lora_scaling=1.0,
            skip_layer_mask=None, skip_layer_strategy=None):
    """Transformer3DModel.forward (transformer3d.py:361-565): timestep [B], [B,1] or per token
    [B,N]; skip_layer_mask [num_layers, B] with a SkipLayerStrategy name (inference / STG).
    Does NOT mutate ``hidden_states`` (the reference does, in place, transformer3d.py:447-466)."""
    dtype = p["patchify_proj.weight"].dtype
    heads = cfg["num_attention_heads"]
    D = heads * cfg["attention_head_dim"]
    enc_bias = None
    if encoder_attention_mask is not None and encoder_attention_mask.ndim == 2:
        enc_bias = ((1 - encoder_attention_mask.to(hidden_states.dtype)) * -10000.0).unsqueeze(1)
    elif encoder_attention_mask is not None:
        enc_bias = encoder_attention_mask
    H, W = ref_image_hidden_states.shape[3], ref_image_hidden_states.shape[4]
    x = unpatchify(hidden_states.clone(), H, W, hidden_states.shape[-1])
    x[:, :, 0:1] = torch.lerp(x[:, :, 0:1], ref_image_hidden_states, 0.85)
    x[:, :, 1:] = torch.lerp(x[:, :, 1:], pose_hidden_states[:, :, 1:], 0.5)
    x, _ = patchify(x)
    h = linear(x, p, "patchify_proj")
    timestep = cfg.get("timestep_scale_multiplier", 1000) * timestep
    freqs = rope_freqs(indices_grid, D, cfg["positional_embedding_theta"],
                       cfg["positional_embedding_max_pos"], dtype)
    B = h.shape[0]
    tmod, emb = adaln_single(p, timestep.flatten(), h.dtype)
    tmod = tmod.view(B, -1, tmod.shape[-1])
    emb = emb.view(B, -1, emb.shape[-1])
    enc = caption_projection(p, encoder_hidden_states).view(B, -1, D)
    for i in range(cfg["num_layers"]):
        h = block(p, i, h, freqs, enc, enc_bias, tmod, heads, lora_scaling,
                  eps=cfg.get("norm_eps", 1e-6),
                  skip_mask=None if skip_layer_mask is None else skip_layer_mask[i],
                  skip_strategy=skip_layer_strategy)
    ssv = p["scale_shift_table"][None, None] + emb[:, :, None]
    shift, scale = ssv[:, :, 0], ssv[:, :, 1]
    h = F.layer_norm(h, (D,), eps=1e-6)
    h = h * (1 + scale) + shift
    return linear(h, p, "proj_out")


def train_step(p, cfg, latents, ref_image_latents, pose_latents, prompt_embeds,
               prompt_attention_mask, t=None, noise=None, lora_scaling=1.0, loss_weight=1.0,
               rf=None):
    """training.py:94-166. If ``t``/``noise`` are None they are drawn exactly as the reference
    draws them (LogNormal sample, then randn_like), so a shared seed reproduces the reference."""
    dtype = p["patchify_proj.weight"].dtype
    latents = latents.to(dtype)
    ref_image_latents = ref_image_latents.to(dtype)
    pose_latents = pose_latents.to(dtype)
    B = latents.shape[0]
    enc = prompt_embeds.expand(B, -1, -1).to(dtype)
    enc_mask = prompt_attention_mask.expand(B, -1)
    tokens, coords = patchify(latents)
    rf = rf or {}
    if t is None:
        t = sample_timesteps(B, rf.get("mu", -0.5), rf.get("sigma", 1.0), rf.get("qmin", 0.005),
                             rf.get("qmax", 0.999), device=latents.device)
    if noise is None:
        noise = torch.randn_like(tokens)
    x_t = add_noise(tokens, noise, t).to(dtype)
    v = velocity_target(tokens, noise, t).to(dtype)
    out = forward(p, cfg, x_t, coords, ref_image_latents, pose_latents, enc, t, enc_mask,
                  lora_scaling)
    std = v.std()
    mse = F.mse_loss(out, v, reduction="mean")
    loss = float(loss_weight) * mse
    rel = loss / (std ** 2 + 1e-12)
    nrmse = torch.sqrt(loss) / (std + 1e-12)
    return {"loss": loss, "rel_mse": rel, "nrmse": nrmse, "sample": out, "t": t, "noise": noise,
            "x_t": x_t, "v_target": v, "coords": coords}


# ----------------------------------------------------------------------------------------------
# inference denoising step
# ----------------------------------------------------------------------------------------------
def pixel_coords(latent_coords, scale_factors=(8, 32, 32), causal_fix=True):
    """latent_to_pixel_coords_from_factors (ltx_video/models/autoencoders/vae_encode.py:215-226)."""
    pc = latent_coords * torch.tensor(scale_factors, device=latent_coords.device)[None, :, None]
    if causal_fix:
        pc[:, 0] = (pc[:, 0] + 1 - scale_factors[0]).clamp(min=0)
    return pc


def fractional_coords(pixel, frame_rate):
    """pipeline_ltx_video.py:1121-1122: float pixel coordinates, time axis / frame_rate."""
    f = pixel.to(torch.float32)
    f[:, 0] = f[:, 0] * (1.0 / frame_rate)
    return f


def linear_quadratic_schedule(num_steps, threshold_noise=0.025, linear_steps=None):
    """rf.py:25-46."""
    if num_steps == 1:
        return torch.tensor([1.0])
    if linear_steps is None:
        linear_steps = num_steps // 2
    lin = [i * threshold_noise / linear_steps for i in range(linear_steps)]
    diff = linear_steps - threshold_noise * num_steps
    qsteps = num_steps - linear_steps
    qcoef = diff / (linear_steps * qsteps ** 2)
    lcoef = threshold_noise / linear_steps - 2 * diff / (qsteps ** 2)
    const = qcoef * (linear_steps ** 2)
    quad = [qcoef * (i ** 2) + lcoef * i + const for i in range(linear_steps, num_steps)]
    sched = [1.0 - x for x in lin + quad + [1.0]]
    return torch.tensor(sched[:-1])


def rf_step(model_output, timestep, sample, timesteps, t_eps=1e-6):
    """RectifiedFlowScheduler.step, deterministic branch (rf.py:305-374): Euler to the next lower
    scheduled timestep, global (0-dim t) or per token ([B,N] t)."""
    padded = torch.cat([timesteps, torch.zeros(1, device=timesteps.device)])
    if timestep.ndim == 0:
        lower = padded[padded < timestep - t_eps][0]
        dt = timestep - lower
    else:
        lower_mask = padded[:, None, None] < timestep[None] - t_eps
        lower, _ = (lower_mask * padded[:, None, None]).max(dim=0)
        dt = (timestep - lower)[..., None]
    return sample - dt * model_output


def denoising_step(latents, noise_pred, current_timestep, conditioning_mask, t, timesteps,
                   t_eps=1e-6):
    """LTXVideoPipeline.denoising_step (pipeline_ltx_video.py:1346-1379)."""
    den = rf_step(noise_pred, t if current_timestep is None else current_timestep, latents,
                  timesteps)
    if conditioning_mask is None:
        return den
    keep = (t - t_eps < (1.0 - conditioning_mask)).unsqueeze(-1)
    return torch.where(keep, den, latents)


def guidance(noise_pred, batch_size, do_cfg, do_stg, guidance_scale=1.0, stg_scale=0.0,
             rescaling_scale=1.0, cfg_star_rescale=False):
    """CFG / CFG* / STG / rescaling of the batched prediction (pipeline_ltx_video.py:1229-1268),
    in the prediction's dtype (eager bf16 ops)."""
    num_conds = 1 + int(do_cfg) + int(do_stg)
    chunks = noise_pred.chunk(num_conds)
    if do_stg:
        text, perturb = chunks[-2:]
    if do_cfg:
        uncond, text = chunks[:2]
        if cfg_star_rescale:
            pf = text.view(batch_size, -1)
            nf = uncond.view(batch_size, -1)
            dot = torch.sum(pf * nf, dim=1, keepdim=True)
            sq = torch.sum(nf ** 2, dim=1, keepdim=True) + 1e-8
            alpha = dot / sq
            uncond = alpha * uncond
        out = uncond + guidance_scale * (text - uncond)
    elif do_stg:
        out = text
    else:
        out = noise_pred
    if do_stg:
        out = out + stg_scale * (text - perturb)
        if rescaling_scale != 1.0 and stg_scale > 0.0:
            text_std = text.view(batch_size, -1).std(dim=1, keepdim=True)
            out_std = out.view(batch_size, -1).std(dim=1, keepdim=True)
            factor = text_std / out_std
            factor = rescaling_scale * factor + (1 - rescaling_scale)
            out = out * factor.view(batch_size, 1, 1)
    return out


def trainable_names(names):
    """apply_training_strategy('lora_audio') (training.py:50-74)."""
    return [n for n in names if ("lora_" in n) or ("caption_projection" in n)]


def param_shapes(cfg, lora_rank=16):
    """Flat name -> shape map for a Transformer3DModel config (parameter names as the
    reference's module tree + peft produce them, base_layer level removed)."""
    heads, hd = cfg["num_attention_heads"], cfg["attention_head_dim"]
    D = heads * hd
    cin = cfg["in_channels"]
    cout = cfg.get("out_channels") or cin
    cap = cfg["caption_channels"]
    ff = 4 * D
    s = {"patchify_proj.weight": (D, cin), "patchify_proj.bias": (D,),
         "scale_shift_table": (2, D), "proj_out.weight": (cout, D), "proj_out.bias": (cout,),
         "adaln_single.emb.timestep_embedder.linear_1.weight": (D, 256),
         "adaln_single.emb.timestep_embedder.linear_1.bias": (D,),
         "adaln_single.emb.timestep_embedder.linear_2.weight": (D, D),
         "adaln_single.emb.timestep_embedder.linear_2.bias": (D,),
         "adaln_single.linear.weight": (6 * D, D), "adaln_single.linear.bias": (6 * D,),
         "caption_projection.linear_1.weight": (D, cap),
         "caption_projection.linear_1.bias": (D,),
         "caption_projection.linear_2.weight": (D, D), "caption_projection.linear_2.bias": (D,)}
    for i in range(cfg["num_layers"]):
        pre = f"transformer_blocks.{i}"
        s[pre + ".scale_shift_table"] = (6, D)
        for a in ("attn1", "attn2"):
            for lin in ("to_q", "to_k", "to_v", "to_out.0"):
                s[f"{pre}.{a}.{lin}.weight"] = (D, D)
                s[f"{pre}.{a}.{lin}.bias"] = (D,)
                if a == "attn2" and lora_rank:
                    s[f"{pre}.{a}.{lin}.lora_A.default.weight"] = (lora_rank, D)
                    s[f"{pre}.{a}.{lin}.lora_B.default.weight"] = (D, lora_rank)
            s[f"{pre}.{a}.q_norm.weight"] = (D,)
            s[f"{pre}.{a}.k_norm.weight"] = (D,)
        s[pre + ".ff.net.0.proj.weight"] = (ff, D)
        s[pre + ".ff.net.0.proj.bias"] = (ff,)
        s[pre + ".ff.net.2.weight"] = (D, ff)
        s[pre + ".ff.net.2.bias"] = (D,)
    return s


def make_params(cfg, seed, dtype=torch.bfloat16, lora_rank=16, device="cpu",
                requires_grad=True):
    """Parameters drawn with oracle/params.py (same values the goldens used)."""
    from params import init_value  # oracle/params.py
    out = {}
    for name, shape in param_shapes(cfg, lora_rank).items():
        v = init_value(name, shape, seed)
        v = v.to(torch.float32 if "lora_" in name else dtype).to(device)
        if requires_grad and (("lora_" in name) or ("caption_projection" in name)):
            v.requires_grad_(True)
        out[name] = v
    return out
