"""Helpers shared by the model-level tests and smoke(): build the MI355X Transformer3DModel from a
flat parameter dict keyed by the reference's canonical names (golden vectors / oracle params)."""
import torch

from params import canonical_name


def build_model(cfg, params, lora_rank=16, device="cuda"):
    from ltx_amd.config import TrainConfig
    from ltx_amd.lora import apply_training_strategy
    from ltx_amd.transformer3d import Transformer3DModel
    from ltx_amd.patchifier import SymmetricPatchifier
    with torch.device("meta"):
        m = Transformer3DModel.from_config(cfg)
        if lora_rank:
            apply_training_strategy(m, TrainConfig(checkpoint_path="-", lora_rank=lora_rank,
                                                   lora_alpha=lora_rank), "lora_audio")
    sd = {}
    for name, _ in m.named_parameters():
        sd[name] = params[canonical_name(name)].detach().to(device).clone()
    m.load_state_dict(sd, assign=True, strict=True)
    for n, p in m.named_parameters():
        p.requires_grad_(("lora_" in n) or ("caption_projection" in n))
    m.patchifier = SymmetricPatchifier(1)
    return m


def grads_by_canonical(model):
    return {canonical_name(n): p.grad for n, p in model.named_parameters() if p.requires_grad}


def rel(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / (b.norm() + 1e-30))


FULL_KEYS = ("proj_out", "scale_shift_table", "adaln_single", "caption_projection", "attn")


def build_full_model(cfg, params, device="cuda"):
    """The model with apply_training_strategy('full') (training.py:75-91: attention weights,
    biases and q/k norms, every scale_shift_table, adaln_single, caption_projection, proj_out)."""
    from ltx_amd.config import TrainConfig
    from ltx_amd.lora import apply_training_strategy
    from ltx_amd.patchifier import SymmetricPatchifier
    from ltx_amd.transformer3d import Transformer3DModel
    with torch.device("meta"):
        m = Transformer3DModel.from_config(cfg)
    m.load_state_dict({n: params[canonical_name(n)].detach().to(device).clone()
                       for n, _ in m.named_parameters()}, assign=True, strict=True)
    apply_training_strategy(m, TrainConfig(checkpoint_path="-"), "full")
    m.patchifier = SymmetricPatchifier(1)
    m.train()
    return m


def noise_crit(name, build, ref16, ref32, factor=1.25, slack=2e-3):
    """err(build_bf16, ref_fp32) <= factor * err(ref_bf16, ref_fp32) + slack."""
    e_b, e_r = rel(build.float(), ref32.float()), rel(ref16.float(), ref32.float())
    assert e_b <= factor * e_r + slack, f"{name}: build err {e_b:.3e} vs reference bf16 noise {e_r:.3e}"
    return e_b, e_r


def loss_crit(name, lb, l16, l32):
    """SURVEY 8(c)-4 on the loss (training.py:159-166): the build's f32 mse within 1e-3 relative
    of the fp32 reference, or within 1.25x the reference's own bf16 distance from it."""
    lb, l16, l32 = float(lb), float(l16), float(l32)
    e_b, e_r = abs(lb - l32) / abs(l32), abs(l16 - l32) / abs(l32)
    assert e_b <= max(1e-3, 1.25 * e_r + 1e-4), f"{name}: loss {lb} vs fp32 {l32} (bf16 ref {l16})"
    return e_b, e_r


def synth_inputs(B, F_, H_, W_, L, n_valid, seed, device="cuda"):
    """Seeded synthetic train_step inputs (latents / pose / ref / one prompt with n_valid tokens)
    plus explicit t and noise, as the oracle takes them (t and noise as inputs)."""
    g = torch.Generator(device=device).manual_seed(seed)
    d = {"in.latents": torch.randn(B, 128, F_, H_, W_, generator=g, device=device),
         "in.ref_image_latents": torch.randn(B, 128, 1, H_, W_, generator=g, device=device),
         "in.pose_latents": torch.randn(B, 128, F_, H_, W_, generator=g, device=device),
         "in.prompt_embeds": torch.randn(1, L, 4096, generator=g, device=device),
         "in.prompt_attention_mask": (torch.arange(L, device=device) < n_valid).long().view(1, L),
         "out.t": torch.rand(B, generator=g, device=device) * 0.9 + 0.05}
    d["out.noise"] = torch.randn(B, F_ * H_ * W_, 128, generator=g, device=device).bfloat16()
    return d


def oracle_step(params, cfg, d, dtype, trainable, device="cuda"):
    """The pinned oracle's train step (oracle/ltx_oracle.py) on the device in `dtype` (LoRA
    adapters always f32, as peft keeps them): (sample, {name: grad}, f32 mse loss)."""
    import ltx_oracle as O
    q = {k: v.detach().to(device).to(torch.float32 if ("lora_" in k or dtype == torch.float32) else dtype)
         .requires_grad_(trainable(k)) for k, v in params.items()}
    r = O.train_step(q, cfg, d["in.latents"], d["in.ref_image_latents"], d["in.pose_latents"],
                     d["in.prompt_embeds"], d["in.prompt_attention_mask"], t=d["out.t"],
                     noise=d["out.noise"].to(dtype))
    r["loss"].backward()
    loss32 = float(((r["sample"].float() - r["v_target"].float()) ** 2).mean())
    return r["sample"].detach(), {k: v.grad for k, v in q.items() if v.requires_grad}, loss32


def build_step(model, d, accum=1):
    """The build's train_step on the inputs of synth_inputs: the f32 mse (before the bf16 loss
    rounding), gradients left in .grad."""
    from ltx_amd.config import TrainConfig
    from ltx_amd.scheduler import RectifiedFlowScheduler
    from ltx_amd.training import train_step
    tc = TrainConfig(checkpoint_path="-", gradient_accumulation_steps=accum)
    _, _, _, ld = train_step(model, {"latents": d["in.latents"], "ref_image_latents": d["in.ref_image_latents"],
                                     "pose_latents": d["in.pose_latents"]},
                             RectifiedFlowScheduler(), model.patchifier, tc, d["in.prompt_embeds"],
                             d["in.prompt_attention_mask"], t=d["out.t"], noise=d["out.noise"])
    return float(ld["_mse_f32"])


def is_lora_trainable(name):
    return ("lora_" in name) or ("caption_projection" in name)


def is_full_trainable(name):
    return any(k in name for k in FULL_KEYS)
