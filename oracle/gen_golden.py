"""Generate the golden vectors under tests/golden/ by running the REFERENCE itself.

TEST INFRASTRUCTURE -- runs only in the build container (where /root/reference exists). It puts
the test-only third-party shim (oracle/shim: diffusers 0.35.1 / peft 0.17.1 restatements, no-op
wandb) ahead of /root/reference on sys.path and imports the reference modules UNMODIFIED.
Only the resulting data files (inputs + expected outputs) are committed; nothing from the
reference travels to the GPU box.

    python oracle/gen_golden.py            # regenerates every fixture

Fixtures (safetensors + a JSON sidecar each):
  tiny_train_step   config T: 2 layers, 4x32 heads, in 128, caption 64, 4 prompt tokens,
                    latents [2,128,2,8,8] (pose lerp exercised). Reference
                    ltx_video/training.py:94-166 train_step (seeded) + loss.backward():
                    captured model inputs (t, noise, x_t, v), out.sample, loss/rel_mse/nrmse,
                    grads of every trainable param (LoRA r=16 A/B fp32, caption_projection bf16),
                    plus the same forward in fp32 (reference noise floor).
  ltx2b_block       LTX-2B widths (D 2048, 32x64 heads, caption 4096), ONE block, latents
                    [1,128,2,4,4], 8 prompt tokens. Weights are NOT stored: they are re-drawn from
                    oracle/params.py (seed recorded) and pinned by a SHA-256. Stores out.sample,
                    loss, LoRA grads, caption-projection bias grads and weight-grad row/col sums.
  rope_2b           precompute_freqs_cis (transformer3d.py:221-277) at D 2048 for int latent
                    coords (training) and float pixel coords (inference), cos/sin bf16.
  patchify          SymmetricPatchifier coords + permutation (symmetric_patchifier.py:33-84).
  rf_sched          RectifiedFlowScheduler add_noise / build_velocity_target / shift_timesteps
                    (rf.py:216-225, 376-426) and the train_step t-sampling (training.py:124-132).
  train_config      load_train_config_from_yaml(configs/train-avatars.yaml) (config.py:62-154).
  infer_step        inference call of the tiny model (CFG+STG batch of 3, float pixel coords,
                    per-token timesteps, every SkipLayerStrategy) and RectifiedFlowScheduler
                    set_timesteps / step, global and per-token (rf.py:179-374).
  tiny_full_step    train_mode='full' step of the tiny model (no LoRA; attention, AdaLN, norms,
                    scale-shift tables, caption projection, proj_out trainable): all grads.
  ckpt_export       save_training_checkpoint of the tiny model: lora_audio (peft merge) and full
                    (state dict) safetensors, tensors + metadata (torch_utils.py:39-133).
  attn_processor    the reference Attention + AttnProcessor2_0 of the tiny model's block 0 (self
                    with RoPE; cross with mask bias + peft LoRA): outputs and input/LoRA grads.

    python oracle/gen_golden.py attn       # regenerates one fixture (gen_<name>)
"""
import dataclasses
import json
import os
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")

sys.path.insert(0, os.path.join(HERE, "shim"))
sys.path.insert(1, REF)
sys.path.insert(2, HERE)

import torch  # noqa: E402
from safetensors.torch import save_file  # noqa: E402

# training.py:21 imports validate_epoch, which drags in the pipeline + VAE; the hot path never
# calls it, so register an inert module under that name before importing the trainer.
_val = types.ModuleType("ltx_video.validation")
_val.validate_epoch = None
sys.modules["ltx_video.validation"] = _val

import ltx_video.training as T  # noqa: E402
from ltx_video.config import load_train_config_from_yaml  # noqa: E402
from ltx_video.models.transformers.symmetric_patchifier import SymmetricPatchifier  # noqa: E402
from ltx_video.models.transformers.transformer3d import Transformer3DModel  # noqa: E402
from ltx_video.schedulers.rf import RectifiedFlowScheduler  # noqa: E402
from ltx_video.utils.diffusers_config_mapping import OURS_TRANSFORMER_CONFIG  # noqa: E402

import params as P  # noqa: E402

TINY_CONFIG = dict(OURS_TRANSFORMER_CONFIG)
TINY_CONFIG.update(num_attention_heads=4, attention_head_dim=32, caption_channels=64,
                   cross_attention_dim=128, num_layers=2)
BLOCK2B_CONFIG = dict(OURS_TRANSFORMER_CONFIG)
BLOCK2B_CONFIG.update(num_layers=1)


def _save(name, tensors, meta):
    os.makedirs(OUT, exist_ok=True)
    tensors = {k: v.detach().cpu().clone().contiguous() for k, v in tensors.items()}
    save_file(tensors, os.path.join(OUT, f"{name}.safetensors"))
    with open(os.path.join(OUT, f"{name}.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    size = sum(t.numel() * t.element_size() for t in tensors.values())
    print(f"  {name}: {len(tensors)} tensors, {size/1e6:.2f} MB")


def _train_cfg(rank):
    cfg = load_train_config_from_yaml(os.path.join(REF, "configs", "train-avatars.yaml"))
    cfg.lora_rank = rank
    cfg.lora_alpha = rank
    cfg.gradient_accumulation_steps = 1
    return cfg


def _build(model_cfg, seed, dtype, rank):
    pf = SymmetricPatchifier(patch_size=1)
    model = Transformer3DModel.from_config(model_cfg)
    model.patchifier = pf
    P.init_module_(model, seed, dtype=dtype)
    model = T.apply_training_strategy(model, _train_cfg(rank), "lora_audio")
    P.init_module_(model, seed, dtype=dtype)  # LoRA adapters now exist: A/B per params.py
    return model, pf


def _capture_train_step(model, pf, batch, prompt, mask, seed, rank):
    """Run the reference train_step (training.py:94-166) under a fixed seed, capturing the
    scheduler inputs and the model's call arguments with hooks (no reference code is edited)."""
    sch = RectifiedFlowScheduler(num_train_timesteps=1000, shifting=None, base_resolution=1024,
                                 sampler="Uniform")
    cap = {}
    add_noise = sch.add_noise

    def add_noise_hook(original_samples, noise, timesteps):
        cap["tokens"] = original_samples.clone()
        cap["noise"] = noise.clone()
        cap["t"] = timesteps.clone()
        return add_noise(original_samples=original_samples, noise=noise, timesteps=timesteps)

    sch.add_noise = add_noise_hook
    core = model.base_model.model if hasattr(model, "base_model") else model

    def pre_hook(mod, args, kwargs):
        # forward mutates hidden_states in place (transformer3d.py:447-466): clone first
        cap["hidden_states"] = kwargs["hidden_states"].clone()
        cap["indices_grid"] = kwargs["indices_grid"].clone()
        cap["encoder_attention_mask"] = kwargs["encoder_attention_mask"].clone()

    def post_hook(mod, args, kwargs, out):
        cap["sample"] = out.sample.detach().clone()

    h1 = core.register_forward_pre_hook(pre_hook, with_kwargs=True)
    h2 = core.register_forward_hook(post_hook, with_kwargs=True)
    torch.manual_seed(seed)
    loss, rel_mse, nrmse, loss_dict = T.train_step(model, batch, sch, pf, _train_cfg(rank), prompt,
                                                   mask, "cpu")
    h1.remove()
    h2.remove()
    loss.backward()
    cap["loss"] = loss.detach().reshape(1)
    cap["rel_mse"] = rel_mse.detach().reshape(1)
    cap["nrmse"] = nrmse.detach().reshape(1)
    cap["v_target"] = sch.build_velocity_target(cap["tokens"], cap["noise"], cap["t"]).to(
        cap["sample"].dtype)
    return cap


def _grads(model):
    out = {}
    for n, p in model.named_parameters():
        if p.requires_grad:
            out[P.canonical_name(n)] = p.grad.detach().clone()
    return out


def gen_tiny():
    seed, rank, B = 1234, 16, 2
    g = torch.Generator().manual_seed(99)
    batch = {
        "latents": torch.randn(B, 128, 2, 8, 8, generator=g),
        "ref_image_latents": torch.randn(B, 128, 1, 8, 8, generator=g),
        "pose_latents": torch.randn(B, 128, 2, 8, 8, generator=g),
    }
    prompt = torch.randn(1, 4, 64, generator=g)
    mask = torch.tensor([[1, 1, 1, 0]], dtype=torch.long)
    model, pf = _build(TINY_CONFIG, seed, torch.bfloat16, rank)
    cap = _capture_train_step(model, pf, batch, prompt, mask, seed=4321, rank=rank)
    grads = _grads(model)
    # fp32 reference of the same forward (same weights, same captured inputs): noise floor
    m32, _ = _build(TINY_CONFIG, seed, torch.float32, rank)
    with torch.no_grad():
        enc = prompt.expand(B, -1, -1).float()
        out32 = m32(hidden_states=cap["hidden_states"].float(), indices_grid=cap["indices_grid"],
                    ref_image_hidden_states=batch["ref_image_latents"].float(),
                    pose_hidden_states=batch["pose_latents"].float(),
                    encoder_hidden_states=enc, timestep=cap["t"],
                    encoder_attention_mask=cap["encoder_attention_mask"]).sample
    tensors = {f"in.{k}": v for k, v in batch.items()}
    tensors["in.prompt_embeds"] = prompt
    tensors["in.prompt_attention_mask"] = mask
    for k in ("tokens", "noise", "t", "hidden_states", "indices_grid", "sample", "loss",
              "rel_mse", "nrmse", "v_target"):
        tensors[f"out.{k}"] = cap[k]
    tensors["out.sample_fp32"] = out32
    for k, v in grads.items():
        tensors[f"grad.{k}"] = v
    weights = {P.canonical_name(n): p.detach().clone() for n, p in model.named_parameters()}
    for k, v in weights.items():
        tensors[f"w.{k}"] = v
    meta = {"config": TINY_CONFIG, "param_seed": seed, "train_seed": 4321, "lora_rank": rank,
            "lora_alpha": rank, "weights_sha256": P.weights_sha256(model),
            "source": "reference ltx_video/training.py:94-166 train_step via oracle/shim"}
    _save("tiny_train_step", tensors, meta)


def gen_block2b():
    seed, rank, B = 2025, 16, 1
    g = torch.Generator().manual_seed(7)
    batch = {
        "latents": torch.randn(B, 128, 2, 4, 4, generator=g),
        "ref_image_latents": torch.randn(B, 128, 1, 4, 4, generator=g),
        "pose_latents": torch.randn(B, 128, 2, 4, 4, generator=g),
    }
    prompt = torch.randn(1, 8, 4096, generator=g)
    mask = torch.tensor([[1, 1, 1, 1, 1, 0, 0, 0]], dtype=torch.long)
    model, pf = _build(BLOCK2B_CONFIG, seed, torch.bfloat16, rank)
    cap = _capture_train_step(model, pf, batch, prompt, mask, seed=99, rank=rank)
    grads = _grads(model)
    tensors = {f"in.{k}": v for k, v in batch.items()}
    tensors["in.prompt_embeds"] = prompt
    tensors["in.prompt_attention_mask"] = mask
    for k in ("tokens", "noise", "t", "hidden_states", "indices_grid", "sample", "loss",
              "rel_mse", "nrmse", "v_target"):
        tensors[f"out.{k}"] = cap[k]
    for k, v in grads.items():
        if "lora_" in k or v.ndim == 1:
            tensors[f"grad.{k}"] = v
        else:  # caption_projection weight grads are 8M/4M elements: keep row and column sums
            tensors[f"gradsum0.{k}"] = v.float().sum(0)
            tensors[f"gradsum1.{k}"] = v.float().sum(1)
    meta = {"config": BLOCK2B_CONFIG, "param_seed": seed, "train_seed": 99, "lora_rank": rank,
            "lora_alpha": rank, "weights_sha256": P.weights_sha256(model),
            "source": "reference ltx_video/training.py:94-166 train_step via oracle/shim"}
    _save("ltx2b_block", tensors, meta)


def gen_rope():
    model = Transformer3DModel.from_config(BLOCK2B_CONFIG)
    model = model.to(torch.bfloat16)
    pf = SymmetricPatchifier(1)
    _, coords = pf.get_latent_coords(13, 24, 24, 1, "cpu"), None
    coords = pf.get_latent_coords(13, 24, 24, 1, "cpu")
    pick = torch.tensor([0, 1, 23, 24, 575, 576, 4000, 7487])
    grid_int = coords[:, :, pick]
    cos_i, sin_i = model.precompute_freqs_cis(grid_int)
    # inference-style fractional pixel coordinates (pipeline_ltx_video.py:1118-1124)
    grid_f = grid_int.float() * torch.tensor([8.0, 32.0, 32.0]).view(1, 3, 1)
    grid_f[:, 0] = (grid_f[:, 0] + 1 - 8).clamp(min=0) / 25.0
    cos_f, sin_f = model.precompute_freqs_cis(grid_f)
    _save("rope_2b", {"grid_int": grid_int, "cos_int": cos_i, "sin_int": sin_i,
                      "grid_float": grid_f, "cos_float": cos_f, "sin_float": sin_f},
          {"dim": 2048, "theta": 10000.0, "max_pos": [20, 2048, 2048],
           "source": "transformer3d.py:221-277"})


def gen_patchify():
    pf = SymmetricPatchifier(1)
    out = {}
    for (b, c, f, h, w) in [(2, 3, 3, 4, 5), (1, 8, 7, 16, 16), (2, 4, 1, 8, 8)]:
        x = torch.arange(b * c * f * h * w, dtype=torch.float32).reshape(b, c, f, h, w)
        tok, coords = pf.patchify(x)
        key = f"{b}x{c}x{f}x{h}x{w}"
        out[f"tokens.{key}"] = tok
        out[f"coords.{key}"] = coords
        out[f"unpatch.{key}"] = pf.unpatchify(tok.contiguous(), h, w, c)
    _save("patchify", out, {"source": "symmetric_patchifier.py:33-84"})


def gen_rf():
    g = torch.Generator().manual_seed(5)
    x0 = torch.randn(3, 64, 16, generator=g).to(torch.bfloat16)
    eps = torch.randn(3, 64, 16, generator=g).to(torch.bfloat16)
    t = torch.tensor([0.05, 0.5, 0.93])
    sch = RectifiedFlowScheduler(num_train_timesteps=1000, shifting=None, base_resolution=1024)
    out = {"x0": x0, "eps": eps, "t": t,
           "x_t": sch.add_noise(original_samples=x0, noise=eps, timesteps=t),
           "v": sch.build_velocity_target(x0, eps, t),
           "shift_none": sch.shift_timesteps(x0.shape, t)}
    sd3 = RectifiedFlowScheduler(shifting="SD3", target_shift_terminal=0.1)
    out["shift_sd3"] = sd3.shift_timesteps(torch.Size([3, 4096, 128]), t)
    sdiff = RectifiedFlowScheduler(shifting="SimpleDiffusion", base_resolution=1024)
    out["shift_simple"] = sdiff.shift_timesteps(torch.Size([3, 4096, 128]), t)
    # train_step t sampling (training.py:124-132) for B = 8 under a seed
    cfg = _train_cfg(16)
    torch.manual_seed(31337)
    logn = torch.distributions.LogNormal(torch.tensor(cfg.rf_log_normal_mu),
                                         torch.tensor(cfg.rf_log_normal_sigma))
    raw = logn.sample((8,))
    t_raw = raw / (1 + raw)
    lo = torch.quantile(t_raw, cfg.rf_quantile_min)
    hi = torch.quantile(t_raw, cfg.rf_quantile_max)
    out["tsample_raw"] = raw
    out["tsample_t"] = t_raw.clamp(min=float(lo), max=float(hi))
    _save("rf_sched", out, {"source": "rf.py:216-225,376-426; training.py:124-132",
                            "tsample_seed": 31337})


def gen_infer():
    """Inference path: one denoising step's transformer call as
    pipeline_ltx_video.py:1089-1228 makes it -- CFG + STG batch of 3 (uncond, cond, perturbed),
    float pixel coordinates / frame_rate, per-token timesteps min(t, 1 - conditioning_mask), a
    skip-layer mask for block 1 of the perturbed batch -- through the reference
    Transformer3DModel.forward for every SkipLayerStrategy; plus RectifiedFlowScheduler
    set_timesteps / step (rf.py:179-374), global and per-token."""
    from ltx_video.utils.skip_layer_strategy import SkipLayerStrategy

    def latent_to_pixel_coords_from_factors(latent_coords, scale_factors, causal_fix=False):
        # vae_encode.py:215-226 (its module imports the VAE, which the shim does not provide)
        pixel_coords = latent_coords * torch.tensor(scale_factors)[None, :, None]
        if causal_fix:
            pixel_coords[:, 0] = (pixel_coords[:, 0] + 1 - scale_factors[0]).clamp(min=0)
        return pixel_coords

    seed, rank, frame_rate = 1234, 16, 25.0
    model, pf = _build(TINY_CONFIG, seed, torch.bfloat16, rank)
    core = model.base_model.model
    core.eval()
    g = torch.Generator().manual_seed(2024)
    F_, H_, W_ = 2, 8, 8
    latents = torch.randn(1, 128, F_, H_, W_, generator=g)
    tokens, lat_coords = pf.patchify(latents)
    ref = torch.randn(1, 128, 1, H_, W_, generator=g)
    pose = torch.randn(1, 128, F_, H_, W_, generator=g)
    neg = torch.randn(1, 4, 64, generator=g)
    pos = torch.randn(1, 4, 64, generator=g)
    nc = 3
    enc = torch.cat([neg, pos, pos]).to(torch.bfloat16)
    enc_mask = torch.tensor([[1, 1, 0, 0], [1, 1, 1, 0], [1, 1, 1, 0]], dtype=torch.long)
    pixel = latent_to_pixel_coords_from_factors(lat_coords, (8, 32, 32), causal_fix=True)
    frac = torch.cat([pixel] * nc).to(torch.float32)
    frac[:, 0] = frac[:, 0] * (1.0 / frame_rate)
    cond_mask = torch.zeros(1, tokens.shape[1])
    cond_mask[:, : H_ * W_] = 1.0  # first latent frame hard-conditioned
    t = torch.tensor(0.7)
    ts_global = t[None].expand(nc).unsqueeze(-1)
    ts_tok = torch.min(ts_global, 1.0 - torch.cat([cond_mask] * nc))
    skip = core.create_skip_layer_mask(1, nc, nc - 1, [1])
    x = torch.cat([tokens] * nc).to(torch.bfloat16)
    kw = dict(indices_grid=frac, ref_image_hidden_states=torch.cat([ref] * nc).to(torch.bfloat16),
              pose_hidden_states=torch.cat([pose] * nc).to(torch.bfloat16),
              encoder_hidden_states=enc, encoder_attention_mask=enc_mask, return_dict=False)
    out = {"in.tokens": x, "in.indices_grid": frac, "in.ref": kw["ref_image_hidden_states"],
           "in.pose": kw["pose_hidden_states"], "in.enc": enc, "in.enc_mask": enc_mask,
           "in.ts_global": ts_global, "in.ts_tok": ts_tok, "in.skip_layer_mask": skip,
           "in.pixel_coords": pixel, "in.cond_mask": cond_mask}
    with torch.no_grad():
        out["out.global"] = core(hidden_states=x.clone(), timestep=ts_global, **kw)[0]
        out["out.tok"] = core(hidden_states=x.clone(), timestep=ts_tok, **kw)[0]
        for s in SkipLayerStrategy:
            out[f"out.tok_{s.name}"] = core(hidden_states=x.clone(), timestep=ts_tok,
                                            skip_layer_mask=skip, skip_layer_strategy=s, **kw)[0]
    # scheduler (rf.py:179-374)
    g2 = torch.Generator().manual_seed(77)
    sample = torch.randn(2, 64, 16, generator=g2)
    v = torch.randn(2, 64, 16, generator=g2)
    for name, sch in (("Uniform", RectifiedFlowScheduler(sampler="Uniform")),
                      ("LinearQuadratic", RectifiedFlowScheduler(sampler="LinearQuadratic")),
                      ("SD3", RectifiedFlowScheduler(sampler="Uniform", shifting="SD3",
                                                     target_shift_terminal=0.1))):
        sch.set_timesteps(num_inference_steps=20, samples_shape=torch.Size([2, 128, 7, 16, 16]))
        out[f"sched.{name}.timesteps"] = sch.timesteps
        tg = sch.timesteps[3]
        out[f"sched.{name}.prev_global"] = sch.step(v, tg, sample, return_dict=False)[0]
        out[f"sched.{name}.prev_global_bf16v"] = sch.step(v.to(torch.bfloat16), tg, sample,
                                                          return_dict=False)[0]
        tt = torch.full((2, 64), float(tg))
        tt[:, 0] = 0.0
        tt[1, 5] = float((sch.timesteps[5] + sch.timesteps[6]) / 2)
        out[f"sched.{name}.t_tok"] = tt
        out[f"sched.{name}.prev_tok"] = sch.step(v, tt, sample, return_dict=False)[0]
    out["sched.sample"] = sample
    out["sched.v"] = v
    meta = {"config": TINY_CONFIG, "param_seed": seed, "lora_rank": rank, "lora_alpha": rank,
            "frame_rate": frame_rate, "t": 0.7, "strategies": [s.name for s in SkipLayerStrategy],
            "source": "reference Transformer3DModel.forward (inference call, "
                      "pipeline_ltx_video.py:1089-1228) + rf.py:179-374 via oracle/shim"}
    _save("infer_step", out, meta)


def gen_ckpt():
    """Checkpoint formats: the reference's save_training_checkpoint
    (torch_utils.py:105-133) of the tiny model in both train modes -- lora_audio exports the peft
    merge (export_merged_safetensors, :66-102), full saves the state dict
    (save_module_safetensors, :39-63) -- read back: tensors + safetensors metadata."""
    import copy
    import tempfile
    from safetensors import safe_open
    from ltx_video.utils.torch_utils import save_training_checkpoint
    seed, rank = 1234, 16
    model, _ = _build(TINY_CONFIG, seed, torch.bfloat16, rank)
    out, meta = {}, {"config": TINY_CONFIG, "param_seed": seed, "lora_rank": rank}
    with tempfile.TemporaryDirectory() as tmp:
        for mode, m in (("lora_audio", model), ("full", copy.deepcopy(model).merge_and_unload())):
            path = os.path.join(tmp, f"model_epoch_3.safetensors")
            save_training_checkpoint(m, path, mode, metadata={"epoch": "3", "source": "gen"},
                                     is_best=(mode == "full"))
            if mode == "full":
                path = os.path.join(tmp, "best_model_epoch_3.safetensors")
            with safe_open(path, framework="pt", device="cpu") as f:
                meta[f"{mode}.metadata"] = f.metadata()
                for k in f.keys():
                    out[f"{mode}.{k}"] = f.get_tensor(k)
    meta["source"] = "reference ltx_video/utils/torch_utils.py:39-133 via oracle/shim"
    _save("ckpt_export", out, meta)


def gen_full():
    """train_mode='full' (training.py:75-91; BASELINE config Z's trainable set):
    the tiny model without LoRA, attn1/attn2 (incl. q/k norms), every scale_shift_table,
    adaln_single, caption_projection and proj_out trainable; train_step + backward."""
    seed, B = 1234, 2
    g = torch.Generator().manual_seed(99)
    batch = {
        "latents": torch.randn(B, 128, 2, 8, 8, generator=g),
        "ref_image_latents": torch.randn(B, 128, 1, 8, 8, generator=g),
        "pose_latents": torch.randn(B, 128, 2, 8, 8, generator=g),
    }
    prompt = torch.randn(1, 4, 64, generator=g)
    mask = torch.tensor([[1, 1, 1, 0]], dtype=torch.long)
    pf = SymmetricPatchifier(patch_size=1)
    model = Transformer3DModel.from_config(TINY_CONFIG)
    model.patchifier = pf
    P.init_module_(model, seed, dtype=torch.bfloat16)
    model = T.apply_training_strategy(model, _train_cfg(16), "full")
    cap = _capture_train_step(model, pf, batch, prompt, mask, seed=4321, rank=16)
    grads = _grads(model)
    tensors = {f"in.{k}": v for k, v in batch.items()}
    tensors["in.prompt_embeds"] = prompt
    tensors["in.prompt_attention_mask"] = mask
    for k in ("tokens", "noise", "t", "hidden_states", "indices_grid", "sample", "loss"):
        tensors[f"out.{k}"] = cap[k]
    for k, v in grads.items():
        tensors[f"grad.{k}"] = v
    meta = {"config": TINY_CONFIG, "param_seed": seed, "train_seed": 4321, "train_mode": "full",
            "trainable": sorted(grads), "weights_sha256": P.weights_sha256(model),
            "source": "reference ltx_video/training.py:75-91 + 94-166 via oracle/shim"}
    _save("tiny_full_step", tensors, meta)


def gen_attn():
    """Operator-level plug-in fixture (Attention.set_processor, attention.py:532-552): the
    reference Attention modules of the tiny model's block 0 with AttnProcessor2_0
    (attention.py:935-1114) -- attn1 (self-attention, q/k RMSNorm + RoPE from the (cos, sin) pair
    of precompute_freqs_cis) and attn2 (cross-attention, key-padding mask bias prepared as in
    transformer3d.py:441-445, peft LoRA r=16 on to_q/to_k/to_v/to_out.0) -- forward and backward
    (seeded output gradients), in bf16 and with fp32 copies of the same weights (noise floor).
    The metadata lists the reference Attention's attribute and submodule names."""
    seed, rank, B, N, L = 1234, 16, 2, 64, 4
    g = torch.Generator().manual_seed(5)
    out = {}
    meta = {"config": TINY_CONFIG, "param_seed": seed, "lora_rank": rank, "lora_alpha": rank,
            "source": "reference attention.py:325-1114 (Attention + AttnProcessor2_0) via oracle/shim"}
    x = torch.randn(B, N, 128, generator=g)
    enc = torch.randn(B, L, 128, generator=g)
    m = torch.tensor([[1, 1, 1, 0], [1, 1, 0, 0]], dtype=torch.long)
    pf = SymmetricPatchifier(1)
    grid = pf.get_latent_coords(1, 8, 8, B, "cpu")
    d1 = torch.randn(B, N, 128, generator=g)
    d2 = torch.randn(B, N, 128, generator=g)
    for tag, dt in (("bf16", torch.bfloat16), ("fp32", torch.float32)):
        model, _ = _build(TINY_CONFIG, seed, dt, rank)
        core = model.base_model.model
        blk = core.transformer_blocks[0]
        cos, sin = core.precompute_freqs_cis(grid)
        bias = ((1 - m.to(dt)) * -10000.0).unsqueeze(1)  # transformer3d.py:441-445
        if tag == "bf16":
            for name, a in (("attn1", blk.attn1), ("attn2", blk.attn2)):
                meta[f"{name}_attributes"] = sorted(k for k in vars(a) if not k.startswith("_"))
                meta[f"{name}_modules"] = sorted(a._modules)
                meta[f"{name}_processor"] = type(a.processor).__name__
            out.update({"in.x": x.to(dt), "in.enc": enc.to(dt), "in.mask": m, "in.mask_bias": bias,
                        "in.cos": cos, "in.sin": sin, "in.dout1": d1.to(dt), "in.dout2": d2.to(dt),
                        "in.indices_grid": grid})
            for n, p in core.named_parameters():
                if n.startswith("transformer_blocks.0.attn"):
                    out["w." + P.canonical_name(n)] = p.detach().clone()
        xs = x.to(dt).requires_grad_()
        o1 = blk.attn1(xs, freqs_cis=(cos, sin))
        o1.backward(d1.to(dt))
        out[f"out.{tag}.o1"] = o1.detach()
        out[f"grad.{tag}.x1"] = xs.grad.detach()
        xs2 = x.to(dt).requires_grad_()
        es = enc.to(dt).requires_grad_()
        o2 = blk.attn2(xs2, freqs_cis=(cos, sin), encoder_hidden_states=es, attention_mask=bias)
        o2.backward(d2.to(dt))
        out[f"out.{tag}.o2"] = o2.detach()
        out[f"grad.{tag}.x2"] = xs2.grad.detach()
        out[f"grad.{tag}.enc2"] = es.grad.detach()
        for n, p in blk.attn2.named_parameters():
            if p.requires_grad:
                out[f"grad.{tag}.attn2.{P.canonical_name(n)}"] = p.grad.detach().clone()
    _save("attn_processor", out, meta)


def gen_config():
    cfg = load_train_config_from_yaml(os.path.join(REF, "configs", "train-avatars.yaml"))
    d = dataclasses.asdict(cfg)
    with open(os.path.join(OUT, "train_config.json"), "w") as f:
        json.dump(d, f, indent=1, sort_keys=True)
    print("  train_config.json")


if __name__ == "__main__":
    torch.set_num_threads(8)
    print("generating goldens into", OUT)
    if len(sys.argv) > 1:
        for name in sys.argv[1:]:
            globals()["gen_" + name]()
        raise SystemExit(0)
    gen_config()
    gen_patchify()
    gen_rf()
    gen_rope()
    gen_tiny()
    gen_block2b()
    gen_infer()
    gen_ckpt()
    gen_full()
    gen_attn()
