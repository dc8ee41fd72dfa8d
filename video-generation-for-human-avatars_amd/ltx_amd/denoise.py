"""One iteration of the LTXVideoPipeline denoising loop on MI355X.

denoise_step() restates pipeline_ltx_video.py:1089-1279 (the loop body) + denoising_step
(:1346-1379) for the part that touches the latent tokens: the CFG / STG batch of num_conds
copies, float pixel-coordinate RoPE grid (/ frame_rate), per-token timesteps under a
conditioning mask, the skip-layer mask of the perturbed batch, the transformer call, guidance
(CFG, CFG*, STG, rescaling) and the rectified-flow Euler update. Everything that runs per step
over the tokens is a HIP kernel (transformer blocks, ltx_pixel_coords_f32, ltx_guidance_bf16,
ltx_rf_euler_step); the VAE, text encoder and conditioning-item preparation stay out of scope
(SURVEY 2).
"""
from typing import Optional, Sequence

import torch

from . import ops


def denoise_step(transformer, scheduler, latents, t, *, prompt_embeds_batch,
                 prompt_attention_mask_batch, ref_image_hidden_states, pose_hidden_states,
                 frame_rate: float, batch_size: int, guidance_scale: float = 1.0,
                 stg_scale: float = 0.0, rescaling_scale: float = 1.0,
                 cfg_star_rescale: bool = False, skip_block_list: Optional[Sequence[int]] = None,
                 skip_layer_strategy=None, conditioning_mask: Optional[torch.Tensor] = None,
                 scale_factors=(8, 32, 32), causal_fix: bool = True,
                 stochastic_sampling: bool = False):
    """latents [B, N, C] (tokens) at scalar timestep t -> latents at the next scheduled timestep.

    prompt_embeds_batch / prompt_attention_mask_batch hold (negative, positive, positive)
    x batch_size as the pipeline builds them; ref/pose are [B, C, 1|F, H, W] latents."""
    do_cfg = guidance_scale > 1.0
    do_stg = stg_scale > 0
    num_conds = 1 + int(do_cfg) + int(do_stg)
    if do_cfg and do_stg:
        indices = slice(0, batch_size * 3)
    elif do_cfg:
        indices = slice(0, batch_size * 2)
    elif do_stg:
        indices = slice(batch_size, batch_size * 3)
    else:
        indices = slice(batch_size, batch_size * 2)
    skip_layer_mask = None
    if do_stg and skip_block_list is not None:
        skip_layer_mask = transformer.create_skip_layer_mask(batch_size, num_conds, num_conds - 1,
                                                             skip_block_list)
    B, C, F, H, W = pose_hidden_states.shape
    dev = latents.device
    indices_grid, _ = ops.pixel_coords(num_conds * B, F, H, W, dev, scale_factors, causal_fix,
                                       frame_rate)
    model_in = torch.cat([latents] * num_conds) if num_conds > 1 else latents
    t_val = float(t)
    current_timestep = torch.full((num_conds * B, 1), t_val, dtype=torch.float32, device=dev)
    if conditioning_mask is not None:
        cm = torch.cat([conditioning_mask] * num_conds).to(device=dev, dtype=torch.float32)
        current_timestep = torch.min(current_timestep, 1.0 - cm)
    dt = transformer.dtype
    noise_pred = transformer(
        model_in.to(dt), indices_grid=indices_grid,
        ref_image_hidden_states=torch.cat([ref_image_hidden_states] * num_conds).to(dt),
        pose_hidden_states=torch.cat([pose_hidden_states] * num_conds).to(dt),
        encoder_hidden_states=prompt_embeds_batch[indices].to(dt),
        encoder_attention_mask=prompt_attention_mask_batch[indices],
        timestep=current_timestep, skip_layer_mask=skip_layer_mask,
        skip_layer_strategy=skip_layer_strategy, return_dict=False)[0]
    noise_pred = ops.guidance(noise_pred, batch_size, do_cfg, do_stg, guidance_scale, stg_scale,
                              rescaling_scale, cfg_star_rescale)
    # current_timestep[:1] (pipeline_ltx_video.py:1270): a [1, 1|N] tensor -> the scheduler's
    # per-token branch with f32 dt, broadcast over the batch
    ts = current_timestep[:1].expand(B, latents.shape[1]).contiguous()
    if stochastic_sampling:
        den = scheduler.step(noise_pred, ts, latents, return_dict=False,
                             stochastic_sampling=True)[0]
        if conditioning_mask is None:
            return den
        keep = (t_val - 1e-6 < (1.0 - conditioning_mask.to(dev))).unsqueeze(-1)
        return torch.where(keep, den, latents)
    return ops.rf_euler_step(noise_pred, ts, latents, scheduler.timesteps,
                             cond_mask=conditioning_mask, t_cond=t_val)
