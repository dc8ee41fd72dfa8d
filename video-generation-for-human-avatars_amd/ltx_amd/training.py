"""Training step, fused AdamW and data-parallel gradient averaging.

train_step keeps the reference signature and semantics (ltx_video/training.py:94-166):
LogNormal(mu, sigma) timesteps -> r/(1+r) -> batch-quantile clamp, optional resolution shift,
noise ~ randn_like(tokens), x_t = (1-t)x0 + t*eps, v = eps - x0, model forward, MSE loss.
Differences that are deliberate and documented:
  * the train-step prologue (patchify + add_noise + velocity + conditioning lerp) is one kernel;
  * the backward is seeded directly with d(loss)/d(out) from the fused MSE kernel
    (grad scale = transformer_loss_weight / gradient_accumulation_steps, the reference's
    `loss / accum` then `.backward()`), so no host sync happens inside the step;
  * t is sampled on the host-side torch RNG exactly as the reference (so seeds reproduce it) but
    without the `float(t_low)` device->host round trip when the tensors are already on the host.
"""
import math

import torch
import torch.distributed as dist

from . import ops
from .patchifier import SymmetricPatchifier


def sample_timesteps(batch, config, device):
    """training.py:124-132."""
    mu = config.rf_log_normal_mu if config.rf_log_normal_mu is not None else 0.0
    sigma = config.rf_log_normal_sigma if config.rf_log_normal_sigma is not None else 1.0
    logn = torch.distributions.LogNormal(torch.tensor(mu, device=device),
                                         torch.tensor(sigma, device=device))
    raw = logn.sample((batch,))
    t_raw = raw / (1 + raw)
    t_low = torch.quantile(t_raw, config.rf_quantile_min)
    t_high = torch.quantile(t_raw, config.rf_quantile_max)
    return t_raw.clamp(min=float(t_low), max=float(t_high))


def train_step(model, batch, scheduler, patchifier, config, prompt_embeds, prompt_attention_mask,
               device=None, t=None, noise=None, backward=True):
    """Returns (loss, rel_mse, nrmse, loss_dict) like the reference; runs the backward too when
    `backward` (the reference calls loss.backward() in train_one_epoch, training.py:203)."""
    dt = torch.bfloat16
    device = device or model.device
    latents = batch["latents"].to(device=device, dtype=dt)
    ref = batch["ref_image_latents"].to(device=device, dtype=dt)
    pose = batch["pose_latents"].to(device=device, dtype=dt)
    B, C, F, H, W = latents.shape
    N = F * H * W
    # convert first, then expand: the batch stays a stride-0 view, which the model recognises as
    # one prompt shared by the batch (caption projection and text K/V computed once)
    enc = prompt_embeds.to(device=device, dtype=dt).expand(B, -1, -1)
    enc_mask = prompt_attention_mask.to(device).expand(B, -1)
    # one coordinate set broadcast over the batch (identical per sample): one shared RoPE table
    coords = patchifier.get_latent_coords(F, H, W, 1, device).expand(B, -1, -1)
    if t is None:
        t = sample_timesteps(B, config, "cpu").to(device)
        t = scheduler.shift_timesteps(torch.Size([B, N, C]), t)
    t = t.to(device=device, dtype=torch.float32)
    if noise is None:
        noise = torch.randn((B, N, C), device=device, dtype=dt)
    _, model_in, v_target = ops.rf_prepare_tokens(latents, ref, pose, noise, t)
    # the conditioning lerp is already applied: hand the model lerp-neutral conditioning views
    out = model._forward_tokens(model_in, coords, enc, t, enc_mask)
    w = float(getattr(config, "transformer_loss_weight", 1.0))
    accum = max(1, int(getattr(config, "gradient_accumulation_steps", 1)))
    stats, dout = ops.mse_fwd_bwd(out, v_target, grad_scale=w / accum, want_grad=backward)
    n = out.numel()
    mse = (stats[0] / n).to(dt)
    loss = w * mse
    std = torch.sqrt(torch.clamp((stats[2] - stats[1] * stats[1] / n) / (n - 1), min=0)).to(dt)
    rel_mse = loss / (std ** 2 + 1e-12)
    nrmse = torch.sqrt(loss) / (std + 1e-12)
    if backward:
        out.backward(dout)
    return loss, rel_mse, nrmse, {"transformer_mse": mse}


class FusedAdamW(torch.optim.Optimizer):
    """torch.optim.AdamW (defaults betas (0.9, 0.999), eps 1e-8, weight_decay 1e-2; the
    reference constructs AdamW(trainable, lr) at training.py:270-271) with one ltx_adamw_step
    kernel per tensor; f32 LoRA adapters and bf16 caption-projection params keep their dtype."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                st["step"] += 1
                ops.adamw_step(p, p.grad.contiguous(), st["exp_avg"], st["exp_avg_sq"], group["lr"],
                               b1, b2, group["eps"], group["weight_decay"], st["step"])
        ops.bump_weight_generation()  # in-place kernel updates: invalidate weight-derived caches


class GradAllReduce:
    """Data-parallel averaging of the trainable gradients (LoRA f32 + caption projection bf16)
    over torch.distributed (RCCL on ROCm, gloo in the CPU tests). Gradients are packed into
    ~bucket_mb f32 buckets in reverse registration order (last blocks first, the order the
    backward produces them) and reduced with AVG; bf16 grads are reduced in f32."""

    def __init__(self, params, bucket_mb=25.0, group=None):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.buckets = []
        cur, size = [], 0
        for p in reversed(self.params):
            cur.append(p)
            size += p.numel() * 4
            if size >= bucket_mb * 1e6:
                self.buckets.append(cur)
                cur, size = [], 0
        if cur:
            self.buckets.append(cur)

    @torch.no_grad()
    def __call__(self):
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(self.group) == 1:
            return
        world = dist.get_world_size(self.group)
        pending = []
        for bucket in self.buckets:
            grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in bucket]
            flat = torch.cat([g.reshape(-1).float() for g in grads])
            work = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            pending.append((bucket, flat, work))
        for bucket, flat, work in pending:
            work.wait()
            flat.div_(world)
            off = 0
            for p in bucket:
                n = p.numel()
                g = flat[off:off + n].view_as(p).to(p.dtype)
                if p.grad is None:
                    p.grad = g
                else:
                    p.grad.copy_(g)
                off += n
