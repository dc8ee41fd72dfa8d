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
    # "_mse_f32": the unrounded f32 mean (parity tests compare losses at 1e-3, below the bf16
    # rounding of the reference's loss scalar); underscore keys are not logged
    return loss, rel_mse, nrmse, {"transformer_mse": mse, "_mse_f32": stats[0] / n}


class FusedAdamW(torch.optim.Optimizer):
    """torch.optim.AdamW (defaults betas (0.9, 0.999), eps 1e-8, weight_decay 1e-2; the
    reference constructs AdamW(trainable, lr) at training.py:270-271) with one ltx_adamw_step
    kernel per tensor; f32 LoRA adapters and bf16 caption-projection params keep their dtype."""

    CHUNK = 2048  # elements per block of the multi-tensor kernel

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2,
                 multi_tensor=True):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.multi_tensor = multi_tensor
        self._tables = []  # pinned host tables of the last steps (alive until their H2D lands)

    @torch.no_grad()
    def step(self, closure=None):
        for group in self.param_groups:
            b1, b2 = group["betas"]
            todo = []
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                st["step"] += 1
                todo.append((p, p.grad.contiguous(), st))
            by_dtype = {}
            for item in todo:
                by_dtype.setdefault(item[0].dtype, []).append(item)
            for dtype, items in by_dtype.items():
                steps = {st["step"] for _, _, st in items}
                if self.multi_tensor and len(items) > 1 and len(steps) == 1 and items[0][0].is_cuda:
                    self._multi(items, dtype, group, b1, b2, steps.pop())
                    continue
                for p, g, st in items:
                    ops.adamw_step(p, g, st["exp_avg"], st["exp_avg_sq"], group["lr"], b1, b2,
                                   group["eps"], group["weight_decay"], st["step"])
        ops.bump_weight_generation()  # in-place kernel updates: invalidate weight-derived caches

    def _multi(self, items, dtype, group, b1, b2, step):
        """One ltx_adamw_multi launch for all tensors of a dtype (bitwise the per-tensor math)."""
        rows = []
        for p, g, st in items:
            ptrs = (p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr())
            n = p.numel()
            for start in range(0, n, self.CHUNK):
                rows.append(ptrs + (start, min(self.CHUNK, n - start)))
        host = torch.tensor(rows, dtype=torch.int64).pin_memory()
        dev = host.to(items[0][0].device, non_blocking=True)
        self._tables = (self._tables + [(host, dev, [g for _, g, _ in items])])[-2:]
        ops.call("ltx_adamw_multi", ops._p(dev), len(rows), 1 if dtype == torch.bfloat16 else 0,
                 float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                 float(group["weight_decay"]), int(step), ops._s())


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


def train_one_epoch(model, dataloader, optimizer, scheduler, patchifier, device, config,
                    prompt_embeds, prompt_attention_mask, epoch, global_step, reducer=None,
                    log_fn=None):
    """training.py:169-231: micro-steps with gradient accumulation, the optimizer step every
    `gradient_accumulation_steps` batches (after the DP gradient all-reduce when `reducer` is
    given), per-step logging of loss / rel_mse / nrmse / lr through `log_fn` (wandb.log in the
    reference). Returns (global_step, mean epoch loss). The loss values stay on the device until
    an optimizer step logs them (one host sync per optimizer step, as the reference's .item())."""
    model.train()
    accum = max(1, int(config.gradient_accumulation_steps))
    optimizer.zero_grad(set_to_none=True)
    losses = []
    for batch_idx, batch in enumerate(dataloader):
        loss, rel_mse, nrmse, loss_dict = train_step(model, batch, scheduler, patchifier, config,
                                                     prompt_embeds, prompt_attention_mask, device)
        losses.append(loss.detach().float())
        if (batch_idx + 1) % accum == 0:
            if reducer is not None:
                reducer()
            optimizer.step()
            optimizer.zero_grad(set_to_none=True)
            global_step += 1
            if log_fn is not None:
                payload = {"train/loss": float(loss), "train/rel_mse": float(rel_mse),
                           "train/nrmse": float(nrmse), "train/epoch": epoch,
                           "train/lr": optimizer.param_groups[0]["lr"]}
                for k, v in (loss_dict or {}).items():
                    if not k.startswith("_"):
                        payload[f"train/{k}"] = float(v)
                log_fn(payload, global_step)
    epoch_loss = float(torch.stack(losses).mean()) if losses else 0.0
    return global_step, epoch_loss


def train_loop(model, config, dataloader, prompt_embeds, prompt_attention_mask, device=None,
               log_fn=None, rank=0):
    """training.py:234-401 for precomputed prompt embeddings (the T5 encode of main() is out of
    scope): trainable set per config.train_mode, FusedAdamW(lr), per-epoch checkpoints every
    `save_every_n_epochs` (best_ prefix on a new best epoch loss) through
    io.save_training_checkpoint, DP gradient averaging when torch.distributed is initialised."""
    import os

    from . import io
    from .scheduler import RectifiedFlowScheduler
    device = device or model.device
    patchifier = model.patchifier or SymmetricPatchifier(1)
    if getattr(config, "gradient_checkpointing", False):
        model.gradient_checkpointing = True
    rf = RectifiedFlowScheduler(num_train_timesteps=config.rf_num_train_timesteps,
                                shifting=config.rf_shifting,
                                base_resolution=config.rf_base_resolution,
                                target_shift_terminal=config.rf_target_shift_terminal,
                                sampler=config.rf_sampler, shift=config.rf_shift)
    params = [p for p in model.parameters() if p.requires_grad]
    optimizer = FusedAdamW(params, lr=config.learning_rate)
    reducer = GradAllReduce(params) if (dist.is_available() and dist.is_initialized()) else None
    best = float("inf")
    global_step = 0
    for epoch in range(config.num_epochs or 0):
        if hasattr(dataloader, "set_epoch"):
            dataloader.set_epoch(epoch)
        global_step, epoch_loss = train_one_epoch(model, dataloader, optimizer, rf, patchifier,
                                                  device, config, prompt_embeds,
                                                  prompt_attention_mask, epoch, global_step,
                                                  reducer, log_fn)
        if log_fn is not None:
            log_fn({"train/epoch_loss": epoch_loss}, global_step)
        if config.output_dir and rank == 0 and (epoch + 1) % config.save_every_n_epochs == 0:
            os.makedirs(config.output_dir, exist_ok=True)
            path = os.path.join(config.output_dir, f"model_epoch_{epoch + 1}.safetensors")
            meta = {"epoch": str(epoch + 1), "global_step": str(global_step),
                    "source": "single_gpu_epoch",
                    "scheduler": {"num_train_timesteps": config.rf_num_train_timesteps,
                                  "shifting": config.rf_shifting,
                                  "base_resolution": config.rf_base_resolution,
                                  "target_shift_terminal": config.rf_target_shift_terminal,
                                  "sampler": config.rf_sampler, "shift": config.rf_shift},
                    "vae": {"timestep_conditioning": True}}
            # the reference never updates best_loss (training.py:315, 395): every finite epoch
            # loss is "best" and the file gets the best_ prefix -- kept for drop-in paths
            io.save_training_checkpoint(model, path, getattr(config, "train_mode", "full"),
                                        metadata=meta, is_best=epoch_loss < best)
    return model
