"""Training step, fused AdamW and data-parallel gradient averaging.

train_step keeps the reference signature and semantics (ltx_video/training.py:94-166):
LogNormal(mu, sigma) timesteps -> r/(1+r) -> batch-quantile clamp, optional resolution shift,
noise ~ randn_like(tokens), x_t = (1-t)x0 + t*eps, v = eps - x0, model forward, MSE loss.
Differences that are deliberate and documented:
  * the train-step prologue (patchify + add_noise + velocity + conditioning lerp) is one kernel;
  * the backward is seeded directly with d(loss)/d(out) from the fused MSE kernel
    (grad scale = transformer_loss_weight / gradient_accumulation_steps, the reference's
    `loss / accum` then `.backward()`), so no host sync happens inside the step;
  * t is sampled on `device` exactly as the reference (training.py:124-132: LogNormal on the
    device RNG, then randn_like for the noise, so a seeded run draws the same t and noise); the
    quantile clamp takes the bounds as 0-dim device tensors instead of `float(t_low)`, which gives
    the same f32 result without the device->host round trip in every micro-step.
"""
import functools
import math

import torch
import torch.distributed as dist

from . import ops
from .patchifier import SymmetricPatchifier


_LOGN_PARAMS = {}  # (mu, sigma, device) -> the LogNormal's 0-dim device loc / scale
_QUANTILES = {}  # (q_min, q_max, device, dtype) -> the two quantile levels as one device tensor


def sample_timesteps(batch, config, device):
    """training.py:124-132: LogNormal(mu, sigma).sample((B,)) -> r/(1+r) -> batch-quantile clamp.

    The draw is the distribution's own arithmetic written out, without its three host syncs per
    micro-step (each drains the device queue, so the step prologue then ran host-bound with the
    GPU idle): torch.tensor(x, device=cuda) is a blocking H2D copy, the distribution validates
    its arguments by reading a device bool back, and torch.normal(mean, std) checks
    std.min() >= 0 with .item(). torch.normal(mean, std) is normal_(0, 1) on its output, then
    output.mul_(std).add_(mean) (ATen normal_out_impl), and LogNormal.sample exponentiates it:
    the same generator draw and the same f32 roundings here."""
    mu = config.rf_log_normal_mu if config.rf_log_normal_mu is not None else 0.0
    sigma = config.rf_log_normal_sigma if config.rf_log_normal_sigma is not None else 1.0
    key = (float(mu), float(sigma), str(torch.device(device)))
    params = _LOGN_PARAMS.get(key)
    if params is None:
        params = (torch.tensor(mu, device=device), torch.tensor(sigma, device=device))
        _LOGN_PARAMS[key] = params
    loc, scale = params
    z = torch.empty(batch, dtype=loc.dtype, device=device).normal_(0.0, 1.0)
    raw = z.mul_(scale).add_(loc).exp_()
    t_raw = raw / (1 + raw)
    # both bounds from one sort: quantile with a q tensor runs the scalar form's arithmetic per q
    # (q as an f32 tensor, rank q (n - 1), the same lerp), so the values are those of two calls
    qkey = (float(config.rf_quantile_min), float(config.rf_quantile_max), str(torch.device(device)), t_raw.dtype)
    qs = _QUANTILES.get(qkey)
    if qs is None:
        qs = torch.tensor([qkey[0], qkey[1]], dtype=t_raw.dtype, device=device)
        _QUANTILES[qkey] = qs
    t_low, t_high = torch.quantile(t_raw, qs).unbind(0)
    # clamp against the 0-dim f32 bounds: the reference's float(t_low) is the same f32 value
    # (exact in double, cast back to f32 by clamp), so only the host sync differs
    return t_raw.clamp(min=t_low, max=t_high)


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
        t = sample_timesteps(B, config, device)
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
        self._tables = []  # pinned host tables of the last builds (alive until their H2D lands)
        self._table_cache = {}  # dtype -> (buffer pointers, device table, rows)

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
        """One ltx_adamw_multi launch for all tensors of a dtype (bitwise the per-tensor math).
        The chunk table (~10^4 rows at LTX-2B: milliseconds of host time) is built once per set
        of buffers and reused while the parameter / grad / state storages stay the same."""
        ptrs = [(p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                 p.numel()) for p, g, st in items]
        key = (dtype, tuple(ptrs))
        hit = self._table_cache.get(dtype)
        if hit is not None and hit[0] == key:
            dev, nrows = hit[1], hit[2]
        else:
            rows = []
            for pp, gp, ap, sp, n in ptrs:
                for start in range(0, n, self.CHUNK):
                    rows.append((pp, gp, ap, sp, start, min(self.CHUNK, n - start)))
            host = torch.tensor(rows, dtype=torch.int64).pin_memory()
            dev = host.to(items[0][0].device, non_blocking=True)
            nrows = len(rows)
            # the pinned host copy stays alive until its H2D has landed (two steps later)
            self._tables = (self._tables + [(host, dev)])[-2:]
            self._table_cache[dtype] = (key, dev, nrows)
        rows = range(nrows)
        ops.call("ltx_adamw_multi", ops._p(dev), len(rows), 1 if dtype == torch.bfloat16 else 0,
                 float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                 float(group["weight_decay"]), int(step), ops._s())


class OverlapHooks:
    """Readiness tracking shared by the reducers that overlap their collectives with the last
    micro-step's backward (GradAllReduce here, zero.Zero2AdamW): ``self.buckets`` is a list of
    dicts with a "params" list, ``self._where`` maps id(param) -> (bucket, index), and the subclass
    implements ``_launch(bi)`` (start bucket bi's collective, set ``self._launched = bi + 1``).

    ``install(model)`` hooks the model: each block reports, at the end of its backward, the grads
    its own kernels wrote into .grad (the attn1 / attn2 parameters: LoRA adapters, and in
    train_mode='full' the attention weights, biases and q/k norm weights); every other trainable
    parameter -- including a block's scale_shift_table, whose gradient autograd accumulates AFTER
    the block's backward returns (through _AdaModFn) -- reports through a post-accumulate-grad
    hook. ``arm()`` before the last backward of an accumulation cycle; from then on a bucket
    launches as soon as all of its grads are final, always in index order on every rank (a ready
    bucket waits for its predecessors), so the collectives match across ranks."""

    # test-only: launch the collectives (and take their stream waits) even at world size 1, so a
    # one-GPU box exercises RCCL's own stream and the armed bucket path (tests/test_dp_gpu.py)
    collectives_at_world1 = False

    def _collectives_on(self):
        return self._world() > 1 or self.collectives_at_world1

    def _init_hooks(self):
        self._armed = False
        self._pending = None   # per bucket: grads not yet final
        self._launched = 0     # buckets [0, _launched) have their collective in flight
        self._works = []
        self._hooks = []
        self._block_cbs = []  # (weakref to block, callback) appended to its _grad_ready_hooks

    def _world(self):
        if not (dist.is_available() and dist.is_initialized()):
            return 1
        return dist.get_world_size(self.group)

    def install(self, model):
        import weakref
        self.uninstall()
        me = weakref.ref(self)

        def block_cb(b, done=None, ps=None, ids=None):
            # done: the subset the block has finished (None: all it writes); only parameters the
            # block's kernels write are reported here
            red = me()
            if red is not None:
                red._ready(ps if done is None else [p for p in done if id(p) in ids])

        in_blocks = set()
        for blk in getattr(model, "transformer_blocks", ()):
            written = [p for name in ("attn1", "attn2") if name in blk._modules
                       for p in blk._modules[name].parameters() if id(p) in self._where]
            if written:
                in_blocks.update(id(p) for p in written)
                cb = functools.partial(block_cb, ps=written, ids={id(p) for p in written})
                blk.__dict__.setdefault("_grad_ready_hooks", []).append(cb)
                self._block_cbs.append((weakref.ref(blk), cb))
        for p in self.params:
            if id(p) not in in_blocks:
                self._hooks.append(p.register_post_accumulate_grad_hook(
                    lambda q: me() is not None and me()._ready([q])))
        return self

    def uninstall(self):
        """Remove this reducer's block callbacks and post-accumulate-grad hooks."""
        for h in self._hooks:
            h.remove()
        self._hooks = []
        for bref, cb in self._block_cbs:
            blk = bref()
            hooks = blk.__dict__.get("_grad_ready_hooks") if blk is not None else None
            if hooks is not None:
                hooks[:] = [h for h in hooks if h is not cb]
        self._block_cbs = []

    def _prepare_arm(self):
        """subclass hook: make the grads views of the buckets before an armed backward"""

    def arm(self):
        """The next backward is the last of the accumulation cycle: reduce during it."""
        if not self._collectives_on():
            return
        self._prepare_arm()
        self._armed = True
        self._pending = [set(id(p) for p in b["params"]) for b in self.buckets]
        self._launched = 0
        self._works = []

    def _ready(self, ps):
        if not self._armed:
            return
        for p in ps:  # (each grad must be final after one report: one accumulation per backward)
            bi, _ = self._where[id(p)]
            self._pending[bi].discard(id(p))
        while self._launched < len(self.buckets) and not self._pending[self._launched]:
            self._launch(self._launched)


class GradAllReduce(OverlapHooks):
    """Data-parallel averaging of the trainable gradients (LoRA f32 + caption projection bf16)
    over torch.distributed (RCCL on ROCm, gloo in the CPU tests), overlapped with the backward.

    * The gradients ARE views of per-dtype flat bucket buffers (``zero_grad`` installs them), so
      the backward's kernels accumulate straight into what gets reduced: no pack, no copy-back.
      f32 buckets are reduced in place; bf16 buckets (caption projection) through an f32 staging
      copy (one cast each way), so the sum is f32 and rounds to bf16 once.
    * Buckets (~bucket_mb of f32 each) follow ``order``: the order the backward completes the
      grads (``Transformer3DModel.grad_ready_order``: last block first).
    * ``arm()`` before the LAST micro-step's backward of an accumulation cycle: a bucket's async
      all-reduce (SUM) is launched as soon as all of its grads are final (OverlapHooks) while the
      remaining blocks' backward runs.
    * ``__call__()`` (before the optimizer step) launches whatever has not been launched, waits
      (a stream wait, no host sync) and divides by the world size. Unarmed, it is the plain
      post-backward reduction of the same buckets: the two paths are bitwise equal.
    """

    def __init__(self, params, bucket_mb=25.0, group=None, order=None):
        params = [p for p in params if p.requires_grad]
        if order is not None:
            ids = {id(p) for p in params}
            ordered = [p for p in order if id(p) in ids]
            rest = [p for p in reversed(params) if id(p) not in {id(q) for q in ordered}]
            params = ordered + rest
        else:
            params = list(reversed(params))  # registration order reversed
        self.params = params
        self.group = group
        self.buckets = []  # each: {"dtype", "params", "offsets", "n", "flat", "stage"}
        open_b = {}
        for p in params:
            b = open_b.get(p.dtype)
            if b is None:
                b = {"dtype": p.dtype, "params": [], "offsets": [], "n": 0, "flat": None,
                     "stage": None}
                open_b[p.dtype] = b
                self.buckets.append(b)
            b["params"].append(p)
            b["offsets"].append(b["n"])
            b["n"] += p.numel()
            if b["n"] * 4 >= bucket_mb * 1e6:
                del open_b[p.dtype]
        self._where = {id(p): (bi, j) for bi, b in enumerate(self.buckets)
                       for j, p in enumerate(b["params"])}
        self._init_hooks()

    # ---- buffers -------------------------------------------------------------------------
    def _alloc(self, b):
        if b["flat"] is None:
            dev = b["params"][0].device
            b["flat"] = torch.zeros(b["n"], dtype=b["dtype"], device=dev)
            if b["dtype"] != torch.float32:
                b["stage"] = torch.empty(b["n"], dtype=torch.float32, device=dev)

    def _view(self, b, j):
        p, off = b["params"][j], b["offsets"][j]
        return b["flat"][off:off + p.numel()].view_as(p)

    @torch.no_grad()
    def zero_grad(self):
        """Zero every bucket (one fill each) and make each p.grad the view of its slice (in place
        of optimizer.zero_grad(set_to_none=True), which would detach the grads from the buckets)."""
        for b in self.buckets:
            self._alloc(b)
            b["flat"].zero_()
            for j, p in enumerate(b["params"]):
                p.grad = self._view(b, j)

    @torch.no_grad()
    def _adopt_grads(self, b):
        """Make the bucket's grads views again if something replaced them (copy them in)."""
        self._alloc(b)
        for j, p in enumerate(b["params"]):
            v = self._view(b, j)
            g = p.grad
            if g is not None and g.data_ptr() == v.data_ptr() and g.dtype == v.dtype:
                continue
            if g is None:
                v.zero_()
            else:
                v.copy_(g)
            p.grad = v

    def _prepare_arm(self):
        for b in self.buckets:
            self._adopt_grads(b)

    @torch.no_grad()
    def _launch(self, bi):
        b = self.buckets[bi]
        buf = b["flat"]
        if b["stage"] is not None:
            b["stage"].copy_(buf)  # bf16 -> f32
            buf = b["stage"]
        self._works.append(dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group,
                                           async_op=True))
        self._launched = bi + 1

    @torch.no_grad()
    def __call__(self):
        world = self._world()
        if not self._collectives_on():
            self._armed = False
            return
        if not self._armed:
            for b in self.buckets:
                self._adopt_grads(b)
            self._launched = 0
            self._works = []
        while self._launched < len(self.buckets):
            self._launch(self._launched)
        for w in self._works:
            w.wait()
        for b in self.buckets:
            if b["stage"] is not None:
                b["stage"].div_(world)
                b["flat"].copy_(b["stage"])  # f32 -> bf16, one rounding
            else:
                b["flat"].div_(world)
        self._armed = False
        self._works = []


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

    def zero():
        if reducer is not None:
            reducer.zero_grad()  # grads stay views of the reducer's buckets
        else:
            optimizer.zero_grad(set_to_none=True)
    zero()
    losses = []
    for batch_idx, batch in enumerate(dataloader):
        last = (batch_idx + 1) % accum == 0
        if last and reducer is not None:
            reducer.arm()  # the all-reduce overlaps this micro-step's backward
        loss, rel_mse, nrmse, loss_dict = train_step(model, batch, scheduler, patchifier, config,
                                                     prompt_embeds, prompt_attention_mask, device)
        losses.append(loss.detach().float())
        if last:
            if reducer is not None:
                reducer()
            optimizer.step()
            zero()
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
    reducer = None
    if dist.is_available() and dist.is_initialized():
        order = model.grad_ready_order() if hasattr(model, "grad_ready_order") else None
        reducer = GradAllReduce(params, order=order).install(model)
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
