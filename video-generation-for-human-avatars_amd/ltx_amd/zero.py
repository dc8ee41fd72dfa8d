"""ZeRO stage 2 for train_mode='full' on MI355X (BASELINE config Z: the reference's
training_deepspeed.py:49-266 with configs/ds_config_zero2.json -- stage 2, bf16, reduce_scatter,
contiguous_gradients, gradient_clipping 1.0, torch AdamW as the client optimizer).

One process per GPU over torch.distributed (RCCL over xGMI; gloo in the CPU tests):
  * every trainable parameter's .data and .grad are views of two flat bf16 buffers (DeepSpeed's
    contiguous_gradients), padded to a multiple of the world size; the backward's kernels
    accumulate straight into the flat grad buffer;
  * step(): the flat grads go to f32 (ltx_cast_bf16_f32) and are reduce-scattered (SUM) in
    buckets, so rank r holds the summed grads of its 1/world shard; the global gradient norm is
    the all-reduced shard sum of squares (ltx_sumsq_f32), and ltx_clip_scale_f32 applies
    1/world and the clip coefficient from device memory (no host sync); AdamW runs on the
    rank's f32 master shard and moments (ltx_adamw_step); the shard is cast to bf16 into the
    flat parameter buffer and all-gathered in place, which updates every rank's weights.
Memory per rank: 2 B/param x 2 (bf16 params + grads, replicated) + 12 B/param / world (f32
master + exp_avg + exp_avg_sq) + a transient f32 grad buffer.
"""
import torch
import torch.distributed as dist

from . import ops
from ._lib import call
from .ops import _p, _s

F32 = torch.float32
BF16 = torch.bfloat16


class Zero2AdamW:
    def __init__(self, params, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2,
                 gradient_clipping=1.0, group=None, bucket_elems=500_000_000):
        self.params = [p for p in params if p.requires_grad]
        if any(p.dtype != BF16 for p in self.params):
            raise TypeError("Zero2AdamW expects bf16 parameters (ds_config bf16.enabled)")
        self.group = group
        dist_on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if dist_on else 1
        self.rank = dist.get_rank(group) if dist_on else 0
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.clip = float(gradient_clipping or 0.0)
        self.bucket = int(bucket_elems)
        dev = self.params[0].device
        total = sum(p.numel() for p in self.params)
        self.numel = total
        self.padded = (total + self.world - 1) // self.world * self.world
        self.shard = self.padded // self.world
        # flat bf16 params / grads; parameters become views (contiguous_gradients)
        self.flat_param = torch.zeros(self.padded, dtype=BF16, device=dev)
        self.flat_grad = torch.zeros(self.padded, dtype=BF16, device=dev)
        off = 0
        with torch.no_grad():
            for p in self.params:
                n = p.numel()
                self.flat_param[off:off + n].copy_(p.detach().reshape(-1))
                p.data = self.flat_param[off:off + n].view_as(p)
                p.grad = self.flat_grad[off:off + n].view_as(p)
                off += n
        lo = self.rank * self.shard
        self.master = torch.empty(self.shard, dtype=F32, device=dev)
        self._cast_to_f32(self.flat_param[lo:lo + self.shard], self.master)
        self.exp_avg = torch.zeros(self.shard, dtype=F32, device=dev)
        self.exp_avg_sq = torch.zeros(self.shard, dtype=F32, device=dev)
        self.g32 = torch.empty(self.padded, dtype=F32, device=dev)
        self.gshard = torch.empty(self.shard, dtype=F32, device=dev)
        self.sumsq = torch.zeros(1, dtype=torch.float64, device=dev)
        self.coef = torch.zeros(1, dtype=F32, device=dev)
        self.step_count = 0
        self.param_groups = [{"lr": lr}]

    # -- device kernels (overridable by the CPU gloo tests, which have no HIP device) ----------
    def _cast_to_f32(self, src, dst):
        call("ltx_cast_bf16_f32", _p(src), _p(dst), src.numel(), _s())

    def _cast_to_bf16(self, src, dst):
        call("ltx_cast_f32_bf16", _p(src), _p(dst), src.numel(), _s())

    def _sumsq(self, x, out):
        call("ltx_sumsq_f32", _p(x), x.numel(), _p(out), 0, _s())

    def _clip_scale(self, x, sumsq, coef):
        call("ltx_clip_scale_f32", _p(x), x.numel(), _p(sumsq), self.clip, 1.0 / self.world,
             _p(coef), _s())

    def _adamw(self, master, grad, m, v, step):
        ops.adamw_step(master, grad, m, v, self.param_groups[0]["lr"], self.betas[0],
                       self.betas[1], self.eps, self.wd, step)

    # -- the step --------------------------------------------------------------------------
    def _reduce_scatter(self):
        self._cast_to_f32(self.flat_grad, self.g32)
        if self.world == 1:
            self.gshard.copy_(self.g32)
            return
        # bucketed reduce_scatter over contiguous slices: bucket k covers the same element
        # range of every rank's shard, so the output lands in place in gshard
        step = max(1, min(self.shard, self.bucket // self.world))
        view = self.g32.view(self.world, self.shard)
        for c0 in range(0, self.shard, step):
            c1 = min(self.shard, c0 + step)
            inp = view[:, c0:c1].contiguous().view(-1)
            out = self.gshard[c0:c1]
            dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=self.group)

    @torch.no_grad()
    def step(self):
        self.step_count += 1
        self._reduce_scatter()
        self._sumsq(self.gshard, self.sumsq)
        if self.world > 1 and self.clip > 0:
            dist.all_reduce(self.sumsq, op=dist.ReduceOp.SUM, group=self.group)
        self._clip_scale(self.gshard, self.sumsq, self.coef)
        self._adamw(self.master, self.gshard, self.exp_avg, self.exp_avg_sq, self.step_count)
        lo = self.rank * self.shard
        self._cast_to_bf16(self.master, self.flat_param[lo:lo + self.shard])
        if self.world > 1:
            dist.all_gather_into_tensor(self.flat_param, self.flat_param[lo:lo + self.shard],
                                        group=self.group)
        ops.bump_weight_generation()  # weights changed in place: rebuild packed copies

    def zero_grad(self, set_to_none=False):
        """Grads stay views of the flat buffer; zeroing keeps them (set_to_none is ignored)."""
        self.flat_grad.zero_()

    def grad_norm(self):
        """The (pre-clip) global norm of the averaged gradients of the last step."""
        return float(self.sumsq.sqrt()) / self.world
