"""ZeRO stage 2 for train_mode='full' on MI355X (BASELINE config Z: the reference's
training_deepspeed.py:49-266 with configs/ds_config_zero2.json -- stage 2, bf16, reduce_scatter,
contiguous_gradients, overlap_comm, gradient_clipping 1.0, torch AdamW as the client optimizer).

One process per GPU over torch.distributed (RCCL over xGMI; gloo in the CPU tests):
  * every trainable parameter's .data and .grad are views of two flat bf16 buffers (DeepSpeed's
    contiguous_gradients), laid out in the order the backward finishes the grads (``order``,
    Transformer3DModel.grad_ready_order: last block first) and cut into buckets of at most
    ``bucket_elems`` elements (ds_config reduce_bucket_size), each padded to a multiple of the
    world size; the backward's kernels accumulate straight into the flat grad buffer;
  * bucket k (elements [start_k, start_k + n_k)) is reduce-scattered (SUM) as ONE contiguous
    tensor, so rank r holds slice r of every bucket (n_k / world elements each): its shard is the
    concatenation of those slices. The reduction is f32 (``reduce_dtype``, default: the bucket is
    cast by ltx_cast_bf16_f32 first) or bf16 (half the bytes on the wire; the sum then rounds to
    bf16 on the way);
  * overlap_comm: ``install(model)`` + ``arm()`` before the last micro-step's backward of an
    accumulation cycle launch each bucket's cast + async reduce-scatter as soon as the backward
    has finished all of its grads (training.OverlapHooks: block hooks + post-accumulate-grad
    hooks), in bucket order on every rank; ``step()`` launches the rest and waits (stream waits,
    no host sync). Unarmed, the same buckets reduce after the backward: bitwise the same result;
  * step(): the global gradient norm is the all-reduced shard sum of squares (ltx_sumsq_f32, f64),
    ltx_clip_scale_f32 applies 1/world and the clip coefficient from device memory (no host sync),
    AdamW runs on the rank's f32 master shard and moments (ltx_adamw_step); each bucket slice is
    cast to bf16 into the flat parameter buffer and all-gathered in place, which updates every
    rank's weights.
Memory per rank: 2 B/param x 2 (bf16 params + grads, replicated) + 12 B/param / world (f32
master + exp_avg + exp_avg_sq) + a transient f32 grad buffer (4 B/param, f32 reduction only).
"""
import torch
import torch.distributed as dist

from . import ops
from ._lib import call
from .ops import _p, _s
from .training import OverlapHooks

F32 = torch.float32
BF16 = torch.bfloat16


class Zero2AdamW(OverlapHooks):
    def __init__(self, params, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2,
                 gradient_clipping=1.0, group=None, bucket_elems=500_000_000, order=None,
                 reduce_dtype=F32):
        params = [p for p in params if p.requires_grad]
        if any(p.dtype != BF16 for p in params):
            raise TypeError("Zero2AdamW expects bf16 parameters (ds_config bf16.enabled)")
        if reduce_dtype not in (F32, BF16):
            raise ValueError("Zero2AdamW: reduce_dtype must be torch.float32 or torch.bfloat16")
        if order is not None:  # the backward's completion order; parameters not in it go last
            ids = {id(p) for p in params}
            ordered, seen = [], set()
            for p in order:
                if id(p) in ids and id(p) not in seen:
                    ordered.append(p)
                    seen.add(id(p))
            params = ordered + [p for p in params if id(p) not in seen]
        self.params = params
        self.group = group
        dist_on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if dist_on else 1
        self.rank = dist.get_rank(group) if dist_on else 0
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.clip = float(gradient_clipping or 0.0)
        self.bucket = max(1, int(bucket_elems))
        self.reduce_dtype = reduce_dtype
        W = self.world
        # buckets: consecutive parameters, <= bucket_elems each (a larger parameter alone), each
        # padded to a multiple of the world size
        self.buckets = []
        cur = None
        for p in params:
            n = p.numel()
            if cur is None or (cur["used"] + n > self.bucket and cur["params"]):
                cur = {"params": [], "offsets": [], "used": 0}
                self.buckets.append(cur)
            cur["params"].append(p)
            cur["offsets"].append(cur["used"])
            cur["used"] += n
        start = soff = 0
        for b in self.buckets:
            b["start"] = start
            b["n"] = (b["used"] + W - 1) // W * W
            b["s"] = b["n"] // W          # this rank's slice of the bucket
            b["soff"] = soff              # ... at this offset of the shard
            start += b["n"]
            soff += b["s"]
        self._where = {id(p): (bi, j) for bi, b in enumerate(self.buckets)
                       for j, p in enumerate(b["params"])}
        self.numel = sum(p.numel() for p in params)
        self.padded = start
        self.shard = soff
        dev = params[0].device
        # flat bf16 params / grads; parameters become views (contiguous_gradients)
        self.flat_param = torch.zeros(self.padded, dtype=BF16, device=dev)
        self.flat_grad = torch.zeros(self.padded, dtype=BF16, device=dev)
        with torch.no_grad():
            for b in self.buckets:
                for p, off in zip(b["params"], b["offsets"]):
                    o = b["start"] + off
                    self.flat_param[o:o + p.numel()].copy_(p.detach().reshape(-1))
                    p.data = self.flat_param[o:o + p.numel()].view_as(p)
                    p.grad = self.flat_grad[o:o + p.numel()].view_as(p)
        self.master = torch.empty(self.shard, dtype=F32, device=dev)
        for b in self.buckets:
            self._cast_to_f32(self._my_slice(self.flat_param, b), self.master[b["soff"]:b["soff"] + b["s"]])
        self.exp_avg = torch.zeros(self.shard, dtype=F32, device=dev)
        self.exp_avg_sq = torch.zeros(self.shard, dtype=F32, device=dev)
        self.g32 = torch.empty(self.padded, dtype=F32, device=dev) if reduce_dtype == F32 else None
        self.gshard = torch.empty(self.shard, dtype=F32, device=dev)
        self.gshard16 = torch.empty(self.shard, dtype=BF16, device=dev) if reduce_dtype == BF16 else None
        self.sumsq = torch.zeros(1, dtype=torch.float64, device=dev)
        self.coef = torch.zeros(1, dtype=F32, device=dev)
        self.step_count = 0
        self.param_groups = [{"lr": lr}]
        self._init_hooks()

    def _my_slice(self, flat, b):
        lo = b["start"] + self.rank * b["s"]
        return flat[lo:lo + b["s"]]

    # -- device kernels (overridable by the CPU gloo tests, which have no HIP device) ----------
    def _cast_to_f32(self, src, dst):
        call("ltx_cast_bf16_f32", _p(src), _p(dst), src.numel(), _s())

    def _cast_to_bf16(self, src, dst):
        call("ltx_cast_f32_bf16", _p(src), _p(dst), src.numel(), _s())

    def _sumsq(self, x, out):
        ops._gemm_workspace(x.device)  # the per-block partials (deterministic order) live there
        call("ltx_sumsq_f32", _p(x), x.numel(), _p(out), 0, _s())

    def _clip_scale(self, x, sumsq, coef):
        call("ltx_clip_scale_f32", _p(x), x.numel(), _p(sumsq), self.clip, 1.0 / self.world,
             _p(coef), _s())

    def _adamw(self, master, grad, m, v, step):
        ops.adamw_step(master, grad, m, v, self.param_groups[0]["lr"], self.betas[0],
                       self.betas[1], self.eps, self.wd, step)

    # -- the reduce-scatter of one bucket (OverlapHooks._launch) --------------------------------
    @torch.no_grad()
    def _launch(self, bi):
        b = self.buckets[bi]
        lo, hi = b["start"], b["start"] + b["n"]
        out_lo, out_hi = b["soff"], b["soff"] + b["s"]
        if self.reduce_dtype == F32:
            inp = self.g32[lo:hi]
            self._cast_to_f32(self.flat_grad[lo:hi], inp)
            out = self.gshard[out_lo:out_hi]
        else:
            inp = self.flat_grad[lo:hi]
            out = self.gshard16[out_lo:out_hi]
        if not self._collectives_on():
            out.copy_(inp)
        else:
            self._works.append(dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM,
                                                          group=self.group, async_op=True))
        self._launched = bi + 1

    def _reduce_scatter(self):
        """Every bucket not launched during an armed backward, then wait for all of them."""
        if not self._armed:
            self._launched = 0
            self._works = []
        while self._launched < len(self.buckets):
            self._launch(self._launched)
        for w in self._works:
            w.wait()
        self._works = []
        self._armed = False
        if self.reduce_dtype == BF16:
            self._cast_to_f32(self.gshard16, self.gshard)

    @torch.no_grad()
    def step(self):
        self.step_count += 1
        self._reduce_scatter()
        self._sumsq(self.gshard, self.sumsq)
        if self._collectives_on() and self.clip > 0:
            dist.all_reduce(self.sumsq, op=dist.ReduceOp.SUM, group=self.group)
        self._clip_scale(self.gshard, self.sumsq, self.coef)
        self._adamw(self.master, self.gshard, self.exp_avg, self.exp_avg_sq, self.step_count)
        for b in self.buckets:
            mine = self._my_slice(self.flat_param, b)
            self._cast_to_bf16(self.master[b["soff"]:b["soff"] + b["s"]], mine)
            if self._collectives_on():
                dist.all_gather_into_tensor(self.flat_param[b["start"]:b["start"] + b["n"]], mine,
                                            group=self.group)
        ops.bump_weight_generation()  # weights changed in place: rebuild packed copies

    def zero_grad(self, set_to_none=False):
        """Grads stay views of the flat buffer; zeroing keeps them (set_to_none is ignored)."""
        self.flat_grad.zero_()

    def grad_norm(self):
        """The (pre-clip) global norm of the averaged gradients of the last step."""
        return float(self.sumsq.sqrt()) / self.world
