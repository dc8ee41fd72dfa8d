"""CPU tests of the host-side mirror (no GPU, no kernel launches): config loading, scheduler
timestep shifts, t sampling, PEFT-compatible module/parameter naming, checkpoint loading and LoRA
merge, and the data-parallel gradient all-reduce over gloo with world_size 2.

Parity anchors: tests/golden/train_config.json (the reference's own load_train_config_from_yaml on
configs/train-avatars.yaml), tests/golden/rf_sched.* (reference RectifiedFlowScheduler), the
tiny_train_step golden's parameter/grad key sets (reference model wrapped by peft)."""
import json
import math
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from safetensors.torch import load_file, save_file

from params import canonical_name

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REF_YAML = "/root/reference/configs/train-avatars.yaml"

TINY = None


def _tiny():
    global TINY
    if TINY is None:
        with open(os.path.join(GOLD, "tiny_train_step.json")) as f:
            meta = json.load(f)
        TINY = (load_file(os.path.join(GOLD, "tiny_train_step.safetensors")), meta)
    return TINY


# ---------------------------------------------------------------------------------- config
def test_train_config_golden_fields():
    """TrainConfig keeps every field name of ltx_video/config.py:6-64 with the golden's values
    type-compatible (the golden is the reference parse of train-avatars.yaml)."""
    from dataclasses import fields

    from ltx_amd.config import TrainConfig
    with open(os.path.join(GOLD, "train_config.json")) as f:
        gold = json.load(f)
    names = {f.name for f in fields(TrainConfig)}
    assert names == set(gold), names ^ set(gold)
    cfg = TrainConfig(**gold)
    assert cfg.gradient_accumulation_steps == 16 and cfg.lora_rank == 32


@pytest.mark.skipif(not os.path.exists(REF_YAML), reason="reference tree not present")
def test_train_config_matches_reference_parse():
    from dataclasses import asdict

    from ltx_amd.config import load_train_config_from_yaml
    with open(os.path.join(GOLD, "train_config.json")) as f:
        gold = json.load(f)
    assert asdict(load_train_config_from_yaml(REF_YAML)) == gold


def test_train_config_quirks(tmp_path):
    """config.py:109-154: sampler aliases, falsy rf floats read as None, checkpoint required."""
    from ltx_amd.config import load_train_config_from_yaml
    p = tmp_path / "c.yaml"
    p.write_text("checkpoint_path: x.safetensors\nsampler: LinearQuadratic\nprecision: bf16\n"
                 "train:\n  rf_log_normal_mu: 0\n  rf_log_normal_sigma: 1.5\n  batch_size: 4\n"
                 "  rf_shifting: SD3\n")
    c = load_train_config_from_yaml(str(p))
    assert c.rf_sampler == "LinearQuadratic"
    assert c.rf_log_normal_mu is None and c.rf_log_normal_sigma == 1.5
    assert c.batch_size == 4 and c.num_epochs is None and c.precision == "bf16"
    assert c.rf_shifting == "SD3" and c.lora_rank == 8
    p.write_text("train: {}\n")
    with pytest.raises(ValueError):
        load_train_config_from_yaml(str(p))


# ------------------------------------------------------------------------------- scheduler
def test_scheduler_shifts_match_reference():
    from ltx_amd.scheduler import RectifiedFlowScheduler
    d = load_file(os.path.join(GOLD, "rf_sched.safetensors"))
    t = d["t"]
    none = RectifiedFlowScheduler(num_train_timesteps=1000, shifting=None, base_resolution=1024)
    assert torch.equal(none.shift_timesteps(d["x0"].shape, t), d["shift_none"])
    sd3 = RectifiedFlowScheduler(shifting="SD3", target_shift_terminal=0.1)
    assert torch.allclose(sd3.shift_timesteps(torch.Size([3, 4096, 128]), t), d["shift_sd3"],
                          rtol=1e-6, atol=1e-7)
    sdf = RectifiedFlowScheduler(shifting="SimpleDiffusion", base_resolution=1024)
    assert torch.allclose(sdf.shift_timesteps(torch.Size([3, 4096, 128]), t), d["shift_simple"],
                          rtol=1e-6, atol=1e-7)


def test_sample_timesteps_matches_reference():
    """training.py:124-132 with the golden's seed: identical draws and quantile clamp."""
    from ltx_amd.config import TrainConfig
    from ltx_amd.training import sample_timesteps
    d = load_file(os.path.join(GOLD, "rf_sched.safetensors"))
    with open(os.path.join(GOLD, "rf_sched.json")) as f:
        meta = json.load(f)
    cfg = TrainConfig(checkpoint_path="-", rf_log_normal_mu=-0.5, rf_log_normal_sigma=1.0)
    torch.manual_seed(meta["tsample_seed"])
    t = sample_timesteps(8, cfg, "cpu")
    assert torch.equal(t, d["tsample_t"])
    assert float(t.min()) >= 0.0 and float(t.max()) <= 1.0


# --------------------------------------------------------------------- module tree / naming
def _meta_model(cfg, r):
    from ltx_amd.config import TrainConfig
    from ltx_amd.lora import apply_training_strategy
    from ltx_amd.transformer3d import Transformer3DModel
    with torch.device("meta"):
        m = Transformer3DModel.from_config(cfg)
        if r:
            apply_training_strategy(m, TrainConfig(checkpoint_path="-", lora_rank=r, lora_alpha=r),
                                    "lora_audio")
    return m


def test_tiny_param_names_match_reference_peft_model():
    d, meta = _tiny()
    m = _meta_model(meta["config"], meta["lora_rank"])
    ours = {canonical_name(n): tuple(p.shape) for n, p in m.named_parameters()}
    ref = {k[2:]: tuple(v.shape) for k, v in d.items() if k.startswith("w.")}
    assert ours == ref
    trainable = {canonical_name(n) for n, p in m.named_parameters() if p.requires_grad}
    assert trainable == {k[5:] for k in d if k.startswith("grad.")}
    # raw (un-canonicalised) names keep peft's layout
    raw = [n for n, _ in m.named_parameters() if "attn2.to_out.0" in n]
    assert any(n.endswith("attn2.to_out.0.base_layer.weight") for n in raw)
    assert any(n.endswith("attn2.to_out.0.lora_B.default.weight") for n in raw)


def test_ltx2b_param_counts():
    """1,923,385,472 base parameters + 7,340,032 LoRA (r=16); 19,927,040 trainable."""
    from ltx_amd.transformer3d import OURS_TRANSFORMER_CONFIG
    m = _meta_model(OURS_TRANSFORMER_CONFIG, 16)
    total = sum(p.numel() for p in m.parameters())
    train = sum(p.numel() for p in m.parameters() if p.requires_grad)
    lora = sum(p.numel() for n, p in m.named_parameters() if "lora_" in n)
    assert train == 19_927_040
    assert total - lora == 1_923_385_472
    assert lora == 28 * 4 * 16 * (2048 + 2048)


def test_full_strategy_trainable_set():
    """training.py:75-91 substring rule ('full' mode): FF and patchify_proj stay frozen."""
    from ltx_amd.config import TrainConfig
    from ltx_amd.lora import apply_training_strategy
    from ltx_amd.transformer3d import OURS_TRANSFORMER_CONFIG
    m = _meta_model(OURS_TRANSFORMER_CONFIG, 0)
    apply_training_strategy(m, TrainConfig(checkpoint_path="-"), "full")
    train = {n for n, p in m.named_parameters() if p.requires_grad}
    assert not any(".ff." in n or n.startswith("patchify_proj") for n in train)
    assert "scale_shift_table" in train and "proj_out.weight" in train
    assert any("attn1.to_q" in n for n in train) and any("attn2.k_norm" in n for n in train)
    assert abs(sum(p.numel() for n, p in m.named_parameters() if n in train) - 983.3e6) < 0.05e6


def test_skip_layer_mask():
    """transformer3d.py:187-203."""
    d, meta = _tiny()
    m = _meta_model(meta["config"], 0)
    assert m.create_skip_layer_mask(2, 3, 1, None) is None
    m = m.to_empty(device="cpu")
    mask = m.create_skip_layer_mask(2, 3, 1, [0])
    assert mask.shape == (len(m.transformer_blocks), 6)
    assert mask[0].tolist() == [1, 0, 1, 1, 0, 1] and mask[1].eq(1).all()


# -------------------------------------------------------------------- checkpoints / merging
def _tiny_state(d):
    return {k[2:]: v for k, v in d.items() if k.startswith("w.") and "lora_" not in k}


def test_from_pretrained_single_file_roundtrip(tmp_path):
    """Single-file safetensors with metadata['config'] (transformer3d.py:337-352), including the
    ComfyUI 'model.diffusion_model.' prefix (transformer3d.py:279-292)."""
    from ltx_amd.patchifier import SymmetricPatchifier
    from ltx_amd.transformer3d import Transformer3DModel
    d, meta = _tiny()
    state = {k: v.contiguous() for k, v in _tiny_state(d).items()}
    md = {"config": json.dumps({"transformer": meta["config"]})}
    for prefix in ("", "model.diffusion_model."):
        path = tmp_path / f"ckpt{len(prefix)}.safetensors"
        save_file({prefix + k: v for k, v in state.items()}, str(path), metadata=md)
        m = Transformer3DModel.from_pretrained(str(path), patchifier=SymmetricPatchifier(1))
        got = m.state_dict()
        assert set(got) == set(state)
        for k, v in state.items():
            assert torch.equal(got[k], v), k
        assert m.dtype == torch.bfloat16 and m.device.type == "cpu"
        assert isinstance(m.patchifier, SymmetricPatchifier)


def test_merged_state_dict_folds_lora():
    """peft merge_and_unload as save_training_checkpoint exports it (torch_utils.py:66-102)."""
    from ltx_amd.lora import merged_state_dict
    d, meta = _tiny()
    m = _meta_model(meta["config"], meta["lora_rank"])
    sd = {}
    for n, _ in m.named_parameters():
        sd[n] = d["w." + canonical_name(n)].clone()
    m.load_state_dict(sd, assign=True, strict=True)
    out = merged_state_dict(m)
    assert not any("lora_" in k or "base_layer" in k for k in out)
    ref_keys = {k for k in _tiny_state(d)}
    assert set(out) == ref_keys
    blk = "transformer_blocks.0.attn2.to_q"
    w = d[f"w.{blk}.weight"].float()
    a = d[f"w.{blk}.lora_A.default.weight"].float()
    b = d[f"w.{blk}.lora_B.default.weight"].float()
    s = meta.get("lora_alpha", meta["lora_rank"]) / meta["lora_rank"]
    assert torch.equal(out[f"{blk}.weight"], (w + s * (b @ a)).to(torch.bfloat16))


def test_product_ops_refuse_cpu_tensors():
    """No CPU fallback: the product path raises instead of computing on the host."""
    from ltx_amd import ops
    with pytest.raises(Exception):
        ops.patchify(torch.zeros(1, 4, 1, 2, 2, dtype=torch.bfloat16))


# ------------------------------------------------------------------------ DP all-reduce (gloo)
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _dp_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ltx_amd.training import GradAllReduce
        torch.manual_seed(0)
        params = [torch.nn.Parameter(torch.zeros(s, dtype=dt)) for s, dt in
                  [((16, 64), torch.float32), ((64, 16), torch.float32), ((300,), torch.bfloat16),
                   ((7, 5), torch.float32), ((1000,), torch.bfloat16)]]
        g = torch.Generator().manual_seed(100 + rank)
        for i, p in enumerate(params):
            if i == 3 and rank == 0:
                continue  # a missing grad on one rank counts as zeros
            p.grad = torch.randn(p.shape, generator=g).to(p.dtype)
        red = GradAllReduce(params, bucket_mb=0.004)  # several buckets
        assert len(red.buckets) > 1
        red()
        torch.save({i: p.grad for i, p in enumerate(params)}, os.path.join(out_dir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_grad_allreduce_gloo_world2():
    world = 2
    with tempfile.TemporaryDirectory() as td:
        mp.start_processes(_dp_worker, args=(world, _free_port(), td), nprocs=world,
                           start_method="spawn", join=True)
        res = [torch.load(os.path.join(td, f"r{r}.pt"), weights_only=True) for r in range(world)]
    shapes = [((16, 64), torch.float32), ((64, 16), torch.float32), ((300,), torch.bfloat16),
              ((7, 5), torch.float32), ((1000,), torch.bfloat16)]
    expect = []
    for i, (s, dt) in enumerate(shapes):
        acc = torch.zeros(s, dtype=torch.float32)
        for r in range(world):
            g = torch.Generator().manual_seed(100 + r)
            for j, (s2, dt2) in enumerate(shapes[:i + 1]):
                if j == 3 and r == 0:
                    continue
                v = torch.randn(s2, generator=g).to(dt2)
            if not (i == 3 and r == 0):
                acc += v.float()
        expect.append((acc / world).to(dt))
    for r in range(world):
        for i, e in enumerate(expect):
            got = res[r][i]
            assert got.dtype == e.dtype
            assert torch.equal(got, e), (r, i)
    assert math.isfinite(float(expect[0].sum()))


class _FakeBlockFn(torch.autograd.Function):
    """y = (x + mods) . W with W (under blk.attn2, as the LoRA adapters / attention weights sit in
    the real block) written straight into .grad and the block's ready hooks called at the end of
    backward: the contract of transformer3d._BlockFn. mods stands for the AdaLN modulation rows
    (scale_shift_table + tmod through _AdaModFn): its gradient is RETURNED, so the table's .grad
    is accumulated by autograd after the hooks have fired."""

    @staticmethod
    def forward(ctx, blk, x, mods):
        ctx.blk = blk
        xm = x + mods
        ctx.save_for_backward(xm)
        return xm @ blk.attn2.w

    @staticmethod
    def backward(ctx, dy):
        (xm,) = ctx.saved_tensors
        blk = ctx.blk
        w = blk.attn2.w
        with torch.no_grad():
            if w.grad is None:
                w.grad = torch.zeros_like(w)
            w.grad.add_(xm.t() @ dy)
        for cb in getattr(blk, "_grad_ready_hooks", ()):
            cb(blk)
        dx = dy @ w.t()
        return None, dx, dx.sum(0, keepdim=True)


class _FakeModel(torch.nn.Module):
    """caption (bf16, autograd-accumulated) -> 3 blocks (f32 grads written by the 'kernel');
    full=True also trains each block's scale_shift_table (autograd-accumulated, like
    train_mode='full')."""

    def __init__(self, full=False):
        super().__init__()
        g = torch.Generator().manual_seed(3)
        self.cap = torch.nn.Parameter(torch.randn(8, 8, generator=g).to(torch.bfloat16))
        self.transformer_blocks = torch.nn.ModuleList()
        for _ in range(3):
            b = torch.nn.Module()
            b.attn2 = torch.nn.Module()
            b.attn2.w = torch.nn.Parameter(torch.randn(8, 8, generator=g) * 0.3)
            b.scale_shift_table = torch.nn.Parameter(torch.randn(1, 8, generator=g) * 0.1,
                                                     requires_grad=full)
            self.transformer_blocks.append(b)

    def forward(self, x):
        h = (x.to(torch.bfloat16) @ self.cap).float()
        for b in self.transformer_blocks:
            h = _FakeBlockFn.apply(b, h, b.scale_shift_table * 1.0)
        return h

    def grad_ready_order(self):
        order = []
        for b in reversed(self.transformer_blocks):
            order += [p for p in b.parameters() if p.requires_grad]
        return order + [self.cap]


def _dp_overlap_worker(rank, world, port, out_dir, full):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ltx_amd.training import GradAllReduce
        res = {}
        for mode in ("overlap", "posthoc"):
            m = _FakeModel(full)
            params = [p for p in m.parameters() if p.requires_grad]
            launched_at_cap, box = [], []
            # registered first: runs before the reducer's own hook on the caption grad
            m.cap.register_post_accumulate_grad_hook(lambda p: launched_at_cap.append(box[0]._launched))
            # a stale reducer installed and removed first: its hooks must be gone
            GradAllReduce(params, bucket_mb=1e-5, order=m.grad_ready_order()).install(m).uninstall()
            snaps = {}

            class Rec(GradAllReduce):  # the bucket contents at the moment its all-reduce launches
                def _launch(self, bi):
                    snaps[bi] = self.buckets[bi]["flat"].clone()
                    super()._launch(bi)
            red = Rec(params, bucket_mb=1e-5, order=m.grad_ready_order()).install(m)
            box.append(red)
            assert all(len(b.__dict__.get("_grad_ready_hooks", [])) == 1 for b in m.transformer_blocks)
            assert len(red.buckets) == len(params)  # one param each
            red.zero_grad()
            g = torch.Generator().manual_seed(100 + rank)
            for step in range(3):  # three micro-steps, the last one armed
                if mode == "overlap" and step == 2:
                    red.arm()
                x = torch.randn(4, 8, generator=g)
                m(x).square().sum().backward()
            red()
            res[mode] = {"grads": [p.grad.clone() for p in params],
                         "views": all(p.grad.data_ptr() == red._view(*[(b, j) for b in red.buckets
                                      for j, q in enumerate(b["params"]) if q is p][0]).data_ptr()
                                      for p in params),
                         "launched_at_cap": launched_at_cap[-1]}
            # local (unreduced) grads of this rank for the expected average
            m2 = _FakeModel(full)
            g = torch.Generator().manual_seed(100 + rank)
            for step in range(3):
                m2(torch.randn(4, 8, generator=g)).square().sum().backward()
            res[mode]["local"] = [p.grad.clone() for p in m2.parameters() if p.requires_grad]
            # every bucket launched holding this rank's complete local gradient
            local = {id(q): g2 for q, g2 in zip(params, res[mode]["local"])}
            res[mode]["complete_at_launch"] = all(
                torch.equal(snaps[bi], torch.cat([local[id(q)].reshape(-1) for q in b["params"]]))
                for bi, b in enumerate(red.buckets))
        torch.save(res, os.path.join(out_dir, f"o{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("full", [False, True], ids=["lora", "full"])
def test_grad_allreduce_overlapped_with_backward_gloo_world2(full):
    """GradAllReduce armed for the last micro-step launches the block buckets from the blocks'
    backward hooks (before the caption grad exists) and ends bitwise equal to the post-backward
    reduction, equal to the f32 mean of the ranks' grads, with .grad kept as bucket views.
    full: each block's scale_shift_table gets its gradient from autograd AFTER the block's hook
    has fired; it must report through its post-accumulate-grad hook, not the block hook, or its
    bucket reduces without the last micro-step's term."""
    world = 2
    with tempfile.TemporaryDirectory() as td:
        mp.start_processes(_dp_overlap_worker, args=(world, _free_port(), td, full), nprocs=world,
                           start_method="spawn", join=True)
        res = [torch.load(os.path.join(td, f"o{r}.pt"), weights_only=True) for r in range(world)]
    for r in range(world):
        ov, ph = res[r]["overlap"], res[r]["posthoc"]
        if not full:
            assert ov["launched_at_cap"] == 3, "the three block buckets launch during the backward"
        else:
            assert ov["launched_at_cap"] >= 1, "block buckets launch during the backward"
        assert ph["launched_at_cap"] == 0
        assert ov["complete_at_launch"] and ph["complete_at_launch"]
        assert ov["views"] and ph["views"]
        for a, b in zip(ov["grads"], ph["grads"]):
            assert torch.equal(a, b)
    for i in range(len(res[0]["overlap"]["grads"])):
        exp = sum(res[r]["overlap"]["local"][i].float() for r in range(world)) / world
        exp = exp.to(res[0]["overlap"]["grads"][i].dtype)
        for r in range(world):
            assert torch.equal(res[r]["overlap"]["grads"][i], exp), (r, i)


# ------------------------------------------------------------------ ZeRO-2 (gloo, world 2 / 3 / 8)
ZSHAPES = [(16, 64), (64,), (300,), (7, 5), (1001,)]
Z_LR, Z_CLIP, Z_STEPS = 1e-2, 0.5, 3


def _ref_adamw(master, g, m, v, step, lr, b1=0.9, b2=0.999, eps=1e-8, wd=1e-2):
    """torch.optim.AdamW's single-tensor update (the math ltx_adamw_step implements)."""
    master.mul_(1 - lr * wd)
    m.lerp_(g, 1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    master.addcdiv_(m, denom, value=-lr / bc1)


def _clip_coef(sumsq, world, clip):
    """ltx_clip_scale_f32's factor: the averaged grads' global norm -> min(1, clip / (norm + 1e-6)),
    applied with the 1/world average as one f32 multiplier"""
    norm = math.sqrt(sumsq) / world
    c = min(1.0, clip / (norm + 1e-6)) if clip > 0 else 1.0
    return torch.tensor(c / world, dtype=torch.float32)


def _zero_cpu_cls():
    """Zero2AdamW with its HIP kernels swapped for torch math: the CPU gloo test checks the
    partition, bucketing, collectives and clip bookkeeping (the kernels are covered on the GPU)."""
    from ltx_amd.zero import Zero2AdamW

    class CpuZero2(Zero2AdamW):
        def _cast_to_f32(self, src, dst):
            dst.copy_(src.float())

        def _cast_to_bf16(self, src, dst):
            dst.copy_(src.to(torch.bfloat16))

        def _sumsq(self, x, out):
            out.fill_(float((x.double() ** 2).sum()))

        def _clip_scale(self, x, sumsq, coef):
            coef.copy_(_clip_coef(float(sumsq), self.world, self.clip))
            x.mul_(coef)

        def _adamw(self, master, g, m, v, step):
            _ref_adamw(master, g, m, v, step, self.lr)
    return CpuZero2


def _exact_grad(shape, g):
    """grads whose f32 sums over up to 8 ranks are exact in any order (multiples of 2^-6 in
    [-2, 2], exact in bf16), so a reduce-scatter matches the sequential sum bit for bit"""
    return (torch.randint(-128, 129, shape, generator=g).float() / 64).to(torch.bfloat16)


class _FakeBlockBf16(torch.nn.Module):
    def __init__(self, g):
        super().__init__()
        self.attn2 = torch.nn.Module()
        self.attn2.w = torch.nn.Parameter((torch.randn(8, 8, generator=g) * 0.3).to(torch.bfloat16))
        self.scale_shift_table = torch.nn.Parameter((torch.randn(1, 8, generator=g) * 0.1).to(torch.bfloat16))


class _FakeZeroModel(torch.nn.Module):
    """bf16 twin of _FakeModel for ZeRO-2 (train_mode='full'): caption + 3 blocks whose attn2
    weight gradient is written by the 'kernel' (block hook) and whose scale_shift_table gradient
    autograd accumulates after the block's backward (post-accumulate-grad hook)."""

    def __init__(self):
        super().__init__()
        g = torch.Generator().manual_seed(3)
        self.cap = torch.nn.Parameter(torch.randn(8, 8, generator=g).to(torch.bfloat16))
        self.transformer_blocks = torch.nn.ModuleList([_FakeBlockBf16(g) for _ in range(3)])

    def forward(self, x):
        h = x.to(torch.bfloat16) @ self.cap
        for b in self.transformer_blocks:
            h = _FakeBlockFn.apply(b, h, b.scale_shift_table * 1.0)
        return h

    def grad_ready_order(self):
        order = []
        for b in reversed(self.transformer_blocks):
            order += [p for p in b.parameters() if p.requires_grad]
        return order + [self.cap]


def _zero_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = {}
        # (a) the partition / bucket / clip bookkeeping against single-process math
        g0 = torch.Generator().manual_seed(7)
        params = [torch.nn.Parameter(torch.randn(s, generator=g0).to(torch.bfloat16)) for s in ZSHAPES]
        opt = _zero_cpu_cls()(params, lr=Z_LR, gradient_clipping=Z_CLIP, bucket_elems=512)
        assert len(opt.buckets) > 2 and all(b["n"] % world == 0 for b in opt.buckets)
        g = torch.Generator().manual_seed(100 + rank)
        for _ in range(Z_STEPS):
            for p in params:  # accumulate into the flat-buffer views, as the kernels do
                p.grad.add_(_exact_grad(p.shape, g))
            opt.step()
            opt.zero_grad()
        res["math"] = [p.detach().clone() for p in params]
        # (b) overlap_comm: the armed path (reduce-scatters launched from the backward's hooks)
        # against the post-hoc one, and the bf16 reduction next to the f32 one
        for mode in ("armed", "posthoc", "bf16"):
            m = _FakeZeroModel()
            launched_at_cap, box = [], []
            m.cap.register_post_accumulate_grad_hook(lambda p: launched_at_cap.append(box[0]._launched))
            kw = dict(lr=Z_LR, gradient_clipping=Z_CLIP, bucket_elems=72, order=m.grad_ready_order())
            if mode == "bf16":
                kw["reduce_dtype"] = torch.bfloat16
            opt = _zero_cpu_cls()(list(m.parameters()), **kw)
            if mode == "armed":
                opt.install(m)
            box.append(opt)
            g = torch.Generator().manual_seed(200 + rank)
            for step in range(2):
                for micro in range(3):
                    if mode == "armed" and micro == 2:
                        opt.arm()
                    x = (torch.randint(-4, 5, (4, 8), generator=g).float() / 4)
                    m(x).float().square().sum().backward()
                opt.step()
                opt.zero_grad()
            res[mode] = {"params": [p.detach().clone() for p in m.parameters()],
                         "launched_at_cap": launched_at_cap[2] if launched_at_cap else -1,
                         "buckets": len(opt.buckets)}
        torch.save(res, os.path.join(out_dir, f"z{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_zero2_gloo_matches_single_process_math(world):
    """Zero2AdamW at world 2, 3 (padded buckets) and 8 over gloo: the final weights of every rank
    are BITWISE those of one process keeping an f32 master of all parameters and applying the
    averaged, globally clipped gradients with torch AdamW's math (the grads are exact under any
    summation order); the overlapped (armed) reduce-scatter path is bitwise the post-hoc one and
    launches the block buckets during the backward; the bf16 reduction stays within bf16 rounding."""
    with tempfile.TemporaryDirectory() as td:
        mp.start_processes(_zero_worker, args=(world, _free_port(), td), nprocs=world,
                           start_method="spawn", join=True)
        res = [torch.load(os.path.join(td, f"z{r}.pt"), weights_only=True) for r in range(world)]
    # (a) reference: one process, f32 master of all params, averaged + globally clipped grads
    g0 = torch.Generator().manual_seed(7)
    params = [torch.randn(s, generator=g0).to(torch.bfloat16) for s in ZSHAPES]
    master = [p.float() for p in params]
    m = [torch.zeros_like(x) for x in master]
    v = [torch.zeros_like(x) for x in master]
    gens = [torch.Generator().manual_seed(100 + r) for r in range(world)]
    for step in range(1, Z_STEPS + 1):
        sums = [torch.zeros_like(x) for x in master]
        for r in range(world):
            for i, s in enumerate(ZSHAPES):
                sums[i] += _exact_grad(s, gens[r]).float()
        sumsq = sum(float((x.double() ** 2).sum()) for x in sums)
        coef = _clip_coef(sumsq, world, Z_CLIP)
        for i in range(len(master)):
            _ref_adamw(master[i], sums[i] * coef, m[i], v[i], step, Z_LR)
    expect = [x.to(torch.bfloat16) for x in master]
    for r in range(world):
        for i, e in enumerate(expect):
            assert torch.equal(res[r]["math"][i], e), (world, r, i)
    # (b) overlap_comm
    for r in range(world):
        armed, post, b16 = res[r]["armed"], res[r]["posthoc"], res[r]["bf16"]
        assert armed["buckets"] > 2
        assert armed["launched_at_cap"] >= 1, "block buckets reduce-scatter during the backward"
        assert post["launched_at_cap"] == 0
        for a, b_, c in zip(armed["params"], post["params"], b16["params"]):
            assert torch.equal(a, b_)
            assert torch.allclose(c.float(), a.float(), rtol=0, atol=2e-2)
        for i, a in enumerate(armed["params"]):
            assert torch.equal(a, res[0]["armed"]["params"][i])  # every rank holds the same weights


def test_sample_timesteps_is_the_lognormal_draw_bitwise():
    """train_step's timestep draw writes LogNormal(mu, sigma).sample((B,)) out (normal_(0, 1),
    mul_(sigma), add_(mu), exp) to avoid the distribution's host syncs; it must stay the same draw
    and the same roundings as the reference's (training.py:124-132)."""
    from ltx_amd.training import sample_timesteps

    class C:
        rf_log_normal_mu, rf_log_normal_sigma = -0.5, 1.0
        rf_quantile_min, rf_quantile_max = 0.01, 0.99

    for seed in (0, 7, 123):
        torch.manual_seed(seed)
        a = sample_timesteps(16, C, "cpu")
        torch.manual_seed(seed)
        raw = torch.distributions.LogNormal(torch.tensor(-0.5), torch.tensor(1.0)).sample((16,))
        t = raw / (1 + raw)
        b = t.clamp(min=float(torch.quantile(t, 0.01)), max=float(torch.quantile(t, 0.99)))
        assert torch.equal(a, b)
