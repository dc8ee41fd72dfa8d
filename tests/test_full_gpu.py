"""train_mode='full' (SURVEY a16, 8f row 2 -- BASELINE config Z's trainable set) on the MI355X:
the tiny model's train step through the HIP library against the REFERENCE's grads for every
trainable tensor (tests/golden/tiny_full_step: attention weights/biases, q/k norm weights, every
scale_shift_table, adaln_single, caption_projection, proj_out), with the SURVEY 8c-4 noise
criterion (the pinned oracle in fp32 on the device as the yardstick)."""
import json
import os

import pytest
import torch
from safetensors.torch import load_file

import ltx_oracle as O
from model_utils import grads_by_canonical, loss_crit, rel

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DEV = "cuda"
FULL_KEYS = ("proj_out", "scale_shift_table", "adaln_single", "caption_projection", "attn")


def _load():
    with open(os.path.join(GOLD, "tiny_full_step.json")) as f:
        meta = json.load(f)
    return load_file(os.path.join(GOLD, "tiny_full_step.safetensors")), meta


def _build_full(cfg, params):
    from ltx_amd.config import TrainConfig
    from ltx_amd.lora import apply_training_strategy
    from ltx_amd.patchifier import SymmetricPatchifier
    from ltx_amd.transformer3d import Transformer3DModel
    from params import canonical_name
    with torch.device("meta"):
        m = Transformer3DModel.from_config(cfg)
    m.load_state_dict({n: params[canonical_name(n)].detach().to(DEV).clone()
                       for n, _ in m.named_parameters()}, assign=True, strict=True)
    apply_training_strategy(m, TrainConfig(checkpoint_path="-"), "full")
    m.patchifier = SymmetricPatchifier(1)
    m.train()
    return m


def _run(model, d):
    from ltx_amd.config import TrainConfig
    from ltx_amd.scheduler import RectifiedFlowScheduler
    from ltx_amd.training import train_step
    c = lambda x: x.to(DEV)  # noqa: E731
    return train_step(model, {"latents": c(d["in.latents"]),
                              "ref_image_latents": c(d["in.ref_image_latents"]),
                              "pose_latents": c(d["in.pose_latents"])},
                      RectifiedFlowScheduler(), model.patchifier,
                      TrainConfig(checkpoint_path="-", gradient_accumulation_steps=1),
                      c(d["in.prompt_embeds"]), c(d["in.prompt_attention_mask"]),
                      t=c(d["out.t"]), noise=c(d["out.noise"]).bfloat16())


def test_full_mode_grads_match_reference():
    d, meta = _load()
    cfg = meta["config"]
    params = O.make_params(cfg, meta["param_seed"], lora_rank=0, requires_grad=False)
    model = _build_full(cfg, params)
    assert sorted(grads_by_canonical(model)) == meta["trainable"]
    loss, _, _, ld = _run(model, d)
    g = grads_by_canonical(model)
    # fp32 oracle on the device: the yardstick of the reference's own bf16 noise
    q = {k: v.to(DEV).float().requires_grad_(any(s in k for s in FULL_KEYS))
         for k, v in params.items()}
    c = lambda x: x.to(DEV)  # noqa: E731
    r = O.train_step(q, cfg, c(d["in.latents"]), c(d["in.ref_image_latents"]),
                     c(d["in.pose_latents"]), c(d["in.prompt_embeds"]),
                     c(d["in.prompt_attention_mask"]), t=c(d["out.t"]),
                     noise=c(d["out.noise"]).float())
    r["loss"].backward()
    # loss: the f32 mse vs the fp32 oracle, the reference's bf16 output as the noise yardstick
    # (the golden holds no v_target: v = noise - x0 in f32, rounded to bf16 as training.py:146 does)
    l16 = float(((d["out.sample"].to(DEV).float() - r["v_target"].detach().bfloat16().float()) ** 2).mean())
    l32 = float(((r["sample"].float() - r["v_target"].float()) ** 2).mean())
    loss_crit("tiny full loss", ld["_mse_f32"], l16, l32)
    assert abs(float(loss) - float(d["out.loss"])) <= 2 ** -7 * abs(float(d["out.loss"]))
    worst = []
    for k, v in d.items():
        if not k.startswith("grad."):
            continue
        name = k[5:]
        assert g[name] is not None, name
        e_b, e_r = rel(g[name], q[name].grad), rel(v.to(DEV), q[name].grad)
        worst.append((e_b - 1.25 * e_r, name, e_b, e_r))
        assert e_b <= 1.25 * e_r + 1e-2, f"{name}: build {e_b:.3e} vs reference bf16 noise {e_r:.3e}"
    worst.sort(reverse=True)
    print("worst margins:", worst[:4])


def test_full_mode_accumulates_over_micro_steps():
    """Two micro-steps accumulate into .grad (the reference's loss.backward() per micro-batch)."""
    d, meta = _load()
    cfg = meta["config"]
    params = O.make_params(cfg, meta["param_seed"], lora_rank=0, requires_grad=False)
    model = _build_full(cfg, params)
    _run(model, d)
    g1 = {k: v.clone() for k, v in grads_by_canonical(model).items()}
    _run(model, d)
    g2 = grads_by_canonical(model)
    for k in g1:
        assert rel(g2[k], 2 * g1[k]) < 2e-2, k


def test_zero2_kernels_match_torch_math():
    """Zero2AdamW at world size 1 through the HIP kernels (cast, sumsq, clip_scale, adamw) vs
    grad-norm clipping + f32-master torch AdamW; params/grads stay views of the flat buffers."""
    from ltx_amd.zero import Zero2AdamW
    g = torch.Generator(device=DEV).manual_seed(3)
    shapes = [(256, 64), (64,), (1000,), (3, 7)]
    params = [torch.nn.Parameter(torch.randn(s, generator=g, device=DEV).bfloat16()) for s in shapes]
    master = [p.detach().float().clone().requires_grad_(True) for p in params]
    ref = torch.optim.AdamW(master, lr=1e-2, foreach=False)
    opt = Zero2AdamW(params, lr=1e-2, gradient_clipping=1.0)
    for p in params:
        assert p.data.untyped_storage().data_ptr() == opt.flat_param.untyped_storage().data_ptr()
        assert p.grad.untyped_storage().data_ptr() == opt.flat_grad.untyped_storage().data_ptr()
    for step in range(4):
        scale = 0.01 if step == 2 else 1.0  # one step under the clip threshold
        grads = [torch.randn(s, generator=g, device=DEV).bfloat16() * scale for s in shapes]
        for p, gr in zip(params, grads):
            p.grad.add_(gr)
        for m, gr in zip(master, grads):
            m.grad = gr.float()
        norm = torch.nn.utils.clip_grad_norm_(master, 1.0)
        opt.step()
        ref.step()
        assert abs(opt.grad_norm() - float(norm)) <= 1e-4 * float(norm)
        opt.zero_grad()
        for p, m in zip(params, master):
            assert torch.equal(p.detach(), m.detach().bfloat16()) or \
                rel(p.detach().float(), m.detach()) < 1e-5
    assert float(opt.flat_grad.abs().max()) == 0.0


def test_full_mode_zero2_loss_curve():
    """5 optimizer steps of the full-mode tiny model with Zero2AdamW (world 1) vs the oracle +
    clip_grad_norm_(1.0) + torch AdamW on the same t / noise streams (bf16 weights on an f32
    master and an all-fp32 trajectory; SURVEY 8c-4 loss criterion per step)."""
    from ltx_amd.zero import Zero2AdamW
    d, meta = _load()
    cfg = meta["config"]
    params = O.make_params(cfg, meta["param_seed"], lora_rank=0, requires_grad=False)
    model = _build_full(cfg, params)
    # lr 1e-4: train-avatars.yaml's learning_rate (the trajectories stay within the per-step noise
    # criterion; at 10x the configured lr a bf16 trajectory drifts past 1e-3 by step 2 by itself)
    opt = Zero2AdamW([p for p in model.parameters() if p.requires_grad], lr=1e-4)
    refs = {}  # bf16 weights + f32 master (the bf16 config), and an all-fp32 trajectory
    for dt in (torch.bfloat16, torch.float32):
        q = {k: v.to(DEV).to(dt).requires_grad_(any(s in k for s in FULL_KEYS)) for k, v in params.items()}
        qt = [v for v in q.values() if v.requires_grad]
        qm = [v.detach().float().clone().requires_grad_(True) for v in qt]
        refs[dt] = (q, qt, qm, torch.optim.AdamW(qm, lr=1e-4, foreach=False))
    g = torch.Generator(device=DEV).manual_seed(11)
    lat = d["in.latents"]
    B, C = lat.shape[:2]
    N = lat[0, 0].numel()
    ours, curves = [], {torch.bfloat16: [], torch.float32: []}
    c = lambda x: x.to(DEV)  # noqa: E731
    for _ in range(5):
        t = torch.rand(B, generator=g, device=DEV) * 0.9 + 0.05
        noise = torch.randn(B, N, C, generator=g, device=DEV).bfloat16()
        dd = dict(d)
        dd["out.t"], dd["out.noise"] = t, noise
        _, _, _, ld = _run(model, dd)
        opt.step()
        opt.zero_grad()
        for dt, (q, qt, qm, ref) in refs.items():
            r = O.train_step(q, cfg, c(d["in.latents"]), c(d["in.ref_image_latents"]),
                             c(d["in.pose_latents"]), c(d["in.prompt_embeds"]),
                             c(d["in.prompt_attention_mask"]), t=t, noise=noise.to(dt))
            r["loss"].backward()
            for v, m in zip(qt, qm):
                m.grad = v.grad.float()
                v.grad = None
            torch.nn.utils.clip_grad_norm_(qm, 1.0)
            ref.step()
            with torch.no_grad():
                for v, m in zip(qt, qm):
                    v.copy_(m.to(dt))
            curves[dt].append(float(((r["sample"].float() - r["v_target"].float()) ** 2).mean()))
        ours.append(float(ld["_mse_f32"]))
    for i, a in enumerate(ours):
        loss_crit(f"full curve step {i}", a, curves[torch.bfloat16][i], curves[torch.float32][i])
