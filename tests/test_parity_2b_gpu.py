"""LTX-2B-width parity on the MI355X for the configurations BASELINE.json names:

  * config X attention: self-attention at B=1, H=32, Nq=Nk=7488, d=64 (97 frames at 768^2) vs the
    reference's own op, F.scaled_dot_product_attention (attention.py:1057-1064), in bf16 and fp32;
  * config X block: one LTX-2B block at latent 13x24x24 (N=7488) through train_step vs the oracle;
  * config A path: a 2-block LTX-2B-width model at B=8 with ONE prompt expanded over the batch
    (the bench's text_shared path: shared text K/V, batch-summed dK/dV, caption projection run
    once) vs the oracle run per sample -- out.sample, every LoRA and caption-projection gradient,
    and the loss;
  * LTX-2B loss curve: 20 seeded optimizer steps of that 2-block model (LoRA r=16, shared prompt,
    B=8) -- train_step + FusedAdamW vs the oracle + torch AdamW in bf16 and in fp32.

Criterion: err(build_bf16, ref_fp32) <= 1.25 * err(ref_bf16, ref_fp32) + slack,
rel-Frobenius, with the oracle / torch's own bf16 op as the bf16 reference; loss scalars (f32
means, not the bf16-rounded scalar) within 1e-3 relative of the fp32 reference or within the
reference's own bf16 noise on that loss, whichever is larger.
"""
import pytest
import torch
import torch.nn.functional as F

import ltx_oracle as O
from model_utils import build_model, grads_by_canonical, rel

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _crit(name, build, ref16, ref32, factor=1.25, slack=2e-3):
    e_b, e_r = rel(build.float(), ref32.float()), rel(ref16.float(), ref32.float())
    assert e_b <= factor * e_r + slack, f"{name}: build err {e_b:.3e} vs reference bf16 noise {e_r:.3e}"
    return e_b, e_r


def _loss_crit(name, lb, l16, l32):
    e_b, e_r = abs(lb - l32) / abs(l32), abs(l16 - l32) / abs(l32)
    assert e_b <= max(1e-3, 1.25 * e_r + 1e-4), f"{name}: loss {lb} vs fp32 {l32} (bf16 ref {l16})"


def _sdpa(q, k, v, B, H, d):
    N = q.shape[0] // B
    sh = lambda x: x.view(B, N, H, d).transpose(1, 2)
    o = F.scaled_dot_product_attention(sh(q), sh(k), sh(v))
    return o.transpose(1, 2).reshape(B * N, H * d)


def test_attention_config_x_self_7488():
    """Config X's SDPA (B=1, 32 heads, Nq=Nk=7488, d=64): forward, lse, dQ/dK/dV."""
    from ltx_amd import ops
    B, H, N, d = 1, 32, 7488, 64
    g = torch.Generator(device=DEV).manual_seed(71)
    q, k, v, do = (torch.randn(B * N, H * d, generator=g, device=DEV).bfloat16() for _ in range(4))
    o, lse = ops.attn_fwd(q, k, v, B, H, d, d ** -0.5)
    dq, dk, dv = ops.attn_bwd(q, k, v, o, do, lse, B, H, d, d ** -0.5)
    outs = {}
    for dt in (torch.bfloat16, torch.float32):
        qq, kk, vv = (t.to(dt).clone().requires_grad_(True) for t in (q, k, v))
        oo = _sdpa(qq, kk, vv, B, H, d)
        oo.backward(do.to(dt))
        outs[dt] = (oo.detach(), qq.grad, kk.grad, vv.grad)
        del qq, kk, vv, oo
        torch.cuda.empty_cache()
    for i, (name, mine) in enumerate((("o", o), ("dq", dq), ("dk", dk), ("dv", dv))):
        _crit(f"X attention {name}", mine, outs[torch.bfloat16][i], outs[torch.float32][i])
    # lse (log2 units) against the fp32 logsumexp of the scaled scores, per head
    qh = q.float().view(N, H, d).transpose(0, 1)
    kh = k.float().view(N, H, d).transpose(0, 1)
    for h in (0, 17, 31):
        ref = torch.logsumexp((qh[h] @ kh[h].t()) * d ** -0.5, -1) / torch.log(torch.tensor(2.0))
        assert float((lse[0, h] - ref).abs().max()) < 1e-2


def _inputs(B, F_, H_, W_, L, n_valid, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    d = {"in.latents": torch.randn(B, 128, F_, H_, W_, generator=g, device=DEV),
         "in.ref_image_latents": torch.randn(B, 128, 1, H_, W_, generator=g, device=DEV),
         "in.pose_latents": torch.randn(B, 128, F_, H_, W_, generator=g, device=DEV),
         "in.prompt_embeds": torch.randn(1, L, 4096, generator=g, device=DEV),
         "in.prompt_attention_mask": (torch.arange(L, device=DEV) < n_valid).long().view(1, L),
         "out.t": torch.rand(B, generator=g, device=DEV) * 0.9 + 0.05}
    d["out.noise"] = torch.randn(B, F_ * H_ * W_, 128, generator=g, device=DEV).bfloat16()
    return d


def _oracle(params, cfg, d, dtype):
    q = {k: v.detach().to(DEV).to(torch.float32 if ("lora_" in k or dtype == torch.float32) else dtype)
         .requires_grad_(("lora_" in k) or ("caption_projection" in k)) for k, v in params.items()}
    r = O.train_step(q, cfg, d["in.latents"], d["in.ref_image_latents"], d["in.pose_latents"],
                     d["in.prompt_embeds"], d["in.prompt_attention_mask"], t=d["out.t"],
                     noise=d["out.noise"].to(dtype))
    r["loss"].backward()
    loss32 = float(((r["sample"].float() - r["v_target"].float()) ** 2).mean())
    return r["sample"].detach(), {k: v.grad for k, v in q.items() if v.requires_grad}, loss32


def _build_step(model, d):
    from ltx_amd.config import TrainConfig
    from ltx_amd.scheduler import RectifiedFlowScheduler
    from ltx_amd.training import train_step
    tc = TrainConfig(checkpoint_path="-", gradient_accumulation_steps=1)
    loss, _, _, ld = train_step(model, {"latents": d["in.latents"], "ref_image_latents": d["in.ref_image_latents"],
                                        "pose_latents": d["in.pose_latents"]},
                                RectifiedFlowScheduler(), model.patchifier, tc, d["in.prompt_embeds"],
                                d["in.prompt_attention_mask"], t=d["out.t"], noise=d["out.noise"])
    return float(ld["_mse_f32"])


def _sample(model, d):
    B = d["in.latents"].shape[0]
    tok, coords = O.patchify(d["in.latents"].bfloat16())
    x = O.add_noise(tok, d["out.noise"], d["out.t"]).bfloat16()
    with torch.no_grad():
        return model(hidden_states=x, indices_grid=coords.to(DEV),
                     ref_image_hidden_states=d["in.ref_image_latents"].bfloat16(),
                     pose_hidden_states=d["in.pose_latents"].bfloat16(),
                     encoder_hidden_states=d["in.prompt_embeds"].bfloat16().expand(B, -1, -1),
                     timestep=d["out.t"], encoder_attention_mask=d["in.prompt_attention_mask"].expand(B, -1)).sample


def _compare_model(tag, cfg, params, d, grad_names=None):
    model = build_model(cfg, params, 16, device=DEV)
    out = _sample(model, d)
    lb = _build_step(model, d)
    g = grads_by_canonical(model)
    s32, g32, l32 = _oracle(params, cfg, d, torch.float32)
    s16, g16, l16 = _oracle(params, cfg, d, torch.bfloat16)
    _crit(f"{tag} sample", out, s16, s32)
    _loss_crit(tag, lb, l16, l32)
    for name in grad_names or g32:
        _crit(f"{tag} {name}", g[name], g16[name], g32[name], slack=5e-3)
    return model


def test_block2b_config_x_latent():
    """One LTX-2B block at config X's latent 13x24x24 (N = 7488), B = 1, 256 text tokens (16 valid)."""
    from ltx_amd.transformer3d import OURS_TRANSFORMER_CONFIG
    cfg = dict(OURS_TRANSFORMER_CONFIG, num_layers=1)
    params = O.make_params(cfg, 29, lora_rank=16, requires_grad=False)
    d = _inputs(1, 13, 24, 24, 256, 16, seed=5)
    _compare_model("X block", cfg, params, d)


def test_two_blocks_b8_shared_prompt():
    """Config A's exact path at LTX-2B widths: B = 8 samples of 7x16x16 (N = 1792), ONE prompt
    of 256 tokens (16 valid) expanded over the batch -> text_shared (shared text K/V,
    batch-summed dK/dV, caption projection once) vs the oracle's per-sample computation; every
    LoRA (2 x 8 tensors) and caption-projection gradient."""
    from ltx_amd.transformer3d import OURS_TRANSFORMER_CONFIG
    cfg = dict(OURS_TRANSFORMER_CONFIG, num_layers=2)
    params = O.make_params(cfg, 31, lora_rank=16, requires_grad=False)
    d = _inputs(8, 7, 16, 16, 256, 16, seed=9)
    _compare_model("A 2-block B8", cfg, params, d)


@pytest.mark.timeout(600)
def test_config_a_exact_28_layers_b8():
    """Config A's benched shape in ONE comparison (VERDICT r05 #5a): the full 28-layer LTX-2B at
    B = 8, N = 1792 (7x16x16), one shared 256-token prompt with 16 valid tokens (bench.py's
    text_shared path), one train_step against the oracle in fp32 and bf16 on the same inputs and
    weights: out.sample, the loss and every trainable gradient (28 x 8 LoRA tensors + the caption
    projection) under SURVEY 8(c)-4's noise criterion."""
    from ltx_amd.transformer3d import OURS_TRANSFORMER_CONFIG
    cfg = dict(OURS_TRANSFORMER_CONFIG)
    assert cfg["num_layers"] == 28
    params = O.make_params(cfg, 61, lora_rank=16, requires_grad=False)
    d = _inputs(8, 7, 16, 16, 256, 16, seed=29)
    _compare_model("A 28-layer B8", cfg, params, d)
    torch.cuda.empty_cache()


def test_ltx2b_loss_curve_shared_prompt():
    """SURVEY 8(c)-5 at LTX-2B widths: 20 optimizer steps (2 blocks, LoRA r=16, B=8 with one
    shared prompt, lr 1e-4): train_step + FusedAdamW vs the oracle + torch AdamW in bf16 and
    fp32 from the same weights, with the same per-step (latents, t, noise) streams."""
    from ltx_amd.training import FusedAdamW
    from ltx_amd.transformer3d import OURS_TRANSFORMER_CONFIG
    cfg = dict(OURS_TRANSFORMER_CONFIG, num_layers=2)
    params = O.make_params(cfg, 37, lora_rank=16, requires_grad=False)
    model = build_model(cfg, params, 16, device=DEV)
    model.train()
    opt = FusedAdamW([p for p in model.parameters() if p.requires_grad], lr=1e-4)
    refs = {}
    for dt in (torch.bfloat16, torch.float32):
        q = {k: v.detach().to(DEV).to(torch.float32 if ("lora_" in k or dt == torch.float32) else dt)
             .requires_grad_(("lora_" in k) or ("caption_projection" in k)) for k, v in params.items()}
        refs[dt] = (q, torch.optim.AdamW([v for v in q.values() if v.requires_grad], lr=1e-4, foreach=False))
    curves = {"build": [], torch.bfloat16: [], torch.float32: []}
    for step in range(20):
        d = _inputs(8, 7, 16, 16, 256, 16, seed=1000 + step)
        curves["build"].append(_build_step(model, d))
        opt.step()
        opt.zero_grad(set_to_none=True)
        for dt, (q, ropt) in refs.items():
            r = O.train_step(q, cfg, d["in.latents"], d["in.ref_image_latents"], d["in.pose_latents"],
                             d["in.prompt_embeds"], d["in.prompt_attention_mask"], t=d["out.t"],
                             noise=d["out.noise"].to(dt))
            r["loss"].backward()
            ropt.step()
            ropt.zero_grad(set_to_none=True)
            curves[dt].append(float(((r["sample"].float() - r["v_target"].float()) ** 2).mean()))
    for i in range(20):
        _loss_crit(f"step {i}", curves["build"][i], curves[torch.bfloat16][i], curves[torch.float32][i])


@pytest.mark.timeout(900)
def test_ltx2b_28_layers_loss_curve_50_steps():
    """SURVEY 8(c)-5 at depth: K = 50 optimizer steps of the full 28-layer LTX-2B (LoRA r=16 on
    attn2, trainable caption projection, lr 1e-4) at B = 1, N = 1792 (7x16x16), one prompt of 256
    tokens (16 valid): train_step + FusedAdamW (training.py:159-166, 199-207, 270-271) against the
    oracle + torch AdamW in fp32 and in bf16 on the GPU from the same weights and the same per-step
    (latents, t, noise), and, every step, against the oracle's fp32 and bf16 forward AT THE BUILD'S
    OWN CURRENT WEIGHTS (the build's adapters and caption projection copied in); the criterion is
    explained at the assertions. Progress goes to gpurun_out/ (one line a step)."""
    import os
    from params import canonical_name
    from ltx_amd.training import FusedAdamW
    from ltx_amd.transformer3d import OURS_TRANSFORMER_CONFIG
    cfg = dict(OURS_TRANSFORMER_CONFIG)  # 28 layers
    assert cfg["num_layers"] == 28
    params = O.make_params(cfg, 41, lora_rank=16, requires_grad=False)
    model = build_model(cfg, params, 16, device=DEV)
    model.train()
    opt = FusedAdamW([p for p in model.parameters() if p.requires_grad], lr=1e-4)
    trainable = lambda k: ("lora_" in k) or ("caption_projection" in k)  # noqa: E731
    refs = {}
    for dt in (torch.bfloat16, torch.float32):
        q = {k: v.detach().to(DEV).to(torch.float32 if ("lora_" in k or dt == torch.float32) else dt)
             .requires_grad_(trainable(k)) for k, v in params.items()}
        refs[dt] = (q, torch.optim.AdamW([v for v in q.values() if v.requires_grad], lr=1e-4, foreach=False))
    del params
    # the oracle at the build's weights: the frozen tensors shared with the reference runs, the
    # trainable ones overwritten from the build before every step
    at = {dt: {k: (v.detach().clone() if trainable(k) else v.detach()) for k, v in refs[dt][0].items()}
          for dt in refs}
    build_names = [(n, canonical_name(n)) for n, p in model.named_parameters() if p.requires_grad]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
    log = open(os.path.join(root, "gpurun_out", "loss_curve_28l_progress.txt"), "w")
    curves = {"build": [], torch.bfloat16: [], torch.float32: [], "at16": [], "at32": []}

    def oracle_loss(q, d, dt):
        r = O.train_step(q, cfg, d["in.latents"], d["in.ref_image_latents"], d["in.pose_latents"],
                         d["in.prompt_embeds"], d["in.prompt_attention_mask"], t=d["out.t"],
                         noise=d["out.noise"].to(dt))
        return r, float(((r["sample"].float() - r["v_target"].float()) ** 2).mean())
    for step in range(50):
        d = _inputs(1, 7, 16, 16, 256, 16, seed=5000 + step)
        with torch.no_grad():
            params_now = dict(model.named_parameters())
            for n, cn in build_names:
                for dt in at:
                    at[dt][cn].copy_(params_now[n].detach())
            for dt, key in ((torch.bfloat16, "at16"), (torch.float32, "at32")):
                curves[key].append(oracle_loss(at[dt], d, dt)[1])
        curves["build"].append(_build_step(model, d))
        opt.step()
        opt.zero_grad(set_to_none=True)
        for dt, (q, ropt) in refs.items():
            r, l32 = oracle_loss(q, d, dt)
            r["loss"].backward()
            ropt.step()
            ropt.zero_grad(set_to_none=True)
            curves[dt].append(l32)
            del r
        b_, h_, f_ = curves["build"][-1], curves["at16"][-1], curves["at32"][-1]
        margin = abs(b_ - f_) / abs(f_) - 1.25 * abs(h_ - f_) / abs(f_)
        log.write(f"step {step}: build {b_:.6f} | oracle trajectories bf16 "
                  f"{curves[torch.bfloat16][-1]:.6f} fp32 {curves[torch.float32][-1]:.6f} | oracle at the "
                  f"build's weights bf16 {h_:.6f} fp32 {f_:.6f} | margin {margin:+.3e}\n")
        log.flush()
    log.close()
    # Over 50 optimizer steps the bf16 and fp32 trajectories drift apart (~2 % by step 33) and cross,
    # so a step where the oracle's own bf16 curve happens to sit on the fp32 one says nothing about
    # the build's accuracy (r04: one such crossing, step 19). The criterion is therefore
    # (a) the noise criterion over the curve: RMS over steps of the build's relative distance to the
    #     fp32 trajectory <= 1.25 x the oracle-bf16 trajectory's + 1e-4, and
    # (b) per step, the noise criterion at a fixed point: the build's loss against the oracle's fp32
    #     loss AT THE BUILD'S OWN WEIGHTS and inputs, within 1.25 x the oracle's bf16 distance from
    #     it at those same weights, + 2e-4 relative (SURVEY 8(c)-4 on one forward; the trajectory
    #     divergence drops out, since all three evaluate the same weights);
    # (c) the same fixed-point distances pooled over the 50 steps (VERDICT r05 #5b): the build's mean
    #     and RMS distance to the fp32 loss at its weights within 1.1 x the oracle-bf16's. A
    #     per-step margin err - 1.25 ref <= 1e-4 is logged but cannot be the bar: ref is ONE draw of
    #     the reference's rounding noise per step (it lands within 7.4e-6 of fp32 at one step), and
    #     with the roles swapped the oracle's own bf16 loss misses that bar against the build at 6
    #     of r05's 50 steps, the build against the oracle at 4 (r05: build mean 2.49e-4 / RMS
    #     3.21e-4 vs reference 2.66e-4 / 3.38e-4; worst per-step margin +1.27e-4, the reference's
    #     against the build +2.9e-4). A systematic
    #     gradient error moves every step's distance, so it shows in the pooled figures first;
    # (d) per step, the build's trajectory within 2e-3 relative of the oracle-bf16 trajectory
    #     (step-level drift of the gradients stays pinned; r05's worst 8.3e-4).
    l32 = curves[torch.float32]
    e_b = [abs(b - f) / abs(f) for b, f in zip(curves["build"], l32)]
    e_r = [abs(h - f) / abs(f) for h, f in zip(curves[torch.bfloat16], l32)]
    rms = lambda v: (sum(x * x for x in v) / len(v)) ** 0.5  # noqa: E731
    mean = lambda v: sum(v) / len(v)  # noqa: E731
    assert rms(e_b) <= 1.25 * rms(e_r) + 1e-4, (rms(e_b), rms(e_r))
    fb, fr = [], []
    for i, (b, h, f) in enumerate(zip(curves["build"], curves["at16"], curves["at32"])):
        eb, er = abs(b - f) / abs(f), abs(h - f) / abs(f)
        fb.append(eb)
        fr.append(er)
        assert eb <= 1.25 * er + 2e-4, f"28-layer step {i}: build {b}, oracle at its weights bf16 {h} fp32 {f}"
    assert mean(fb) <= 1.1 * mean(fr), f"pooled fixed-point distance: build {mean(fb):.3e} vs bf16 {mean(fr):.3e}"
    assert rms(fb) <= 1.1 * rms(fr), f"pooled fixed-point RMS: build {rms(fb):.3e} vs bf16 {rms(fr):.3e}"
    for i, (b, h) in enumerate(zip(curves["build"], curves[torch.bfloat16])):
        assert abs(b - h) <= 2e-3 * abs(h), f"28-layer step {i}: build {b} vs oracle-bf16 trajectory {h}"


def test_text_stack_matches_per_block():
    """The batched text side (_TextStack: all blocks' text K/V as one grouped-extension GEMM, the
    2n adapters' lora_down / lora_wgrad as grouped launches, one encoder-gradient GEMM over
    K = n*2D) against the per-block path (LTX_TEXT_BATCH=0) on the config-A path at LTX-2B widths
    (3 blocks, B = 8, shared prompt): the LoRA products are the same kernels on the same operands,
    so to_k / to_v adapter grads of the LAST block (whose dK/dV do not depend on the encoder
    gradient) agree to rounding; every other output within bf16 noise of each other."""
    from ltx_amd import transformer3d as T
    cfg = dict(T.OURS_TRANSFORMER_CONFIG, num_layers=3)
    params = O.make_params(cfg, 41, lora_rank=16, requires_grad=False)
    d = _inputs(8, 7, 16, 16, 256, 16, seed=13)
    res = {}
    saved = T._TEXT_BATCH
    try:
        for batched in (False, True):
            T._TEXT_BATCH = batched
            model = build_model(cfg, params, 16, device=DEV)
            assert model._text_batchable() == batched
            loss = _build_step(model, d)
            res[batched] = (loss, grads_by_canonical(model))
    finally:
        T._TEXT_BATCH = saved
    (l0, g0), (l1, g1) = res[False], res[True]
    assert abs(l0 - l1) <= 1e-4 * abs(l0), (l0, l1)
    assert set(g0) == set(g1)
    for name in g0:
        e = rel(g1[name].float(), g0[name].float())
        assert e <= 1e-2, f"{name}: batched vs per-block {e:.3e}"


def test_text_stack_grouped_knorm():
    """The batched text side's attn2 k_norm as ONE grouped launch for every block, forward and
    backward (LTX_TEXT_KNORM_GROUPED, ltx_qk_norm_{fwd,bwd}_grouped), and the query-batch sums of
    the text-key gradients as one launch (LTX_TEXT_BSUM_GROUPED), against one launch per block:
    the same kernels per row, so the loss is bitwise and the grads agree to the run-to-run order of
    the adapter-gradient atomics."""
    from ltx_amd import transformer3d as T
    cfg = dict(T.OURS_TRANSFORMER_CONFIG, num_layers=3)
    params = O.make_params(cfg, 43, lora_rank=16, requires_grad=False)
    d = _inputs(8, 7, 16, 16, 256, 16, seed=17)
    res = {}
    saved = T._TEXT_KNORM_GROUPED, T._TEXT_BSUM_GROUPED
    try:
        # per block; grouped k_norm with per-block batch sums; grouped k_norm + grouped batch sums
        for mode, (kn, bs) in {"block": (False, False), "knorm": (True, False), "both": (True, True)}.items():
            T._TEXT_KNORM_GROUPED, T._TEXT_BSUM_GROUPED = kn, bs
            model = build_model(cfg, params, 16, device=DEV)
            assert model._text_batchable()
            loss = _build_step(model, d)
            res[mode] = (loss, grads_by_canonical(model))
    finally:
        T._TEXT_KNORM_GROUPED, T._TEXT_BSUM_GROUPED = saved
    l0, g0 = res["block"]
    for mode in ("knorm", "both"):
        l1, g1 = res[mode]
        assert l0 == l1, (mode, l0, l1)
        assert set(g0) == set(g1)
        for name in g0:
            e = rel(g1[name].float(), g0[name].float())
            assert e <= 1e-5, f"{mode} {name}: grouped vs per-block {e:.3e}"


def test_frozen_caption_projection_keeps_text_adapter_grads():
    """LoRA on attn2 with caption_projection FROZEN: enc2 then carries no grad, so the
    batched text side -- whose backward runs as enc2's -- must not be used; the per-block path
    computes every to_k / to_v adapter gradient. They must equal (to rounding) the grads of the
    same step with a trainable caption projection (batched text side), and match the oracle."""
    from ltx_amd.transformer3d import OURS_TRANSFORMER_CONFIG
    from model_utils import oracle_step
    cfg = dict(OURS_TRANSFORMER_CONFIG, num_layers=2)
    params = O.make_params(cfg, 53, lora_rank=16, requires_grad=False)
    d = _inputs(8, 7, 16, 16, 256, 16, seed=19)
    res = {}
    for frozen in (False, True):
        model = build_model(cfg, params, 16, device=DEV)
        if frozen:
            for p in model.caption_projection.parameters():
                p.requires_grad_(False)
        _build_step(model, d)
        res[frozen] = grads_by_canonical(model)
    g_tr, g_fr = res[False], res[True]
    lora_names = [n for n in g_tr if "lora_" in n]
    assert sorted(n for n in g_fr) == sorted(lora_names)
    for n in lora_names:
        assert g_fr[n] is not None and float(g_fr[n].abs().max()) > 0, n
        assert rel(g_fr[n].float(), g_tr[n].float()) <= 1e-2, n
    _, g32, _ = oracle_step(params, cfg, d, torch.float32, lambda k: "lora_" in k)
    _, g16, _ = oracle_step(params, cfg, d, torch.bfloat16, lambda k: "lora_" in k)
    for n in lora_names:
        _crit(f"frozen-caption {n}", g_fr[n], g16[n], g32[n], slack=5e-3)


def test_four_blocks_config_x_grads():
    """Config X gradients over depth: 4 LTX-2B blocks at latent 13x24x24 (N = 7488), B = 1,
    256 text tokens (16 valid): out.sample, loss and every LoRA / caption-projection gradient."""
    from ltx_amd.transformer3d import OURS_TRANSFORMER_CONFIG
    cfg = dict(OURS_TRANSFORMER_CONFIG, num_layers=4)
    params = O.make_params(cfg, 59, lora_rank=16, requires_grad=False)
    d = _inputs(1, 13, 24, 24, 256, 16, seed=23)
    _compare_model("X 4-block", cfg, params, d)
