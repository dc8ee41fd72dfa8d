"""train_mode='full' at LTX-2B widths on the MI355X (BASELINE config Z's workload: training.py:75-91
trainable set, ds_config_zero2.json:1-17 optimizer), against the pinned oracle:

  * a 2-block LTX-2B-width model at B = 8 with ONE prompt expanded over the batch (the bench's
    text_shared path) in train_mode='full': out.sample, the loss and EVERY trainable gradient --
    attn1 / attn2 weights, biases and q/k norm weights, every scale_shift_table, adaln_single,
    caption_projection, proj_out -- through the 2B-width weight-gradient path (token-axis
    transposes + NT GEMM + AccumulateGrad roundings, ops.wgrad_into);
  * 3 optimizer steps of it with Zero2AdamW (flat bf16 buffers, f32 master shard, clip 1.0) vs
    the oracle + clip_grad_norm_(1.0) + torch AdamW on an f32 master, in bf16 and in fp32.

Criterion: err(build_bf16, ref_fp32) <= 1.25 * err(ref_bf16, ref_fp32) + slack,
rel-Frobenius; losses within max(1e-3, 1.25 x the reference's own bf16 noise) of fp32.
"""
import pytest
import torch

import ltx_oracle as O
from model_utils import (build_full_model, build_step, grads_by_canonical, is_full_trainable,
                         loss_crit, noise_crit, oracle_step, synth_inputs)

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _cfg(layers=2):
    from ltx_amd.transformer3d import OURS_TRANSFORMER_CONFIG
    return dict(OURS_TRANSFORMER_CONFIG, num_layers=layers)


def _sample(model, d):
    B = d["in.latents"].shape[0]
    tok, coords = O.patchify(d["in.latents"].bfloat16())
    x = O.add_noise(tok, d["out.noise"], d["out.t"]).bfloat16()
    with torch.no_grad():
        return model(hidden_states=x, indices_grid=coords.to(DEV),
                     ref_image_hidden_states=d["in.ref_image_latents"].bfloat16(),
                     pose_hidden_states=d["in.pose_latents"].bfloat16(),
                     encoder_hidden_states=d["in.prompt_embeds"].bfloat16().expand(B, -1, -1),
                     timestep=d["out.t"],
                     encoder_attention_mask=d["in.prompt_attention_mask"].expand(B, -1)).sample


def test_full_mode_2b_two_blocks_b8_every_grad():
    cfg = _cfg(2)
    params = O.make_params(cfg, 43, lora_rank=0, requires_grad=False)
    d = synth_inputs(8, 7, 16, 16, 256, 16, seed=17)
    model = build_full_model(cfg, params)
    out = _sample(model, d)
    lb = build_step(model, d)
    g = grads_by_canonical(model)
    s32, g32, l32 = oracle_step(params, cfg, d, torch.float32, is_full_trainable)
    s16, g16, l16 = oracle_step(params, cfg, d, torch.bfloat16, is_full_trainable)
    assert sorted(g) == sorted(g32), "the full-mode trainable set (training.py:75-91)"
    # 2 blocks x (attn1 + attn2: 4 weights + 4 biases + 2 norm weights) + 2 tables + adaln_single (6)
    # + caption_projection (4) + proj_out (2) + the head's scale_shift_table
    assert len(g) == 2 * 21 + 6 + 4 + 2 + 1, len(g)
    noise_crit("Z sample", out, s16, s32)
    loss_crit("Z loss", lb, l16, l32)
    worst = []
    for name in sorted(g32):
        assert g[name] is not None, name
        e_b, e_r = noise_crit(f"Z {name}", g[name], g16[name], g32[name], slack=5e-3)
        worst.append((e_b - 1.25 * e_r, name))
    print("worst margins:", sorted(worst, reverse=True)[:4])


def test_full_mode_2b_zero2_three_steps():
    """3 steps of Zero2AdamW (world 1: the flat-buffer cast / sum-of-squares / clip / AdamW kernels)
    on the 2-block full-mode model vs oracle + clip_grad_norm_(1.0) + torch AdamW (f32 master of
    the bf16 weights, DeepSpeed bf16's arrangement), bf16 and fp32 trajectories."""
    from ltx_amd.zero import Zero2AdamW
    cfg = _cfg(2)
    params = O.make_params(cfg, 47, lora_rank=0, requires_grad=False)
    model = build_full_model(cfg, params)
    opt = Zero2AdamW([p for p in model.parameters() if p.requires_grad], lr=1e-4, gradient_clipping=1.0)
    refs = {}
    for dt in (torch.bfloat16, torch.float32):
        q = {k: v.detach().to(DEV).to(dt).requires_grad_(is_full_trainable(k)) for k, v in params.items()}
        qt = [v for v in q.values() if v.requires_grad]
        qm = [v.detach().float().clone().requires_grad_(True) for v in qt]
        refs[dt] = (q, qt, qm, torch.optim.AdamW(qm, lr=1e-4, foreach=False))
    for step in range(3):
        d = synth_inputs(8, 7, 16, 16, 256, 16, seed=2000 + step)
        lb = build_step(model, d)
        opt.step()
        opt.zero_grad()
        losses, norms = {}, {}
        for dt, (q, qt, qm, ropt) in refs.items():
            r = O.train_step(q, cfg, d["in.latents"], d["in.ref_image_latents"], d["in.pose_latents"],
                             d["in.prompt_embeds"], d["in.prompt_attention_mask"], t=d["out.t"],
                             noise=d["out.noise"].to(dt))
            r["loss"].backward()
            for v, m in zip(qt, qm):
                m.grad = v.grad.float()
                v.grad = None
            norms[dt] = float(torch.nn.utils.clip_grad_norm_(qm, 1.0))
            ropt.step()
            with torch.no_grad():
                for v, m in zip(qt, qm):
                    v.copy_(m.to(dt))
            losses[dt] = float(((r["sample"].float() - r["v_target"].float()) ** 2).mean())
        loss_crit(f"Z step {step}", lb, losses[torch.bfloat16], losses[torch.float32])
        # the global grad norm the clip used, against the references' (bf16 noise yardstick)
        n_b, n16, n32 = opt.grad_norm(), norms[torch.bfloat16], norms[torch.float32]
        assert abs(n_b - n32) <= max(1e-3 * n32, 1.25 * abs(n16 - n32) + 1e-4 * n32), (step, n_b, n16, n32)
    # weights after 3 steps: within the bf16 reference's distance of the fp32 trajectory
    from params import canonical_name
    mine = {canonical_name(n): p.detach() for n, p in model.named_parameters() if p.requires_grad}
    q16, q32 = refs[torch.bfloat16][0], refs[torch.float32][0]
    for name in mine:
        d0 = params[name].to(DEV).float()
        noise_crit(f"Z update {name}", mine[name].float() - d0, q16[name].detach().float() - d0,
                   q32[name].detach().float() - d0, factor=1.25, slack=2e-2)
