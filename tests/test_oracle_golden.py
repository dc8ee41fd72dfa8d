"""Pin the CPU oracle (oracle/ltx_oracle.py) to golden vectors produced by the REFERENCE itself
(oracle/gen_golden.py imports /root/reference unmodified through the diffusers/peft shim).
CPU only; these tests are what makes the oracle trustworthy as the GPU parity checker."""
import json
import os

import pytest
import torch
from safetensors.torch import load_file

import ltx_oracle as O
from params import canonical_name

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    with open(os.path.join(GOLD, name + ".json")) as f:
        meta = json.load(f)
    return load_file(os.path.join(GOLD, name + ".safetensors")), meta


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


def test_patchify_bit_exact():
    d, _ = _load("patchify")
    for key in [k[len("tokens."):] for k in d if k.startswith("tokens.")]:
        b, c, f, h, w = map(int, key.split("x"))
        x = torch.arange(b * c * f * h * w, dtype=torch.float32).reshape(b, c, f, h, w)
        tok, coords = O.patchify(x)
        assert torch.equal(tok, d["tokens." + key])
        assert torch.equal(coords, d["coords." + key])
        assert torch.equal(O.unpatchify(tok, h, w, c), d["unpatch." + key])


def test_rf_scheduler_and_t_sampling():
    d, meta = _load("rf_sched")
    assert torch.equal(O.add_noise(d["x0"], d["eps"], d["t"]), d["x_t"])
    assert torch.equal(O.velocity_target(d["x0"], d["eps"], d["t"]), d["v"])
    torch.manual_seed(meta["tsample_seed"])
    t = O.sample_timesteps(8)
    assert torch.equal(t, d["tsample_t"])


def test_rope_tables():
    d, meta = _load("rope_2b")
    for kind in ("int", "float"):
        cos, sin = O.rope_freqs(d["grid_" + kind], meta["dim"], meta["theta"], meta["max_pos"],
                                torch.bfloat16)
        assert torch.equal(cos, d["cos_" + kind]), kind
        assert torch.equal(sin, d["sin_" + kind]), kind


def _params_from_golden(d):
    p = {}
    for k, v in d.items():
        if k.startswith("w."):
            name = k[2:]
            t = v.clone()
            if ("lora_" in name) or ("caption_projection" in name):
                t.requires_grad_(True)
            p[name] = t
    return p


def test_tiny_train_step_matches_reference():
    d, meta = _load("tiny_train_step")
    p = _params_from_golden(d)
    B = d["in.latents"].shape[0]
    torch.manual_seed(meta["train_seed"])
    r = O.train_step(p, meta["config"], d["in.latents"], d["in.ref_image_latents"],
                     d["in.pose_latents"], d["in.prompt_embeds"], d["in.prompt_attention_mask"])
    assert torch.equal(r["t"], d["out.t"])
    assert torch.equal(r["noise"], d["out.noise"])
    assert torch.equal(r["x_t"], d["out.hidden_states"])
    assert torch.equal(r["v_target"], d["out.v_target"])
    # same ops in the same dtypes on the same torch build -> expected bitwise; allow 1 bf16 ulp
    assert _rel(r["sample"], d["out.sample"]) < 2e-3
    assert abs(float(r["loss"]) - float(d["out.loss"])) <= 0.01 * abs(float(d["out.loss"]))
    r["loss"].backward()
    for k, v in d.items():
        if k.startswith("grad."):
            name = k[5:]
            assert _rel(p[name].grad, v) < 5e-3, name
    assert B == 2


def test_block2b_matches_reference():
    d, meta = _load("ltx2b_block")
    cfg = meta["config"]
    p = O.make_params(cfg, meta["param_seed"], lora_rank=meta["lora_rank"])
    torch.manual_seed(meta["train_seed"])
    r = O.train_step(p, cfg, d["in.latents"], d["in.ref_image_latents"], d["in.pose_latents"],
                     d["in.prompt_embeds"], d["in.prompt_attention_mask"])
    assert torch.equal(r["x_t"], d["out.hidden_states"])
    assert _rel(r["sample"], d["out.sample"]) < 2e-3
    r["loss"].backward()
    for k, v in d.items():
        if k.startswith("grad."):
            assert _rel(p[k[5:]].grad, v) < 5e-3, k
        elif k.startswith("gradsum0."):
            assert _rel(p[k[9:]].grad.float().sum(0), v) < 5e-3, k
        elif k.startswith("gradsum1."):
            assert _rel(p[k[9:]].grad.float().sum(1), v) < 5e-3, k


def test_param_init_is_pinned():
    """The 2B-width weights are re-drawn from a seed, not stored: pin the draw by SHA-256."""
    d, meta = _load("ltx2b_block")
    from params import weights_sha256

    class _Holder(torch.nn.Module):
        def __init__(self, params):
            super().__init__()
            for k, v in params.items():
                self.register_parameter(k.replace(".", "__"), torch.nn.Parameter(v.detach()))

    p = O.make_params(meta["config"], meta["param_seed"], lora_rank=meta["lora_rank"],
                      requires_grad=False)
    import hashlib
    h = hashlib.sha256()
    for name in sorted(p):
        h.update(canonical_name(name).encode())
        h.update(p[name].detach().to(torch.float32).contiguous().numpy().tobytes())
    assert h.hexdigest() == meta["weights_sha256"]


# ---- inference denoising step ---------------------------------------------
def _infer_inputs(d):
    return dict(indices_grid=d["in.indices_grid"], ref_image_hidden_states=d["in.ref"],
                pose_hidden_states=d["in.pose"], encoder_hidden_states=d["in.enc"],
                encoder_attention_mask=d["in.enc_mask"])


def test_infer_pixel_coords_match_reference():
    d, meta = _load("infer_step")
    _, lat = O.patchify(torch.zeros(1, 1, 2, 8, 8))
    pc = O.pixel_coords(lat, (8, 32, 32), causal_fix=True)
    assert torch.equal(pc, d["in.pixel_coords"])
    frac = O.fractional_coords(torch.cat([pc] * 3), meta["frame_rate"])
    assert torch.equal(frac, d["in.indices_grid"])


@pytest.mark.parametrize("case", ["global", "tok", "tok_AttentionSkip", "tok_AttentionValues",
                                  "tok_Residual", "tok_TransformerBlock"])
def test_infer_forward_matches_reference(case):
    d, meta = _load("infer_step")
    tiny, _ = _load("tiny_train_step")  # same config and parameter seed -> same weights
    p = {k[2:]: v for k, v in tiny.items() if k.startswith("w.")}
    ts = d["in.ts_global"] if case == "global" else d["in.ts_tok"]
    strat = case[4:] if case.startswith("tok_") else None
    with torch.no_grad():
        out = O.forward(p, meta["config"], d["in.tokens"], timestep=ts,
                        skip_layer_mask=d["in.skip_layer_mask"] if strat else None,
                        skip_layer_strategy=strat, **_infer_inputs(d))
    assert _rel(out, d["out." + case]) < 2e-3, case


@pytest.mark.parametrize("name", ["Uniform", "LinearQuadratic", "SD3"])
def test_infer_scheduler_matches_reference(name):
    d, _ = _load("infer_step")
    from ltx_amd.scheduler import RectifiedFlowScheduler
    kw = {"Uniform": {}, "LinearQuadratic": {"sampler": "LinearQuadratic"},
          "SD3": {"shifting": "SD3", "target_shift_terminal": 0.1}}[name]
    sch = RectifiedFlowScheduler(**kw)
    sch.set_timesteps(num_inference_steps=20, samples_shape=torch.Size([2, 128, 7, 16, 16]))
    ts = d[f"sched.{name}.timesteps"]
    assert torch.allclose(sch.timesteps, ts, rtol=0, atol=1e-7)
    s, v = d["sched.sample"], d["sched.v"]
    assert torch.equal(O.rf_step(v, ts[3], s, ts), d[f"sched.{name}.prev_global"])
    assert torch.equal(O.rf_step(v.to(torch.bfloat16), ts[3], s, ts),
                       d[f"sched.{name}.prev_global_bf16v"])
    assert torch.equal(O.rf_step(v, d[f"sched.{name}.t_tok"], s, ts), d[f"sched.{name}.prev_tok"])


@pytest.mark.parametrize("sampler", ["LinearQuadratic", "Uniform"])
def test_reference_scheduler_cases(sampler):
    """The reference's own tests/test_scheduler.py cases, restated against the oracle step."""
    from ltx_amd.scheduler import RectifiedFlowScheduler
    sch = RectifiedFlowScheduler(sampler=sampler)
    g = torch.Generator().manual_seed(0)
    lat = torch.randn(2, 4096, 128, generator=g)
    sch.set_timesteps(num_inference_steps=20, samples_shape=lat.shape)
    ts = sch.timesteps
    for i, t in enumerate(ts):
        v = torch.randn(lat.shape, generator=g)
        nt = ts[i + 1] if i < len(ts) - 1 else 0.0
        assert torch.allclose(O.rf_step(v, t, lat, ts), lat - (t - nt) * v, atol=1e-6)
        tt = torch.full(lat.shape[:2], float(t))
        tt[:, 0] = 0.0
        out = O.rf_step(v, tt, lat, ts)
        assert torch.allclose(out[:, 1:], (lat - (t - nt) * v)[:, 1:], atol=1e-6)
        assert torch.allclose(out[:, 0], lat[:, 0], atol=1e-6)
        tm = (ts[i] + ts[i + 1]) / 2 if i < len(ts) - 1 else ts[i] / 2
        out = O.rf_step(v, torch.full(lat.shape[:2], float(tm)), lat, ts)
        assert torch.allclose(out, lat - (tm - nt) * v, atol=1e-6)


# ---- train_mode='full'  ------------------------------------------------
FULL_KEYS = ("proj_out", "scale_shift_table", "adaln_single", "caption_projection", "attn")


def test_full_mode_step_matches_reference():
    d, meta = _load("tiny_full_step")
    cfg = meta["config"]
    p = O.make_params(cfg, meta["param_seed"], lora_rank=0, requires_grad=False)
    for k, v in p.items():
        v.requires_grad_(any(s in k for s in FULL_KEYS))
    assert sorted(k for k, v in p.items() if v.requires_grad) == meta["trainable"]
    torch.manual_seed(meta["train_seed"])
    r = O.train_step(p, cfg, d["in.latents"], d["in.ref_image_latents"], d["in.pose_latents"],
                     d["in.prompt_embeds"], d["in.prompt_attention_mask"])
    assert torch.equal(r["x_t"], d["out.hidden_states"])
    assert _rel(r["sample"], d["out.sample"]) < 2e-3
    r["loss"].backward()
    for k, v in d.items():
        if k.startswith("grad."):
            assert _rel(p[k[5:]].grad, v) < 5e-3, k
