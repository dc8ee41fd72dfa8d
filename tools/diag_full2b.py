"""Diagnostic: full-mode 2-block LTX-2B-width grads, build (text_shared / materialised prompt) vs
oracle fp32 / bf16: per-tensor rel errors, sorted by margin over 1.25x the reference noise."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("video-generation-for-human-avatars_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))
import torch

import ltx_oracle as O
from model_utils import (build_full_model, build_step, grads_by_canonical, is_full_trainable,
                         oracle_step, rel, synth_inputs)
from ltx_amd.transformer3d import OURS_TRANSFORMER_CONFIG

cfg = dict(OURS_TRANSFORMER_CONFIG, num_layers=2)
params = O.make_params(cfg, 43, lora_rank=0, requires_grad=False)
d = synth_inputs(8, 7, 16, 16, 256, 16, seed=17)
_, g32, l32 = oracle_step(params, cfg, d, torch.float32, is_full_trainable)
_, g16, l16 = oracle_step(params, cfg, d, torch.bfloat16, is_full_trainable)
res = {}
for shared in (True, False):
    model = build_full_model(cfg, params)
    dd = dict(d)
    if not shared:  # a materialised copy per sample: the per-sample text path
        dd["in.prompt_embeds"] = d["in.prompt_embeds"].expand(8, -1, -1).contiguous()
        dd["in.prompt_attention_mask"] = d["in.prompt_attention_mask"].expand(8, -1).contiguous()
    lb = build_step(model, dd)
    res[shared] = (lb, grads_by_canonical(model))
    del model
print(f"loss build shared {res[True][0]:.6f} per-sample {res[False][0]:.6f} fp32 {l32:.6f} bf16 {l16:.6f}")
rows = []
for n in sorted(g32):
    er = rel(g16[n], g32[n])
    es = rel(res[True][1][n], g32[n])
    ep = rel(res[False][1][n], g32[n])
    rows.append((es - 1.25 * er, n, es, ep, er, float(g32[n].float().norm())))
rows.sort(reverse=True)
for m, n, es, ep, er, nrm in rows[:16]:
    print(f"{m:+.2e}  shared {es:.3e}  per-sample {ep:.3e}  ref-bf16 {er:.3e}  |g| {nrm:.3e}  {n}")
