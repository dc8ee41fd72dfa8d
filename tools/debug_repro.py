"""Find the first non-reproducible quantity of the build's train step: two identical models, the
same inputs, per-step grads / weights compared (names + max |diff|)."""
import os
import sys

import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(R, "video-generation-for-human-avatars_amd"), os.path.join(R, "oracle"),
          os.path.join(R, "tests")):
    sys.path.insert(0, p)
import ltx_oracle as O  # noqa: E402
from model_utils import build_model, build_step, synth_inputs  # noqa: E402
from ltx_amd.training import FusedAdamW  # noqa: E402
from ltx_amd.transformer3d import OURS_TRANSFORMER_CONFIG  # noqa: E402

layers, B = int(sys.argv[1]), int(sys.argv[2])
cfg = dict(OURS_TRANSFORMER_CONFIG, num_layers=layers)
params = O.make_params(cfg, 43, lora_rank=16, requires_grad=False)
runs, keep = [], []
for run in range(2):
    model = build_model(cfg, params, 16, device="cuda")
    model.train()
    opt = FusedAdamW([p for p in model.parameters() if p.requires_grad], lr=1e-4)
    rec = []
    for step in range(2):
        d = synth_inputs(B, 7, 16, 16, 256, 16, seed=7000 + step)
        loss = build_step(model, d)
        g = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.requires_grad}
        opt.step()
        opt.zero_grad(set_to_none=True)
        w = {n: p.detach().clone() for n, p in model.named_parameters() if p.requires_grad}
        rec.append((loss, g, w))
    runs.append(rec)
    keep.append((model, opt))
    junk = torch.empty(1 << 30, dtype=torch.uint8, device="cuda").fill_(0xFF)
    del junk
for step in range(2):
    (l0, g0, w0), (l1, g1, w1) = runs[0][step], runs[1][step]
    print(f"step {step}: loss {l0} vs {l1}")
    bad = [(n, float((g0[n].float() - g1[n].float()).abs().max()), g0[n].dtype) for n in g0 if not torch.equal(g0[n], g1[n])]
    print(f"  grads differing: {len(bad)} of {len(g0)}")
    for b in bad[:40]:
        print("   ", b)
    badw = [n for n in w0 if not torch.equal(w0[n], w1[n])]
    print(f"  weights differing: {len(badw)}: {badw[:10]}")
