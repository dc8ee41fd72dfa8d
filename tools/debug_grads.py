"""Debug helper: per-parameter gradient errors of the tiny model vs the reference golden."""
import os, sys, json
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "video-generation-for-human-avatars_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import torch
from safetensors.torch import load_file
from model_utils import build_model, grads_by_canonical, rel
import test_model_gpu as T

d, meta = T._load("tiny_train_step")
params = {k[2:]: v for k, v in d.items() if k.startswith("w.")}
model = build_model(meta["config"], params, meta["lora_rank"])
loss, _, _ = T._build_run(model, d, meta["config"])
g = grads_by_canonical(model)
for k, v in d.items():
    if k.startswith("grad."):
        n = k[5:]
        print(f"{n:70s} build {float(g[n].float().norm()):.4e} ref {float(v.float().norm()):.4e} rel {rel(g[n].float(), v.cuda().float()):.3e}")
