"""Helpers shared by the model-level tests and smoke(): build the MI355X Transformer3DModel from a
flat parameter dict keyed by the reference's canonical names (golden vectors / oracle params)."""
import torch

from params import canonical_name


def build_model(cfg, params, lora_rank=16, device="cuda"):
    from ltx_amd.config import TrainConfig
    from ltx_amd.lora import apply_training_strategy
    from ltx_amd.transformer3d import Transformer3DModel
    from ltx_amd.patchifier import SymmetricPatchifier
    with torch.device("meta"):
        m = Transformer3DModel.from_config(cfg)
        if lora_rank:
            apply_training_strategy(m, TrainConfig(checkpoint_path="-", lora_rank=lora_rank,
                                                   lora_alpha=lora_rank), "lora_audio")
    sd = {}
    for name, _ in m.named_parameters():
        sd[name] = params[canonical_name(name)].detach().to(device).clone()
    m.load_state_dict(sd, assign=True, strict=True)
    for n, p in m.named_parameters():
        p.requires_grad_(("lora_" in n) or ("caption_projection" in n))
    m.patchifier = SymmetricPatchifier(1)
    return m


def grads_by_canonical(model):
    return {canonical_name(n): p.grad for n, p in model.named_parameters() if p.requires_grad}


def rel(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / (b.norm() + 1e-30))
