"""apply_training_strategy (ltx_video/training.py:42-91) without the peft dependency.

'lora_audio': wraps transformer_blocks.{i}.attn2.{to_q,to_k,to_v,to_out.0} in LoraLinear (peft
0.17.1 parameter names and init: kaiming-uniform(a=sqrt(5)) A, zero B, f32 adapters on the bf16
base, scaling = alpha / r) and makes only `lora_*` and `caption_projection` trainable.
'full': the reference's substring rule (training.py:75-91); the fused block backward raises for
it until the wgrad path (next row) lands.
"""
import torch

from .transformer3d import LoraLinear


def lora_target_modules(num_blocks):
    out = []
    for i in range(num_blocks):
        out += [f"transformer_blocks.{i}.attn2.to_q", f"transformer_blocks.{i}.attn2.to_k",
                f"transformer_blocks.{i}.attn2.to_v", f"transformer_blocks.{i}.attn2.to_out.0"]
    return out


def inject_lora(model, targets, r, alpha):
    for name in targets:
        parent_name, _, child = name.rpartition(".")
        parent = model.get_submodule(parent_name)
        base = getattr(parent, child) if not child.isdigit() else parent[int(child)]
        if isinstance(base, LoraLinear):
            continue
        wrapped = LoraLinear(base, r, alpha)
        if child.isdigit():
            parent[int(child)] = wrapped
        else:
            setattr(parent, child, wrapped)
    return model


def apply_training_strategy(model, config, train_mode: str):
    if train_mode == "lora_audio":
        inject_lora(model, lora_target_modules(len(model.transformer_blocks)), config.lora_rank,
                    config.lora_alpha)
        for n, p in model.named_parameters():
            p.requires_grad = ("lora_" in n) or ("caption_projection" in n)
        return model
    for n, p in model.named_parameters():
        p.requires_grad = any(k in n for k in ("proj_out", "scale_shift_table", "adaln_single",
                                              "caption_projection", "attn", "attn2"))
    return model


def trainable_parameters(model):
    return [(n, p) for n, p in model.named_parameters() if p.requires_grad]


@torch.no_grad()
def merged_state_dict(model):
    """peft merge_and_unload(): W + s*B@A folded into each wrapped base weight, adapter keys
    dropped (what save_training_checkpoint exports, torch_utils.py:66-102)."""
    out = {}
    skip = set()
    for name, mod in model.named_modules():
        if isinstance(mod, LoraLinear):
            out[name + ".weight"] = mod.merged_weight()
            if mod.base_layer.bias is not None:
                out[name + ".bias"] = mod.base_layer.bias.detach().clone()
            skip.add(name + ".")
    for k, v in model.state_dict().items():
        if any(k.startswith(s) for s in skip):
            continue
        out[k] = v
    return out


@torch.no_grad()
def unload_lora(model):
    """peft merge_and_unload in place: base_layer.weight += (B @ A) * scaling (promoted add
    rounded to the base dtype), each LoraLinear replaced by its base nn.Linear."""
    for name, mod in list(model.named_modules()):
        if isinstance(mod, LoraLinear):
            a = mod.lora_A["default"].weight
            b = mod.lora_B["default"].weight
            mod.base_layer.weight.data += (b @ a) * mod.scaling
            parent_name, _, child = name.rpartition(".")
            parent = model.get_submodule(parent_name)
            if child.isdigit():
                parent[int(child)] = mod.base_layer
            else:
                setattr(parent, child, mod.base_layer)
    return model
