"""peft 0.17.1 LoRA restatement (test-only). get_peft_model wraps each target nn.Linear in a
LoraLinear whose parameters are named `<target>.base_layer.weight`,
`<target>.lora_A.default.weight`, `<target>.lora_B.default.weight`, exactly as peft names
them. autocast_adapter_dtype=True (peft default) keeps the adapters in fp32 on a bf16 base."""
import math

import torch
import torch.nn as nn


class LoraConfig:
    def __init__(self, r=8, lora_alpha=8, target_modules=None, lora_dropout=0.0, bias="none",
                 **kwargs):
        self.r = r
        self.lora_alpha = lora_alpha
        self.target_modules = list(target_modules or [])
        self.lora_dropout = lora_dropout
        self.bias = bias


class LoraLinear(nn.Module):
    def __init__(self, base_layer, r, lora_alpha):
        super().__init__()
        self.base_layer = base_layer
        self.r = r
        self.scaling = lora_alpha / r
        self.lora_A = nn.ModuleDict({"default": nn.Linear(base_layer.in_features, r, bias=False)})
        self.lora_B = nn.ModuleDict({"default": nn.Linear(r, base_layer.out_features, bias=False)})
        nn.init.kaiming_uniform_(self.lora_A["default"].weight, a=math.sqrt(5))
        nn.init.zeros_(self.lora_B["default"].weight)
        adapter_dtype = base_layer.weight.dtype
        if adapter_dtype in (torch.float16, torch.bfloat16):
            adapter_dtype = torch.float32  # autocast_adapter_dtype=True
        self.lora_A.to(device=base_layer.weight.device, dtype=adapter_dtype)
        self.lora_B.to(device=base_layer.weight.device, dtype=adapter_dtype)

    @property
    def in_features(self):
        return self.base_layer.in_features

    @property
    def out_features(self):
        return self.base_layer.out_features

    @property
    def weight(self):
        return self.base_layer.weight

    @property
    def bias(self):
        return self.base_layer.bias

    def forward(self, x, *args, **kwargs):
        result = self.base_layer(x, *args, **kwargs)
        result_dtype = result.dtype
        lora_A = self.lora_A["default"]
        lora_B = self.lora_B["default"]
        x = x.to(lora_A.weight.dtype)
        result = result + lora_B(lora_A(x)) * self.scaling
        return result.to(result_dtype)


class _BaseModel(nn.Module):
    def __init__(self, model):
        super().__init__()
        self.model = model

    def forward(self, *args, **kwargs):
        return self.model(*args, **kwargs)


class PeftModel(nn.Module):
    def __init__(self, model):
        super().__init__()
        self.base_model = _BaseModel(model)

    def forward(self, *args, **kwargs):
        return self.base_model.model(*args, **kwargs)

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            return getattr(self.base_model.model, name)

    @torch.no_grad()
    def merge_and_unload(self):
        """peft 0.17.1 LoraModel.merge_and_unload (safe_merge=False): per LoRA Linear,
        delta = (B @ A) * scaling in the adapter dtype (get_delta_weight), then
        base_layer.weight.data += delta (in-place, promoted add rounded to the base dtype);
        the wrapper is replaced by its base layer."""
        model = self.base_model.model
        for name, mod in list(model.named_modules()):
            if isinstance(mod, LoraLinear):
                wa = mod.lora_A["default"].weight
                wb = mod.lora_B["default"].weight
                delta = (wb @ wa) * mod.scaling
                mod.base_layer.weight.data += delta
                parent_name, _, child = name.rpartition(".")
                parent = model.get_submodule(parent_name)
                if child.isdigit():
                    parent[int(child)] = mod.base_layer
                else:
                    setattr(parent, child, mod.base_layer)
        return model


def get_peft_model(model, peft_config, **kwargs):
    for name in peft_config.target_modules:
        parent_name, _, child_name = name.rpartition(".")
        parent = model.get_submodule(parent_name)
        setattr(parent, child_name,
                LoraLinear(getattr(parent, child_name), peft_config.r, peft_config.lora_alpha))
    return PeftModel(model)
