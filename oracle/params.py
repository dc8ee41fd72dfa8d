"""Deterministic parameter initialisation shared by the golden generator, the oracle and the
tests -- TEST INFRASTRUCTURE (see oracle/README.md).

Every tensor is drawn from its own CPU generator seeded by ``seed + crc32(name)`` so the values
do not depend on module construction order: the reference's module tree (with the test-only
peft shim) and the build's module tree produce bit-identical weights for the same names.

Rules (by parameter name):
  * 2-D ``*.weight``                  N(0,1) / sqrt(fan_in)
  * ``*norm*.weight`` (1-D, q/k norms) 1 + 0.1 N(0,1)
  * ``*.bias``                        0.1 N(0,1)
  * ``*scale_shift_table``            N(0,1) / sqrt(D)
  * ``*lora_A*``                      N(0,1) / sqrt(in_features)       (fp32)
  * ``*lora_B*``                      0.05 N(0,1)                        (fp32; peft would zero it,
                                                                          the goldens use non-zero B
                                                                          so dL/dA is exercised)
"""
import hashlib
import zlib

import torch


def _gen(seed: int, name: str) -> torch.Generator:
    g = torch.Generator(device="cpu")
    g.manual_seed((int(seed) + zlib.crc32(name.encode())) & 0x7FFFFFFFFFFFFFFF)
    return g


def init_value(name: str, shape, seed: int) -> torch.Tensor:
    g = _gen(seed, name)
    shape = tuple(shape)
    x = torch.randn(shape, generator=g, dtype=torch.float32)
    if "lora_A" in name:
        return x / (shape[1] ** 0.5)
    if "lora_B" in name:
        return 0.05 * x
    if name.endswith("scale_shift_table"):
        return x / (shape[-1] ** 0.5)
    if name.endswith(".bias"):
        return 0.1 * x
    if len(shape) == 1:  # RMSNorm weights (q_norm / k_norm)
        return 1.0 + 0.1 * x
    return x / (shape[1] ** 0.5)


def canonical_name(name: str) -> str:
    """peft wraps targets: '<t>.base_layer.weight' is the same tensor as '<t>.weight'."""
    return name.replace("base_model.model.", "").replace(".base_layer.", ".")


@torch.no_grad()
def init_module_(module: torch.nn.Module, seed: int, dtype=torch.bfloat16,
                 adapter_dtype=torch.float32) -> None:
    """Overwrite every parameter of ``module`` in place (names as module.named_parameters())."""
    for name, p in module.named_parameters():
        canon = canonical_name(name)
        v = init_value(canon, p.shape, seed)
        target = adapter_dtype if "lora_" in canon else dtype
        p.data = v.to(target)


def weights_sha256(module: torch.nn.Module) -> str:
    h = hashlib.sha256()
    named = [(canonical_name(n), p) for n, p in module.named_parameters()]
    for name, p in sorted(named, key=lambda kv: kv[0]):
        h.update(name.encode())
        h.update(p.detach().to(torch.float32).contiguous().numpy().tobytes())
    return h.hexdigest()
