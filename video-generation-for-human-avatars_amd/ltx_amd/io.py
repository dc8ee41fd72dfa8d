"""On-disk formats around the training step.

* Precomputed latents: ``{stem}.pt`` = {"latents": Tensor[1,128,F,H,W]} in the encoder dir, the
  pose-frame latents ``{stem}.pt`` and the reference-image latent ``{stem}_ref.pt`` in the
  condition dir (ltx_video/dataset.py:5-97, written by save_vae_latents.py /
  save_condition_encoder_latents.py). LatentPairDataset / collate_latent_pairs keep the
  reference's names, pairing rule and output dict. Files load with torch.load(weights_only=True):
  nothing in a latent file is executed.
* LatentLoader: the DataLoader the MI355X step wants -- rank-strided shard of the dataset per DP
  rank (one process per GPU), pinned host batches and the H2D copy on a side stream one batch
  ahead, so the copy overlaps the previous step's kernels (the timed region of bench.py is
  HBM-resident; this is the data-path for real training).
* Checkpoints: single-file safetensors with metadata["config"] = JSON {"transformer": {...}}
  (+ "scheduler"), as ltx_video/utils/torch_utils.py:39-133 writes them and
  Transformer3DModel.from_pretrained / RectifiedFlowScheduler.from_pretrained read them.
  lora_audio checkpoints export the peft merge (W + (B @ A) * scaling, rounded to the base dtype,
  adapters dropped); full checkpoints save the state dict.
"""
import json
import os
from pathlib import Path
from typing import Dict, List, Optional

import torch
from torch.utils.data import Dataset


# ---------------------------------------------------------------------------------------------
# latents
# ---------------------------------------------------------------------------------------------
def load_latents_pt(path):
    """{"latents": Tensor} from a precomputed-latent .pt file (no code execution on load)."""
    data = torch.load(path, map_location="cpu", weights_only=True)
    return data["latents"]


def save_latents_pt(latents, path):
    torch.save({"latents": latents.detach().cpu()}, path)


def collate_latent_pairs(batch: List[Dict]):
    """dataset.py:5-44."""
    return {
        "latents": torch.stack([b["latents"] for b in batch], dim=0),
        "pose_latents": torch.stack([b["pose_latents"] for b in batch], dim=0),
        "ref_image_latents": torch.stack([b["ref_image_latents"] for b in batch], dim=0),
        "stem": [b["stem"] for b in batch],
    }


class LatentPairDataset(Dataset):
    """dataset.py:47-97: encoder latents {stem}.pt (not *_ref) paired with the condition dir's
    {stem}.pt (pose) and {stem}_ref.pt (reference image); stems sorted, unpaired ones skipped."""

    def __init__(self, condition_latents_dir: str, encoder_latents_dir: str):
        self.condition_dir = Path(condition_latents_dir)
        self.encoder_dir = Path(encoder_latents_dir)
        files = [f for f in sorted(self.encoder_dir.glob("*.pt")) if not f.stem.endswith("_ref")]
        self.items = [f.stem for f in files
                      if (self.condition_dir / f"{f.stem}.pt").exists()
                      and (self.condition_dir / f"{f.stem}_ref.pt").exists()]

    def __len__(self):
        return len(self.items)

    def __getitem__(self, idx):
        stem = self.items[idx]
        latents = load_latents_pt(self.encoder_dir / f"{stem}.pt").squeeze()
        pose = load_latents_pt(self.condition_dir / f"{stem}.pt").squeeze()
        ref = load_latents_pt(self.condition_dir / f"{stem}_ref.pt").squeeze()
        if ref.ndim == 3:
            ref = ref.unsqueeze(1)
        return {"latents": latents, "pose_latents": pose, "ref_image_latents": ref, "stem": stem}


class LatentLoader:
    """Rank-strided batches of a LatentPairDataset on `device`, prefetched one batch ahead:
    pinned host collate, then a non-blocking H2D copy on a side stream; the consumer's stream
    waits on it. drop_last like the reference's DataLoader (training.py:586-592 uses shuffle)."""

    def __init__(self, dataset, batch_size, device, rank=0, world_size=1, shuffle=True, seed=0,
                 drop_last=True, dtype=torch.bfloat16):
        self.ds, self.bs, self.device = dataset, batch_size, torch.device(device)
        self.rank, self.world, self.shuffle, self.seed = rank, world_size, shuffle, seed
        self.drop_last, self.dtype, self.epoch = drop_last, dtype, 0
        self.stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None

    def set_epoch(self, epoch):
        self.epoch = epoch

    def _indices(self):
        n = len(self.ds)
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            order = torch.randperm(n, generator=g).tolist()
        else:
            order = list(range(n))
        mine = order[self.rank::self.world]
        nb = len(mine) // self.bs if self.drop_last else -(-len(mine) // self.bs)
        return [mine[i * self.bs:(i + 1) * self.bs] for i in range(nb)]

    def __len__(self):
        return len(self._indices())

    def _host_batch(self, idx):
        b = collate_latent_pairs([self.ds[i] for i in idx])
        for k in ("latents", "pose_latents", "ref_image_latents"):
            t = b[k].to(self.dtype)
            b[k] = t.pin_memory() if self.stream is not None else t
        return b

    def _to_device(self, hb):
        if self.stream is None:
            return {k: (v.to(self.device) if torch.is_tensor(v) else v) for k, v in hb.items()}
        with torch.cuda.stream(self.stream):
            db = {k: (v.to(self.device, non_blocking=True) if torch.is_tensor(v) else v)
                  for k, v in hb.items()}
        return db

    def __iter__(self):
        batches = self._indices()
        nxt = self._to_device(self._host_batch(batches[0])) if batches else None
        for i in range(len(batches)):
            cur = nxt
            if self.stream is not None:
                torch.cuda.current_stream(self.device).wait_stream(self.stream)
                for v in cur.values():
                    if torch.is_tensor(v):
                        v.record_stream(torch.cuda.current_stream(self.device))
            if i + 1 < len(batches):
                nxt = self._to_device(self._host_batch(batches[i + 1]))
            yield cur


# ---------------------------------------------------------------------------------------------
# checkpoints
# ---------------------------------------------------------------------------------------------
def _config_dict(module):
    cfg = getattr(module, "config", None)
    if cfg is None:
        return None
    return {k: v for k, v in dict(cfg).items() if not str(k).startswith("_")}


def _string_meta(meta):
    return {str(k): (v if isinstance(v, str) else str(v)) for k, v in meta.items()}


def save_module_safetensors(module, target_path, metadata: Optional[dict] = None):
    """torch_utils.py:39-63: the state dict (CPU) + metadata with an embedded config."""
    from safetensors.torch import save_file
    state = {k: v.detach().cpu().contiguous() for k, v in module.state_dict().items()}
    meta = dict(metadata or {})
    if "config" not in meta:
        cfg = _config_dict(module)
        if cfg is not None:
            meta["config"] = json.dumps({"transformer": cfg})
    save_file(state, target_path, metadata=_string_meta(meta))


def export_merged_safetensors(model, target_path, metadata: Optional[dict] = None):
    """torch_utils.py:66-102: peft merge_and_unload of a copy -> safetensors; the model being
    trained is not modified. The merge runs on CPU f32 tensors (delta = (B @ A) * scaling, then
    the promoted add rounded to the base dtype)."""
    from safetensors.torch import save_file
    state = merged_state_dict_cpu(model)
    meta = dict(metadata or {})
    cfg = _config_dict(model)
    if cfg is not None:
        root = {"transformer": cfg}
        sch = meta.pop("scheduler", None)
        if sch is not None:
            root["scheduler"] = sch
        meta["config"] = json.dumps(root)
    save_file(state, target_path, metadata=_string_meta(meta))


@torch.no_grad()
def merged_state_dict_cpu(model):
    from .transformer3d import LoraLinear
    out, wrapped = {}, []
    for name, mod in model.named_modules():
        if isinstance(mod, LoraLinear):
            wrapped.append(name + ".")
            w = mod.base_layer.weight.detach().cpu()
            a = mod.lora_A["default"].weight.detach().cpu()
            b = mod.lora_B["default"].weight.detach().cpu()
            delta = (b @ a) * mod.scaling
            merged = w.clone()
            merged += delta
            out[name + ".weight"] = merged
            if mod.base_layer.bias is not None:
                out[name + ".bias"] = mod.base_layer.bias.detach().cpu().clone()
    for k, v in model.state_dict().items():
        if not any(k.startswith(p) for p in wrapped):
            out[k] = v.detach().cpu().contiguous()
    return out


def save_training_checkpoint(model, target_path, train_mode, metadata: Optional[dict] = None,
                             is_best=False):
    """torch_utils.py:105-133 (best_ prefix, merged export for lora_audio)."""
    if is_best:
        d, f = os.path.dirname(target_path), os.path.basename(target_path)
        if not f.startswith("best_"):
            f = f"best_{f}"
        target_path = os.path.join(d, f)
    if train_mode == "lora_audio":
        export_merged_safetensors(model, target_path, metadata)
    else:
        save_module_safetensors(model, target_path, metadata)
    return target_path
