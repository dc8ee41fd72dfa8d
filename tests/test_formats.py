"""On-disk formats, CPU only:
  * checkpoints: our save_training_checkpoint of the tiny model equals, tensor for tensor, what
    the REFERENCE's torch_utils.py wrote for the same weights (tests/golden/ckpt_export.*, made
    by oracle/gen_golden.py through the diffusers/peft shim), in both train modes; the file
    round-trips through Transformer3DModel.from_pretrained;
  * precomputed latents: LatentPairDataset pairing / squeeze / ref-frame rules of
    ltx_video/dataset.py:47-97 on .pt files written here, and LatentLoader's rank sharding.
The shim's ConfigMixin keeps its config in a plain dict, so the reference file's
metadata["config"] reads '{"transformer": {}}'; with diffusers' FrozenDict it carries every
public config key -- which is what ours writes (checked to round-trip)."""
import json
import os

import pytest
import torch
from safetensors import safe_open
from safetensors.torch import load_file

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _golden():
    with open(os.path.join(GOLD, "ckpt_export.json")) as f:
        meta = json.load(f)
    return load_file(os.path.join(GOLD, "ckpt_export.safetensors")), meta


def _tiny_model_cpu(cfg, rank):
    """Our module tree on the CPU with the tiny golden weights (construction and export need no
    GPU; only forward/backward launch kernels)."""
    from ltx_amd.config import TrainConfig
    from ltx_amd.lora import apply_training_strategy
    from ltx_amd.transformer3d import Transformer3DModel
    from params import canonical_name
    d = load_file(os.path.join(GOLD, "tiny_train_step.safetensors"))
    params = {k[2:]: v for k, v in d.items() if k.startswith("w.")}
    with torch.device("meta"):
        m = Transformer3DModel.from_config(cfg)
        apply_training_strategy(m, TrainConfig(checkpoint_path="-", lora_rank=rank,
                                               lora_alpha=rank), "lora_audio")
    sd = {n: params[canonical_name(n)].clone() for n, _ in m.named_parameters()}
    m.load_state_dict(sd, assign=True, strict=True)
    return m


@pytest.mark.parametrize("mode", ["lora_audio", "full"])
def test_checkpoint_export_matches_reference(tmp_path, mode):
    from ltx_amd import io
    gold, meta = _golden()
    m = _tiny_model_cpu(meta["config"], meta["lora_rank"])
    path = str(tmp_path / "model_epoch_3.safetensors")
    if mode == "full":  # the reference saves a merged plain model's state dict
        from ltx_amd.lora import unload_lora
        m = unload_lora(m)
    out = io.save_training_checkpoint(m, path, mode, metadata={"epoch": "3", "source": "gen"},
                                      is_best=(mode == "full"))
    assert os.path.basename(out) == ("best_model_epoch_3.safetensors" if mode == "full"
                                     else "model_epoch_3.safetensors")
    with safe_open(out, framework="pt", device="cpu") as f:
        md = f.metadata()
        ours = {k: f.get_tensor(k) for k in f.keys()}
    ref = {k[len(mode) + 1:]: v for k, v in gold.items() if k.startswith(mode + ".")}
    assert set(ours) == set(ref)
    for k, v in ref.items():
        assert ours[k].dtype == v.dtype and torch.equal(ours[k], v), k
    ref_md = meta[f"{mode}.metadata"]
    assert {k: v for k, v in md.items() if k != "config"} == \
        {k: v for k, v in ref_md.items() if k != "config"}
    cfg = json.loads(md["config"])["transformer"]
    # every constructor argument (register_to_config records __init__ args only)
    for k in ("num_attention_heads", "attention_head_dim", "in_channels", "num_layers",
              "caption_channels", "cross_attention_dim", "qk_norm", "positional_embedding_theta",
              "positional_embedding_max_pos", "timestep_scale_multiplier", "norm_eps"):
        assert cfg[k] == meta["config"][k], k


def test_checkpoint_round_trips_through_from_pretrained(tmp_path):
    from ltx_amd import io
    from ltx_amd.transformer3d import Transformer3DModel
    gold, meta = _golden()
    m = _tiny_model_cpu(meta["config"], meta["lora_rank"])
    path = io.save_training_checkpoint(m, str(tmp_path / "m.safetensors"), "lora_audio",
                                       metadata={"scheduler": {"sampler": "LinearQuadratic"}})
    loaded = Transformer3DModel.from_pretrained(path)
    sd = loaded.state_dict()
    for k, v in gold.items():
        if k.startswith("lora_audio."):
            assert torch.equal(sd[k[len("lora_audio."):]], v), k
    from ltx_amd.scheduler import RectifiedFlowScheduler
    sch = RectifiedFlowScheduler.from_pretrained(path)
    assert sch.sampler == "LinearQuadratic"


def test_latent_pair_dataset_rules(tmp_path):
    from ltx_amd import io
    enc, cond = tmp_path / "enc", tmp_path / "cond"
    enc.mkdir()
    cond.mkdir()
    g = torch.Generator().manual_seed(0)
    stems = ["b_clip", "a_clip", "c_noref"]
    for s in stems:
        io.save_latents_pt(torch.randn(1, 8, 3, 4, 4, generator=g), enc / f"{s}.pt")
        io.save_latents_pt(torch.randn(1, 8, 3, 4, 4, generator=g), cond / f"{s}.pt")
    io.save_latents_pt(torch.randn(1, 8, 1, 4, 4, generator=g), cond / "a_clip_ref.pt")
    io.save_latents_pt(torch.randn(8, 4, 4, generator=g), cond / "b_clip_ref.pt")  # no frame dim
    io.save_latents_pt(torch.randn(1, 8, 1, 4, 4, generator=g), enc / "a_clip_ref.pt")  # ignored
    ds = io.LatentPairDataset(str(cond), str(enc))
    assert ds.items == ["a_clip", "b_clip"]  # sorted, unpaired c_noref dropped, *_ref skipped
    item = ds[1]
    assert item["latents"].shape == (8, 3, 4, 4) and item["pose_latents"].shape == (8, 3, 4, 4)
    assert item["ref_image_latents"].shape == (8, 1, 4, 4)
    assert torch.equal(item["latents"], io.load_latents_pt(enc / "b_clip.pt").squeeze())
    b = io.collate_latent_pairs([ds[0], ds[1]])
    assert b["latents"].shape == (2, 8, 3, 4, 4) and b["stem"] == ["a_clip", "b_clip"]
    # rank-strided shards cover the dataset once
    seen = []
    for r in range(2):
        ld = io.LatentLoader(ds, 1, "cpu", rank=r, world_size=2, shuffle=True, seed=5)
        for bt in ld:
            seen += bt["stem"]
            assert bt["latents"].dtype == torch.bfloat16
    assert sorted(seen) == ["a_clip", "b_clip"]
