"""TrainConfig + YAML loader with the reference's field names and parsing behaviour
(ltx_video/config.py:6-154), so configs/train-avatars.yaml drops in unchanged.

Kept quirks (documented, pinned by tests/golden/train_config.json):
  * `precision: "bf16"` stays the string 'bf16' (training.py:30 only reacts to 'bfloat16'); this
    build always computes in bf16 regardless, as BASELINE.json requires.
  * falsy values of rf_shift / rf_target_shift_terminal / rf_log_normal_mu / _sigma become None
    (config.py:125-141): a mu of 0 is read as "unset".
"""
from dataclasses import dataclass
from typing import Optional

import yaml


@dataclass
class TrainConfig:
    checkpoint_path: str
    condition_latents_dir: Optional[str] = None
    encoder_latents_dir: Optional[str] = None
    val_condition_latents_dir: Optional[str] = None
    val_encoder_latents_dir: Optional[str] = None
    videos: Optional[str] = None
    output_dir: Optional[str] = None
    batch_size: Optional[int] = None
    num_epochs: Optional[int] = None
    learning_rate: Optional[float] = None
    lora_rank: int = 8
    lora_alpha: int = 8
    precision: str = "bfloat16"
    gradient_checkpointing: bool = False
    gradient_accumulation_steps: int = 1
    use_deepspeed: bool = False
    deepspeed_config: Optional[str] = None
    local_rank: int = -1
    rf_num_train_timesteps: int = 1000
    rf_sampler: str = "Uniform"
    rf_shift: Optional[float] = None
    rf_shifting: Optional[str] = None
    rf_base_resolution: int = 32 * 32
    rf_target_shift_terminal: Optional[float] = None
    rf_log_normal_mu: Optional[float] = None
    rf_log_normal_sigma: Optional[float] = None
    rf_quantile_min: float = 0.005
    rf_quantile_max: float = 0.999
    wandb_project: str = "ltx-video-avatars"
    wandb_run_name: Optional[str] = None
    log_every_n_steps: int = 10
    save_every_n_epochs: int = 1
    decoder_train: bool = False
    transformer_loss_weight: float = 1.0
    decoder_loss_l1_weight: float = 0.1
    decoder_loss_lpips_weight: float = 0.0
    decoder_t_max: float = 0.1


_SAMPLERS = {"uniform": "Uniform", "linear-quadratic": "LinearQuadratic",
             "linearquadratic": "LinearQuadratic", "from_checkpoint": "Uniform"}


def _opt_float(block, key):
    v = block.get(key)
    return float(v) if v else None


def load_train_config_from_yaml(yaml_path: str) -> TrainConfig:
    with open(yaml_path, "r") as f:
        cfg = yaml.safe_load(f)
    checkpoint_path = cfg.get("checkpoint_path", None)
    if not checkpoint_path:
        raise ValueError("checkpoint_path is required in YAML for training.")
    sampler = cfg.get("sampler", None)
    rf_sampler = _SAMPLERS.get(sampler.lower(), "Uniform") if isinstance(sampler, str) else "Uniform"
    t = cfg.get("train", {}) or {}
    return TrainConfig(
        checkpoint_path=checkpoint_path,
        precision=cfg.get("precision", "bfloat16"),
        condition_latents_dir=t.get("condition_latents_dir"),
        encoder_latents_dir=t.get("encoder_latents_dir"),
        val_condition_latents_dir=t.get("val_condition_latents_dir"),
        val_encoder_latents_dir=t.get("val_encoder_latents_dir"),
        videos=t.get("videos"),
        output_dir=t.get("output_dir"),
        batch_size=int(t["batch_size"]) if "batch_size" in t else None,
        num_epochs=int(t["num_epochs"]) if "num_epochs" in t else None,
        learning_rate=float(t["learning_rate"]) if "learning_rate" in t else None,
        lora_rank=int(t.get("lora_rank", 8)),
        lora_alpha=int(t.get("lora_alpha", 8)),
        gradient_checkpointing=bool(t.get("gradient_checkpointing", False)),
        gradient_accumulation_steps=int(t.get("gradient_accumulation_steps", 1)),
        use_deepspeed=bool(t.get("use_deepspeed", False)),
        deepspeed_config=t.get("deepspeed_config"),
        local_rank=int(t.get("local_rank", -1)),
        rf_sampler=rf_sampler,
        rf_num_train_timesteps=int(t.get("rf_num_train_timesteps", 1000)),
        rf_shift=_opt_float(t, "rf_shift"),
        rf_shifting=t.get("rf_shifting"),
        rf_base_resolution=int(t.get("rf_base_resolution", 32 * 32)),
        rf_target_shift_terminal=_opt_float(t, "rf_target_shift_terminal"),
        rf_log_normal_mu=_opt_float(t, "rf_log_normal_mu"),
        rf_log_normal_sigma=_opt_float(t, "rf_log_normal_sigma"),
        rf_quantile_min=float(t.get("rf_quantile_min", 0.005)),
        rf_quantile_max=float(t.get("rf_quantile_max", 0.999)),
        wandb_project=t.get("wandb_project", "ltx-video-avatars"),
        wandb_run_name=t.get("wandb_run_name"),
        log_every_n_steps=int(t.get("log_every_n_steps", 10)),
        save_every_n_epochs=int(t.get("save_every_n_epochs", 1)),
        decoder_train=bool(t.get("decoder_train", False)),
        transformer_loss_weight=float(t.get("transformer_loss_weight", 1.0)),
        decoder_loss_l1_weight=float(t.get("decoder_loss_l1_weight", 0.1)),
        decoder_loss_lpips_weight=float(t.get("decoder_loss_lpips_weight", 0.0)),
        decoder_t_max=float(t.get("decoder_t_max", 0.1)),
    )
