"""RectifiedFlowScheduler (ltx_video/schedulers/rf.py:179-426): training side and the
inference step.

add_noise / build_velocity_target keep the reference signatures and its f32 results (kernel
ltx_rf_noise_velocity_f32); train_step's fused prologue (ltx_rf_prepare_tokens) computes the same
f32 values and rounds them to the model dtype once, where the reference casts at
training.py:143,146.
shift_timesteps implements the SD3 and SimpleDiffusion resolution shifts (rf.py:49-149);
anything else is the reference's silent no-op. The timestep shift math acts on [B] scalars and
stays in torch (host-side plumbing), as does the 20-entry schedule of set_timesteps.
step() is the Euler update over the latent tokens: the fused kernel ltx_rf_euler_step
(next-lower-timestep search + update, global or per-token timesteps).
"""
import json
import math
from dataclasses import dataclass
from pathlib import Path
from typing import Optional, Union

import torch

from . import ops


def _tokens_per_sample(samples_shape):
    """The token count m the resolution shifts key on (rf.py:50-57, 115-122): the sequence axis of
    a (b, t, c) token tensor, or the product of the spatial axes of a (b, c, h, w) /
    (b, c, f, h, w) latent."""
    rank = len(samples_shape)
    if rank == 3:
        return samples_shape[1]
    if rank in (4, 5):
        return math.prod(samples_shape[2:])
    raise ValueError("Samples must have shape (b, t, c), (b, c, h, w) or (b, c, f, h, w)")


def linear_quadratic_schedule(num_steps, threshold_noise=0.025, linear_steps=None):
    """rf.py:25-46. The noise level s(i) climbs linearly to `threshold_noise` over the first
    `linear_steps` steps, then along the quadratic a*i^2 + b*i + c that continues it and reaches 1
    at i = num_steps; the schedule is 1 - s(i) for i < num_steps (same double-precision
    expressions as the reference, so the f32 tensor is identical)."""
    if num_steps == 1:
        return torch.tensor([1.0])
    lin = num_steps // 2 if linear_steps is None else linear_steps
    quad = num_steps - lin
    gap = lin - threshold_noise * num_steps
    a = gap / (lin * quad ** 2)
    b = threshold_noise / lin - 2 * gap / (quad ** 2)
    c = a * (lin ** 2)
    levels = [i * threshold_noise / lin for i in range(lin)]
    levels += [a * (i ** 2) + b * i + c for i in range(lin, num_steps)]
    return torch.tensor([1.0 - s for s in levels])


def simple_diffusion_resolution_dependent_timestep_shift(samples_shape, timesteps, n=32 * 32):
    """rf.py:108-127: shift the log-SNR of t by 2 log(m / n), m = tokens per sample."""
    m = _tokens_per_sample(samples_shape)
    log_snr = torch.log((timesteps / (1 - timesteps)) ** 2)
    return torch.sigmoid(0.5 * (log_snr + 2 * math.log(m / n)))


def time_shift(mu: float, sigma: float, t):
    """rf.py:49-50: e^mu / (e^mu + (1/t - 1)^sigma)."""
    e = math.exp(mu)
    return e / (e + (1 / t - 1) ** sigma)


def get_normal_shift(n_tokens, min_tokens=1024, max_tokens=4096, min_shift=0.95, max_shift=2.05):
    """rf.py:53-62: the shift interpolated linearly in the token count through
    (min_tokens, min_shift) and (max_tokens, max_shift)."""
    slope = (max_shift - min_shift) / (max_tokens - min_tokens)
    return slope * n_tokens + (min_shift - slope * min_tokens)


def strech_shifts_to_terminal(shifts, terminal=0.1):
    """rf.py:65-92 (the reference's spelling): rescale 1 - shifts so that the last entry lands on
    `terminal`."""
    if shifts.numel() == 0:
        raise ValueError("The 'shifts' tensor must not be empty.")
    if not 0 < terminal < 1:
        raise ValueError("The terminal value must be between 0 and 1 (exclusive).")
    rest = 1 - shifts
    return 1 - rest / (rest[-1] / (1 - terminal))


def sd3_resolution_dependent_timestep_shift(samples_shape, timesteps, target_shift_terminal=None):
    """rf.py:95-105: time_shift by the token-count-dependent normal shift, optionally stretched
    to a terminal value."""
    out = time_shift(get_normal_shift(_tokens_per_sample(samples_shape)), 1, timesteps)
    return out if target_shift_terminal is None else strech_shifts_to_terminal(out, target_shift_terminal)


@dataclass
class RectifiedFlowSchedulerOutput:
    """rf.py:157-170."""
    prev_sample: torch.Tensor
    pred_original_sample: Optional[torch.Tensor] = None

    def __getitem__(self, i):
        return (self.prev_sample,)[i]


class RectifiedFlowScheduler:
    order = 1

    def __init__(self, num_train_timesteps=1000, shifting: Optional[str] = None,
                 base_resolution: int = 32 ** 2, target_shift_terminal: Optional[float] = None,
                 sampler: Optional[str] = "Uniform", shift: Optional[float] = None):
        self.num_train_timesteps = num_train_timesteps
        self.shifting = shifting
        self.base_resolution = base_resolution
        self.target_shift_terminal = target_shift_terminal
        self.sampler = sampler
        self.shift = shift
        self.init_noise_sigma = 1.0
        self.num_inference_steps = None
        self.config = {"num_train_timesteps": num_train_timesteps, "shifting": shifting,
                       "base_resolution": base_resolution,
                       "target_shift_terminal": target_shift_terminal, "sampler": sampler,
                       "shift": shift}
        self.timesteps = self.sigmas = self.get_initial_timesteps(num_train_timesteps, shift=shift)

    @classmethod
    def from_config(cls, config):
        keys = ("num_train_timesteps", "shifting", "base_resolution", "target_shift_terminal",
                "sampler", "shift")
        return cls(**{k: v for k, v in dict(config).items() if k in keys})

    @staticmethod
    def from_pretrained(pretrained_model_path: Union[str, Path]):
        """Single-file safetensors (metadata['config']['scheduler']) or a diffusers directory
        (scheduler/scheduler_config.json), rf.py:250-274."""
        path = Path(pretrained_model_path)
        if path.is_file():
            from safetensors import safe_open
            with safe_open(str(path), framework="pt", device="cpu") as f:
                config = json.loads(f.metadata()["config"])["scheduler"]
        else:
            with open(path / "scheduler" / "scheduler_config.json") as f:
                config = json.load(f)
        return RectifiedFlowScheduler.from_config(config)

    def get_initial_timesteps(self, num_timesteps: int, shift: Optional[float] = None):
        """rf.py:198-214."""
        if self.sampler == "Uniform":
            return torch.linspace(1, 1 / num_timesteps, num_timesteps)
        if self.sampler == "LinearQuadratic":
            return linear_quadratic_schedule(num_timesteps)
        if self.sampler == "Constant":
            assert shift is not None, "Shift must be provided for constant time shift sampler."
            return time_shift(shift, 1, torch.linspace(1, 1 / num_timesteps, num_timesteps))
        return None

    def set_timesteps(self, num_inference_steps=None, samples_shape=None, timesteps=None,
                      device=None):
        """rf.py:227-248."""
        if timesteps is not None and num_inference_steps is not None:
            raise ValueError("You cannot provide both `timesteps` and `num_inference_steps`.")
        if timesteps is None:
            num_inference_steps = min(self.num_train_timesteps, num_inference_steps)
            timesteps = self.get_initial_timesteps(num_inference_steps, shift=self.shift).to(device)
            timesteps = self.shift_timesteps(samples_shape, timesteps)
        else:
            timesteps = torch.Tensor(timesteps).to(device)
            num_inference_steps = len(timesteps)
        self.timesteps = timesteps
        self.num_inference_steps = num_inference_steps
        self.sigmas = self.timesteps

    def scale_model_input(self, sample, timestep=None):
        return sample

    def step(self, model_output, timestep, sample, return_dict=True, stochastic_sampling=False,
             generator=None, **kwargs):
        """rf.py:305-374 on the device: Euler from `timestep` (0-dim global or [B,N] per token)
        to the next lower scheduled timestep, in ltx_rf_euler_step. stochastic_sampling
        re-noises the x0 estimate to the next timestep (rf.py:359-365)."""
        if self.num_inference_steps is None:
            raise ValueError("Number of inference steps is 'None', you need to run "
                             "'set_timesteps' after creating the scheduler")
        if not torch.is_tensor(timestep):
            timestep = torch.tensor(float(timestep))
        if stochastic_sampling:
            return self._stochastic_step(model_output, timestep, sample, return_dict, generator)
        prev = ops.rf_euler_step(model_output, timestep, sample, self.timesteps)
        if not return_dict:
            return (prev,)
        return RectifiedFlowSchedulerOutput(prev_sample=prev)

    def _stochastic_step(self, model_output, timestep, sample, return_dict, generator):
        """x0 = sample - t * v; prev = add_noise(x0, randn, t - dt) (rf.py:359-365). The
        Euler kernel gives sample - dt * v with the same dt; x0 and the re-noising are
        rf_noise_velocity's f32 arithmetic."""
        dev = sample.device
        t = timestep.to(device=dev, dtype=torch.float32)
        zero = torch.zeros((), device=dev)
        # dt from the kernel on a unit prediction: sample' = 0 - dt * 1
        unit = torch.ones(sample.shape[:-1] + (1,), dtype=torch.float32, device=dev)
        dt = -ops.rf_euler_step(unit, t, torch.zeros_like(unit), self.timesteps)
        tt = t.reshape(t.shape + (1,)) if t.ndim else t
        x0 = sample - tt * model_output
        next_t = tt - dt if t.ndim else (t - dt.reshape(-1)[0] + zero)
        noise = torch.randn(sample.shape, generator=generator, device=dev, dtype=sample.dtype)
        prev = self.add_noise_f32(x0, noise, next_t)
        if not return_dict:
            return (prev,)
        return RectifiedFlowSchedulerOutput(prev_sample=prev)

    @staticmethod
    def add_noise_f32(x0, noise, t):
        """rf.py:376-386 in f32 (append_dims broadcasting)."""
        s = t.reshape(t.shape + (1,) * (x0.ndim - t.ndim)) if t.ndim else t
        return (1 - s) * x0 + s * noise

    def shift_timesteps(self, samples_shape, timesteps):
        if self.shifting == "SD3":
            return sd3_resolution_dependent_timestep_shift(samples_shape, timesteps,
                                                           self.target_shift_terminal)
        if self.shifting == "SimpleDiffusion":
            return simple_diffusion_resolution_dependent_timestep_shift(
                samples_shape, timesteps, self.base_resolution)
        return timesteps

    def noise_and_velocity(self, tokens, noise, timesteps):
        """Both RF quantities in one kernel pass, rounded to bf16 (what train_step casts them to,
        training.py:143,146): (x_t, v_target)."""
        return ops.rf_noise_velocity(tokens, noise, timesteps.float())

    def add_noise(self, original_samples, noise, timesteps):
        """rf.py:376-386: (1 - t) x0 + t eps with [B] timesteps, in the reference's result dtype
        (f32 for f32 timesteps: the f32 kernel form, no bf16 rounding)."""
        return ops.rf_noise_velocity_f32(original_samples, noise, timesteps, want_v=False)[0]

    def build_velocity_target(self, tokens, noise, t):
        """rf.py:400-426: alpha'(t) x0 + sigma'(t) eps = eps - x0, f32 like the reference."""
        return ops.rf_noise_velocity_f32(tokens, noise, t, want_x=False)[1]

    def alpha(self, t):
        return 1 - t

    def sigma(self, t):
        return t
