"""RectifiedFlowScheduler, training side (ltx_video/schedulers/rf.py:179-426).

add_noise / build_velocity_target keep the reference signatures; on ROCm tensors both run in the
fused kernel ltx_rf_noise_velocity (f32 arithmetic, bf16 result -- the reference computes the
same f32 values and train_step casts them to the model dtype at training.py:143,146).
shift_timesteps implements the SD3 and SimpleDiffusion resolution shifts (rf.py:49-149);
anything else is the reference's silent no-op. The timestep shift math acts on [B] scalars and
stays in torch (host-side plumbing).
"""
import math
from typing import Optional

import torch

from . import ops


def simple_diffusion_resolution_dependent_timestep_shift(samples_shape, timesteps, n=32 * 32):
    if len(samples_shape) == 3:
        _, m, _ = samples_shape
    elif len(samples_shape) in (4, 5):
        m = math.prod(samples_shape[2:])
    else:
        raise ValueError("Samples must have shape (b, t, c), (b, c, h, w) or (b, c, f, h, w)")
    snr = (timesteps / (1 - timesteps)) ** 2
    shift_snr = torch.log(snr) + 2 * math.log(m / n)
    return torch.sigmoid(0.5 * shift_snr)


def time_shift(mu: float, sigma: float, t):
    return math.exp(mu) / (math.exp(mu) + (1 / t - 1) ** sigma)


def get_normal_shift(n_tokens, min_tokens=1024, max_tokens=4096, min_shift=0.95, max_shift=2.05):
    m = (max_shift - min_shift) / (max_tokens - min_tokens)
    b = min_shift - m * min_tokens
    return m * n_tokens + b


def strech_shifts_to_terminal(shifts, terminal=0.1):
    if shifts.numel() == 0:
        raise ValueError("The 'shifts' tensor must not be empty.")
    if terminal <= 0 or terminal >= 1:
        raise ValueError("The terminal value must be between 0 and 1 (exclusive).")
    one_minus_z = 1 - shifts
    scale_factor = one_minus_z[-1] / (1 - terminal)
    return 1 - (one_minus_z / scale_factor)


def sd3_resolution_dependent_timestep_shift(samples_shape, timesteps, target_shift_terminal=None):
    if len(samples_shape) == 3:
        _, m, _ = samples_shape
    elif len(samples_shape) in (4, 5):
        m = math.prod(samples_shape[2:])
    else:
        raise ValueError("Samples must have shape (b, t, c), (b, c, h, w) or (b, c, f, h, w)")
    shift = get_normal_shift(m)
    out = time_shift(shift, 1, timesteps)
    if target_shift_terminal is not None:
        out = strech_shifts_to_terminal(out, target_shift_terminal)
    return out


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

    def shift_timesteps(self, samples_shape, timesteps):
        if self.shifting == "SD3":
            return sd3_resolution_dependent_timestep_shift(samples_shape, timesteps,
                                                           self.target_shift_terminal)
        if self.shifting == "SimpleDiffusion":
            return simple_diffusion_resolution_dependent_timestep_shift(
                samples_shape, timesteps, self.base_resolution)
        return timesteps

    def noise_and_velocity(self, tokens, noise, timesteps):
        """Both RF quantities in one kernel pass: (x_t, v_target), bf16."""
        return ops.rf_noise_velocity(tokens, noise, timesteps.float())

    def add_noise(self, original_samples, noise, timesteps):
        return self.noise_and_velocity(original_samples, noise, timesteps)[0]

    def build_velocity_target(self, tokens, noise, t):
        return self.noise_and_velocity(tokens, noise, t)[1]

    def alpha(self, t):
        return 1 - t

    def sigma(self, t):
        return t
