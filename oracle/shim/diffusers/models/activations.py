"""diffusers 0.35.1 activations.py: GELU (Linear then F.gelu), GEGLU, ApproximateGELU."""
import torch.nn as nn
import torch.nn.functional as F


class GELU(nn.Module):
    def __init__(self, dim_in, dim_out, approximate="none", bias=True):
        super().__init__()
        self.proj = nn.Linear(dim_in, dim_out, bias=bias)
        self.approximate = approximate

    def gelu(self, gate):
        return F.gelu(gate, approximate=self.approximate)

    def forward(self, hidden_states):
        return self.gelu(self.proj(hidden_states))


class GEGLU(nn.Module):
    def __init__(self, dim_in, dim_out, bias=True):
        super().__init__()
        self.proj = nn.Linear(dim_in, dim_out * 2, bias=bias)

    def forward(self, hidden_states, *args, **kwargs):
        hidden_states, gate = self.proj(hidden_states).chunk(2, dim=-1)
        return hidden_states * F.gelu(gate)


class ApproximateGELU(nn.Module):
    def __init__(self, dim_in, dim_out, bias=True):
        super().__init__()
        self.proj = nn.Linear(dim_in, dim_out, bias=bias)

    def forward(self, x):
        x = self.proj(x)
        return x * (1.702 * x).sigmoid()
