import torch


class ModelMixin(torch.nn.Module):
    """dtype/device as diffusers reports them: first floating parameter."""

    @property
    def dtype(self):
        for p in self.parameters():
            if p.is_floating_point():
                return p.dtype
        return torch.float32

    @property
    def device(self):
        return next(self.parameters()).device
