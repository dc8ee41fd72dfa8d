"""SymmetricPatchifier (ltx_video/models/transformers/symmetric_patchifier.py:10-84), patch 1.

patchify / unpatchify / get_latent_coords run as bit-exact HIP kernels (ltx_patchify_bf16,
ltx_unpatchify_bf16, ltx_latent_coords). Unlike the reference, whose einops views alias the
input, the outputs are fresh buffers (the reference's in-place aliasing is what makes
Transformer3DModel.forward mutate its input, transformer3d.py:447-466; this build does not).
"""
from . import ops


class SymmetricPatchifier:
    def __init__(self, patch_size: int = 1):
        if patch_size != 1:
            raise NotImplementedError("LTX-Video 2B uses patch_size 1 (the VAE patchifies)")
        self._patch_size = (1, patch_size, patch_size)

    @property
    def patch_size(self):
        return self._patch_size

    def get_latent_coords(self, latent_num_frames, latent_height, latent_width, batch_size, device):
        return ops.latent_coords(batch_size, latent_num_frames, latent_height, latent_width, device)

    def patchify(self, latents):
        b, _, f, h, w = latents.shape
        return ops.patchify(latents), self.get_latent_coords(f, h, w, b, latents.device)

    def unpatchify(self, latents, output_height, output_width, out_channels):
        b, n, c = latents.shape
        f = n // (output_height * output_width)
        return ops.unpatchify(latents, f, output_height, output_width)
