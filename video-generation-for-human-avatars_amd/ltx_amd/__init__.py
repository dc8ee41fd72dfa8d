"""MI355X-native LTX-Video 2B training step (hot path of lusinlu/Video-Generation-for-Human-Avatars).

Host-side mirror of the reference's call surface (Transformer3DModel, SymmetricPatchifier,
RectifiedFlowScheduler, TrainConfig, train_step) over the C-ABI kernel library libltxhip.so.
"""
__version__ = "0.1.0"
