"""Host (Python) time per train step by function: cProfile over 4 steps of bench.py's config-A step
after warm-up (the device work is asynchronous; this is the enqueue side only)."""
import cProfile, os, pstats, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch
import bench
from ltx_amd import _lib
from ltx_amd.config import TrainConfig
from ltx_amd.scheduler import RectifiedFlowScheduler
from ltx_amd.training import FusedAdamW, GradAllReduce, train_step

dev = torch.device("cuda", 0)
_lib.ensure_device(dev)
model = bench.build_model(dev, mode="lora_audio")
batch, prompt, mask = bench.synthetic_batch(dev, 0)
cfg = TrainConfig(checkpoint_path="-", batch_size=bench.B_PER_GPU, learning_rate=1e-4, lora_rank=16,
                  lora_alpha=16, gradient_accumulation_steps=16, rf_log_normal_mu=-0.5, rf_log_normal_sigma=1.0)
sched = RectifiedFlowScheduler(num_train_timesteps=1000, shifting=None)
trainable = [p for p in model.parameters() if p.requires_grad]
red = GradAllReduce(trainable, order=model.grad_ready_order()).install(model)
red.zero_grad()
step = lambda: train_step(model, batch, sched, model.patchifier, cfg, prompt, mask, dev)
for _ in range(3):
    step()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(4):
    step()
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("cumulative").print_stats(45)
st.sort_stats("tottime").print_stats(25)
