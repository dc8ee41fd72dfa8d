"""Which PyTorch (aten) kernels does one training micro-step launch besides libltxhip's, and from
where? torch.profiler over 3 steps (bench.py's model / batch, no optimizer step), aten ops with a
CUDA-side time, grouped by op + input shapes, with the Python frame that issued them."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))
import torch
import bench
from ltx_amd import _lib
from ltx_amd.config import TrainConfig
from ltx_amd.scheduler import RectifiedFlowScheduler
from ltx_amd.training import GradAllReduce, train_step

dev = torch.device("cuda", 0)
_lib.ensure_device(dev)
model = bench.build_model(dev, mode="lora_audio")
batch, prompt, mask = bench.synthetic_batch(dev, 0)
cfg = TrainConfig(checkpoint_path="-", batch_size=bench.B_PER_GPU, learning_rate=1e-4, lora_rank=16,
                  lora_alpha=16, gradient_accumulation_steps=16)
sched = RectifiedFlowScheduler(num_train_timesteps=1000, shifting=None)
trainable = [p for p in model.parameters() if p.requires_grad]
red = GradAllReduce(trainable, order=model.grad_ready_order()).install(model)
red.zero_grad()
for _ in range(2):
    train_step(model, batch, sched, model.patchifier, cfg, prompt, mask, dev)
torch.cuda.synchronize()
from torch.profiler import profile, ProfilerActivity
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    for _ in range(3):
        train_step(model, batch, sched, model.patchifier, cfg, prompt, mask, dev)
    torch.cuda.synchronize()
ev = prof.key_averages(group_by_stack_n=4)
rows = [e for e in ev if e.device_time_total > 0 and e.key.startswith("aten::")]
rows.sort(key=lambda e: -e.device_time_total)
for e in rows[:25]:
    print(f"{e.key:34s} calls/step {e.count / 3:6.1f}  device us/step {e.device_time_total / 3:8.1f}")
    for fr in (e.stack or [])[:4]:
        print("      ", fr)
