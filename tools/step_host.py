"""Host-side enqueue time per train step vs the synchronized step time (is the step CPU-bound?).
Reuses bench.py's model / batch construction; prints enqueue ms (no sync), step ms (sync) and
the GPU-idle estimate."""
import os, sys, time
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
                  lora_alpha=16, gradient_accumulation_steps=1)
sched = RectifiedFlowScheduler(num_train_timesteps=1000, shifting=None)
trainable = [p for p in model.parameters() if p.requires_grad]
opt = FusedAdamW(trainable, lr=1e-4)
red = GradAllReduce(trainable, order=model.grad_ready_order()).install(model)
red.zero_grad()


def step():
    red.arm()
    train_step(model, batch, sched, model.patchifier, cfg, prompt, mask, dev)
    red()
    opt.step()
    red.zero_grad()


for _ in range(3):
    step()
torch.cuda.synchronize()
enq = []
t0 = time.perf_counter()
for _ in range(5):
    a = time.perf_counter()
    step()
    enq.append(time.perf_counter() - a)
torch.cuda.synchronize()
tot = (time.perf_counter() - t0) / 5
print(f"enqueue ms/step {1e3 * sum(enq) / len(enq):.2f} (min {1e3 * min(enq):.2f})  step ms {1e3 * tot:.2f}", flush=True)
