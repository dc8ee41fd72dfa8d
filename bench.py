"""LTX-2B LoRA training-step benchmark on MI355X (BASELINE.json metric).

  python bench.py [--gpus N --steps K --warmup W]            (N = 1)
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W  (N > 1, one rank per GPU, RCCL)

Workload (BASELINE.json configs[1]): LTX-Video 2B (28 layers, D 2048, 32x64 heads,
FF 8192, caption 4096), bf16, random-init weights of that architecture, LoRA r=16 (alpha 16) on
attn2 q/k/v/out + trainable caption_projection, synthetic 49-frame 512x512 VAE latents
[8,128,7,16,16] per GPU (N = 1792 tokens), pose [8,128,7,16,16], ref [8,128,1,16,16],
T5-shaped prompt [1,256,4096] with the first 16 tokens valid. One "step" = one micro-batch
forward + backward (train_step); every 16th step also runs the DP gradient all-reduce and the
AdamW update (gradient_accumulation_steps 16, train-avatars.yaml:23), inside the timed region.

Prints ONE JSON line (rank 0): value = samples/s summed over ranks (= tokens/s / 1792), plus the
roofline of the dominant kernel (the kernel class with the most launch time in the timed region,
timed live with HIP events on its stream; algorithmic FLOPs per launch), a per-kernel table, and
the CPU baseline (the oracle restatement, rank 0 at N=1 only).
"""
import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "video-generation-for-human-avatars_amd"))

import torch
import torch.distributed as dist

MFMA_BF16_PEAK_TFLOPS = 2500.0   # MI355X dense bf16 (MI355X_MICROARCH.md, spec)
HBM_PEAK_GBS = 8000.0
B_PER_GPU, F_LAT, H_LAT, W_LAT, L_TXT = 8, 7, 16, 16, 256
N_VALID_TXT = 16  # valid caption tokens of the synthetic prompt (mask below)
LORA_RANK = 16
ACCUM = 16


def step_flops_per_sample(N, r=LORA_RANK, D=2048, FF=8192, Lyr=28, L=L_TXT, C=128, Cc=4096, L_att=None):
    """Algorithmic FLOPs of one fwd+bwd per sample: dgrad-only for frozen
    weights, wgrad for LoRA and caption_projection, attention bwd = 2x fwd, no recompute.
    L_att: caption keys counted in the cross-attention contractions (default L = 256, SURVEY
    8d; the valid-token count 16 leaves out the padding keys, whose products are exact zeros that
    the kernels skip)."""
    L_att = L if L_att is None else L_att
    lin = 2 * N * D * D * 6 + 4 * L * D * D + 4 * N * D * FF
    att = 4 * N * N * D + 4 * N * L_att * D
    lora = 8 * r * D * (N + L)
    fwd = Lyr * (lin + att + lora) + 4 * N * C * D + 2 * L * (Cc * D + D * D)
    bwd = Lyr * (lin + 2 * att + 2 * lora) + 2 * N * D * C + 2 * L * (Cc * D + D * D) + 2 * L * D * D
    return fwd, bwd


FULL_KEYS = ("proj_out", "scale_shift_table", "adaln_single", "caption_projection", "attn")


def build_model(device, seed=1234, mode="lora_audio"):
    from ltx_amd.config import TrainConfig
    from ltx_amd.lora import apply_training_strategy
    from ltx_amd.patchifier import SymmetricPatchifier
    from ltx_amd.transformer3d import OURS_TRANSFORMER_CONFIG, Transformer3DModel
    with torch.device("meta"):
        model = Transformer3DModel.from_config(OURS_TRANSFORMER_CONFIG)
        if mode != "full":
            apply_training_strategy(model, TrainConfig(checkpoint_path="-", lora_rank=LORA_RANK,
                                                       lora_alpha=LORA_RANK), "lora_audio")
    g = torch.Generator(device=device).manual_seed(seed)
    sd = {}
    for name, p in model.named_parameters():
        dt = torch.float32 if "lora_" in name else torch.bfloat16
        t = torch.empty(p.shape, dtype=torch.float32, device=device)
        if p.dim() == 2:
            t.normal_(0, 1.0 / math.sqrt(p.shape[1]), generator=g)
        elif "norm" in name:
            t.fill_(1.0)
        elif name.endswith("scale_shift_table"):
            t.normal_(0, 1.0 / math.sqrt(p.shape[-1]), generator=g)
        else:
            t.normal_(0, 0.02, generator=g)
        if "lora_B" in name:
            t.normal_(0, 0.01, generator=g)  # non-zero so the dA path carries signal
        sd[name] = t.to(dt)
    model.load_state_dict(sd, assign=True, strict=True)
    for n, p in model.named_parameters():
        if mode == "full":  # training.py:75-91 trainable set (config Z)
            p.requires_grad_(any(k in n for k in FULL_KEYS))
        else:
            p.requires_grad_(("lora_" in n) or ("caption_projection" in n))
    model.patchifier = SymmetricPatchifier(1)
    model.train()
    return model


def synthetic_batch(device, rank):
    g = torch.Generator().manual_seed(20251015 + rank)
    B = B_PER_GPU
    batch = {"latents": torch.randn(B, 128, F_LAT, H_LAT, W_LAT, generator=g),
             "ref_image_latents": torch.randn(B, 128, 1, H_LAT, W_LAT, generator=g),
             "pose_latents": torch.randn(B, 128, F_LAT, H_LAT, W_LAT, generator=g)}
    batch = {k: v.to(device=device, dtype=torch.bfloat16) for k, v in batch.items()}
    prompt = torch.randn(1, L_TXT, 4096, generator=g).to(device=device, dtype=torch.bfloat16)
    mask = (torch.arange(L_TXT) < N_VALID_TXT).long().view(1, L_TXT).to(device)
    return batch, prompt, mask


def selfcheck(device):
    """After the timed region: the step's two dominant kernel families on a config-A shape against
    torch fp32 (rel-Frobenius), so a bench line from a broken build cannot pass as a fast one (a
    kernel writing garbage makes the chip clock up: zero-ish operands cost less energy). The QKV
    GEMM (14336 x 6144 x 2048, the ring kernel) and the self-attention forward (B 1, 32 x 64 heads,
    N 1792, the pipelined kernel) on seeded random inputs."""
    from ltx_amd import ops
    g = torch.Generator(device="cpu").manual_seed(7)
    a = torch.randn(14336, 2048, generator=g).to(device, torch.bfloat16)
    w = (torch.randn(6144, 2048, generator=g) / 2048 ** 0.5).to(device, torch.bfloat16)
    ref = a.float() @ w.float().t()
    gemm_err = float((ops.gemm(a, w).float() - ref).norm() / ref.norm())
    del a, w, ref
    q, k, v = (torch.randn(1792, 2048, generator=g).to(device, torch.bfloat16) for _ in range(3))
    o, _ = ops.attn_fwd(q, k, v, 1, 32, 64, 64 ** -0.5)
    qh, kh, vh = (t.float().view(1, 1792, 32, 64).transpose(1, 2) for t in (q, k, v))
    ref = torch.nn.functional.scaled_dot_product_attention(qh, kh, vh).transpose(1, 2).reshape(1792, 2048)
    attn_err = float((o.float() - ref).norm() / ref.norm())
    ok = gemm_err < 1e-2 and attn_err < 2e-2
    if not ok:
        print(f"bench selfcheck FAILED: gemm rel err {gemm_err:.3e}, attention rel err {attn_err:.3e}",
              file=sys.stderr, flush=True)
    return {"ok": ok, "gemm_rel_err": round(gemm_err, 6), "attn_fwd_rel_err": round(attn_err, 6),
            "what": "ring GEMM 14336x6144x2048 and self-attention forward (1x32x1792x64) vs torch fp32"}


def cpu_baseline(budget_layers=28, warmup=2, timed=5):
    """The oracle restatement (oracle/ltx_oracle.py) on the host cores, as BASELINE.md 4 plans it:
    config A at B=1, N = 1792, all 28 blocks, `warmup` untimed + `timed` timed fwd+bwd steps, the
    MEDIAN timed step is the per-sample time (~35 s of CPU work). Threads: the box's CPU share
    for one GPU (16; os.cpu_count() reports the whole host, shared with the other GPUs' jobs)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import ltx_oracle as O
    from ltx_amd.transformer3d import OURS_TRANSFORMER_CONFIG
    threads = int(os.environ.get("LTX_CPU_BASELINE_THREADS", min(16, os.cpu_count() or 1)))
    torch.set_num_threads(threads)
    cfg = dict(OURS_TRANSFORMER_CONFIG)
    cfg["num_layers"] = budget_layers
    g = torch.Generator().manual_seed(0)
    p = {}
    for name, shape in O.param_shapes(cfg, LORA_RANK).items():
        t = torch.randn(shape, generator=g) * (1.0 / math.sqrt(shape[-1]) if len(shape) == 2 else 0.02)
        if len(shape) == 1 and "norm" in name:
            t = torch.ones(shape)
        t = t.to(torch.float32 if "lora_" in name else torch.bfloat16)
        if ("lora_" in name) or ("caption_projection" in name):
            t.requires_grad_(True)
        p[name] = t
    lat = torch.randn(1, 128, F_LAT, H_LAT, W_LAT, generator=g)
    ref = torch.randn(1, 128, 1, H_LAT, W_LAT, generator=g)
    pose = torch.randn(1, 128, F_LAT, H_LAT, W_LAT, generator=g)
    prompt = torch.randn(1, L_TXT, 4096, generator=g)
    mask = (torch.arange(L_TXT) < 16).long().view(1, L_TXT)
    times = []
    for _ in range(warmup + timed):
        t0 = time.perf_counter()
        r = O.train_step(p, cfg, lat, ref, pose, prompt, mask)
        r["loss"].backward()
        times.append(time.perf_counter() - t0)
        for v in p.values():
            v.grad = None
    steady = sorted(times[warmup:])
    per_sample = steady[len(steady) // 2] * (28.0 / budget_layers)
    # config T ("config A at B = 1 and config T"): the tiny 2-layer model, one
    # 1x8x8 latent, steady-state median of 20 steps after 3 warm-ups
    tcfg = {"num_layers": 2, "num_attention_heads": 4, "attention_head_dim": 32, "in_channels": 128,
            "out_channels": 128, "cross_attention_dim": 128, "caption_channels": 64}
    tcfg = {**OURS_TRANSFORMER_CONFIG, **tcfg}
    tp = {}
    for name, shape in O.param_shapes(tcfg, LORA_RANK).items():
        t = torch.randn(shape, generator=g) * (1.0 / math.sqrt(shape[-1]) if len(shape) == 2 else 0.02)
        if len(shape) == 1 and "norm" in name:
            t = torch.ones(shape)
        t = t.to(torch.float32 if "lora_" in name else torch.bfloat16)
        if ("lora_" in name) or ("caption_projection" in name):
            t.requires_grad_(True)
        tp[name] = t
    tl = [torch.randn(1, 128, 1, 8, 8, generator=g) for _ in range(3)]
    tprompt = torch.randn(1, 4, 64, generator=g)
    tmask = torch.ones(1, 4, dtype=torch.long)
    tt = []
    for i in range(23):
        t0 = time.perf_counter()
        r = O.train_step(tp, tcfg, tl[0], tl[1], tl[2], tprompt, tmask)
        r["loss"].backward()
        if i >= 3:
            tt.append(time.perf_counter() - t0)
        for v in tp.values():
            v.grad = None
    tt.sort()
    cpu_model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": 1.0 / per_sample, "unit": "samples/s", "cores": torch.get_num_threads(),
            "kind": "port", "host_cpu_count": os.cpu_count(), "cpu_model": cpu_model,
            "step_s": [round(x, 3) for x in times], "median_step_s": round(per_sample, 3),
            "config_t_ms_per_step": round(tt[len(tt) // 2] * 1e3, 2),
            "tokens_per_s": F_LAT * H_LAT * W_LAT / per_sample,
            "sample": (f"oracle/ltx_oracle.py train_step fwd+bwd, B=1, N={F_LAT*H_LAT*W_LAT}, "
                       f"{budget_layers}/28 LTX-2B blocks, {warmup} warm-up + {timed} timed steps, "
                       f"median ({sum(times[warmup:]):.1f} s timed); torch {torch.__version__} CPU, "
                       f"{torch.get_num_threads()} threads = the gpurun box's CPU share for one GPU "
                       f"(os.cpu_count()={os.cpu_count()} is the whole shared host)")}


def _kernel_key(name):
    """rocprofv3 / bench kernel name -> comparison key: no argument list, no 'void ', no spaces,
    and trailing template arguments that are 0 (defaulted parameters print as ', 0') dropped."""
    k = name.split("(")[0].replace("void ", "").replace(" ", "")
    while k.endswith(",0>"):
        k = k[:-3] + ">"
    return k


def load_traffic(label):
    """Measured HBM bytes per launch of the kernel(s) behind `label`, from the NEWEST committed
    PMC summary profiles/r*_traffic.json (tools/kernel_traffic.py: FETCH_SIZE x2 + WRITE_SIZE,
    separate passes, means over every dispatch of the name). Returns (bytes, file name) or
    (None, reason)."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_traffic.json")))
    if not files:
        return None, "no profiles/r*_traffic.json"
    path = files[-1]
    try:
        with open(path) as f:
            table = json.load(f)["bytes_per_launch"]
    except (OSError, ValueError, KeyError) as exc:
        return None, f"{os.path.basename(path)}: {exc!r}"[:160]
    keyed = {_kernel_key(k): v for k, v in table.items()}
    names = [_kernel_key(n) for n in label.split(": ", 1)[-1].split(" + ")]
    vals = [keyed.get(n) for n in names]
    if any(v is None for v in vals):
        return None, f"{os.path.basename(path)} has no entry for {label}"
    return float(sum(vals)), os.path.basename(path)


def infer_main(args):
    """--infer: one LTXVideoPipeline denoising step per "step": CFG 3.0 +
    STG 1.0 (AttentionValues on block 19) + rescaling 0.7, first latent frame hard-conditioned
    (per-token timesteps), `--infer-batch` videos of 49f 512x512 -> transformer batch 3 x B of
    N = 1792 tokens, guidance + Euler update included. Prints its own JSON line (not the
    training metric)."""
    torch.cuda.set_device(0)
    device = torch.device("cuda", 0)
    from ltx_amd import _lib
    from ltx_amd.denoise import denoise_step
    from ltx_amd.scheduler import RectifiedFlowScheduler
    from ltx_amd.transformer3d import SkipLayerStrategy
    _lib.ensure_device(device)
    model = build_model(device)
    model.eval()
    for p in model.parameters():
        p.requires_grad_(False)
    B = args.infer_batch
    N = F_LAT * H_LAT * W_LAT
    g = torch.Generator().manual_seed(20251015)
    lat = torch.randn(B, N, 128, generator=g).to(device)
    ref = torch.randn(B, 128, 1, H_LAT, W_LAT, generator=g).to(device, torch.bfloat16)
    pose = torch.randn(B, 128, F_LAT, H_LAT, W_LAT, generator=g).to(device, torch.bfloat16)
    neg = torch.randn(B, L_TXT, 4096, generator=g)
    pos = torch.randn(B, L_TXT, 4096, generator=g)
    enc = torch.cat([neg, pos, pos]).to(device, torch.bfloat16)
    m = (torch.arange(L_TXT) < 16).long().view(1, L_TXT)
    mask = torch.cat([torch.ones(B, L_TXT, dtype=torch.long), m.expand(2 * B, -1)]).to(device)
    cond = torch.zeros(B, N, device=device)
    cond[:, : H_LAT * W_LAT] = 1.0
    sch = RectifiedFlowScheduler(sampler="LinearQuadratic")
    sch.set_timesteps(num_inference_steps=max(args.steps + args.warmup, 2), device=device)
    kw = dict(prompt_embeds_batch=enc, prompt_attention_mask_batch=mask,
              ref_image_hidden_states=ref, pose_hidden_states=pose, frame_rate=25.0,
              batch_size=B, guidance_scale=3.0, stg_scale=1.0, rescaling_scale=0.7,
              skip_block_list=[19], skip_layer_strategy=SkipLayerStrategy.AttentionValues,
              conditioning_mask=cond)
    with torch.no_grad():
        for i in range(args.warmup):
            lat = denoise_step(model, sch, lat, sch.timesteps[i], **kw)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.warmup, args.warmup + args.steps):
            lat = denoise_step(model, sch, lat, sch.timesteps[i], **kw)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
    fwd, _ = step_flops_per_sample(N, r=LORA_RANK)
    tflops = fwd * 3 * B * args.steps / (elapsed * 1e12)
    print(json.dumps({
        "metric": "LTX-2B inference denoising steps/sec (CFG+STG: transformer batch 3 x videos)",
        "value": round(args.steps / elapsed, 4), "unit": "steps/s",
        "tokens_per_s": round(3 * B * N * args.steps / elapsed, 1),
        "ms_per_step": round(elapsed * 1e3 / args.steps, 3), "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "higher_is_better": True, "dtype": "bf16",
        "data": "synthetic latents/pose/ref/prompts; random-init LTX-2B weights",
        "config": {"workload": "denoise_step: CFG 3.0 + STG 1.0 (AttentionValues, block 19) + "
                               "rescale 0.7, per-token timesteps (first frame conditioned), "
                               "49f 512x512 -> N=1792", "videos": B, "transformer_batch": 3 * B},
        "fwd_tflops": round(tflops, 1), "mfma_frac": round(tflops / MFMA_BF16_PEAK_TFLOPS, 4),
    }), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--infer", action="store_true", help="inference denoising-step benchmark")
    ap.add_argument("--infer-batch", type=int, default=1)
    ap.add_argument("--config", choices=["a", "x"], default="a",
                    help="a: 49f 512x512 (N=1792, the metric); x: 97f 768x768 (N=7488, "
                         "BASELINE configs[3], long-sequence stress)")
    ap.add_argument("--batch", type=int, default=None, help="micro-batch per GPU (default 8)")
    ap.add_argument("--grad-ckpt", action="store_true", help="per-block gradient checkpointing")
    ap.add_argument("--lora-rank", type=int, default=16,
                    help="LoRA rank (alpha = rank): 16 is the BASELINE config, 32 the yaml default")
    ap.add_argument("--fixed-global-batch", action="store_true",
                    help="scale gradient accumulation 16 -> 16/N so the global batch per optimizer "
                         "step stays 128 samples (SURVEY 8e: loss-curve parity with 1 GPU)")
    ap.add_argument("--mode", choices=["lora", "full"], default="lora",
                    help="full: train_mode='full' + ZeRO-2 AdamW (BASELINE configs[4], "
                         "ds_config_zero2.json: grad accumulation 3, clip 1.0)")
    args = ap.parse_args()
    global F_LAT, H_LAT, W_LAT, B_PER_GPU, ACCUM, LORA_RANK
    LORA_RANK = args.lora_rank
    if args.config == "x":
        F_LAT, H_LAT, W_LAT = 13, 24, 24
    if args.batch:
        B_PER_GPU = args.batch
    if args.infer:
        return infer_main(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # rehearsal overrides for a one-GPU box (all ranks on cuda:0 over gloo); the driver's
        # multi-GPU runs use the defaults: one GPU per rank, RCCL ("nccl")
        backend = os.environ.get("LTX_BENCH_BACKEND", "nccl")
        if os.environ.get("LTX_BENCH_SAME_DEVICE") == "1":
            local_rank = 0
        torch.cuda.set_device(local_rank)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    device = torch.device("cuda", torch.cuda.current_device())

    from ltx_amd import _lib, ops
    from ltx_amd.config import TrainConfig
    from ltx_amd.scheduler import RectifiedFlowScheduler
    from ltx_amd.training import FusedAdamW, GradAllReduce, train_step
    _lib.ensure_device(device)

    full = args.mode == "full"
    if full:
        ACCUM = 3  # ds_config_zero2.json gradient_accumulation_steps
    elif args.fixed_global_batch:
        ACCUM = max(1, ACCUM // world)
    model = build_model(device, mode="full" if full else "lora_audio")
    model.gradient_checkpointing = bool(args.grad_ckpt)
    batch, prompt, mask = synthetic_batch(device, rank)
    cfg = TrainConfig(checkpoint_path="-", batch_size=B_PER_GPU, learning_rate=1e-4,
                      lora_rank=LORA_RANK, lora_alpha=LORA_RANK, gradient_accumulation_steps=ACCUM,
                      rf_log_normal_mu=-0.5, rf_log_normal_sigma=1.0)
    sched = RectifiedFlowScheduler(num_train_timesteps=1000, shifting=None)
    trainable = [p for p in model.parameters() if p.requires_grad]
    if full:
        from ltx_amd.zero import Zero2AdamW
        # ds_config_zero2.json: reduce_scatter of f32 grads in 5e8-element buckets, overlap_comm:
        # buckets in the backward's completion order, launched from its hooks on the last micro-step
        opt = Zero2AdamW(trainable, lr=cfg.learning_rate, gradient_clipping=1.0,
                         order=model.grad_ready_order()).install(model)
        reducer = lambda: None  # noqa: E731  (the reduce-scatter is inside Zero2AdamW.step)
    else:
        opt = FusedAdamW(trainable, lr=cfg.learning_rate)
        # bucketed all-reduce overlapped with the last micro-step's backward (grads live in the
        # reducer's buckets; zero_grad keeps them there)
        reducer = GradAllReduce(trainable, order=model.grad_ready_order()).install(model)
        reducer.zero_grad()
    torch.manual_seed(20251015 + rank)

    N = F_LAT * H_LAT * W_LAT
    timer = ops.LaunchTimer()

    def one_step(i):
        last = (i + 1) % ACCUM == 0
        if last:
            (opt if full else reducer).arm()
        train_step(model, batch, sched, model.patchifier, cfg, prompt, mask, device)
        if last:
            reducer()
            opt.step()
            if full:
                opt.zero_grad(set_to_none=True)
            else:
                reducer.zero_grad()

    for i in range(args.warmup):
        one_step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.warmup, args.warmup + args.steps):
        one_step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # per-kernel durations with HIP events on the launch stream, in further steps of the same loop
    # right after the timed region (an event pair around every launch costs the step ~5 %, so the
    # timed region stays un-instrumented): one step with every GEMM / attention launch bracketed
    # ranks the kernels; then `prof_steps` steps bracket only the dominant one (few events, the
    # per-launch figure the roofline uses)
    i0 = args.warmup + args.steps
    ops.set_launch_timer(timer)
    one_step(i0)
    ops.set_launch_timer(None)
    kernels = timer.summary()
    prof_steps = min(args.steps, 4)
    dom_timer = ops.LaunchTimer(only=kernels[0]["kernel"])
    ops.set_launch_timer(dom_timer)
    for i in range(i0 + 1, i0 + 1 + prof_steps):
        one_step(i)
    ops.set_launch_timer(None)
    dom = dom_timer.summary()[0]

    samples = B_PER_GPU * args.steps * world
    value = samples / elapsed
    fwd, bwd = step_flops_per_sample(N, r=LORA_RANK)
    if full:  # + wgrad of every attention projection, adaln_single, proj_out (2*M*K*N each)
        bwd += 28 * (2 * N * 2048 * 2048 * 6 + 4 * L_TXT * 2048 * 2048) + 2 * N * 2048 * 128
    step_tflops = (fwd + bwd) * B_PER_GPU * args.steps / (elapsed * 1e12)  # per GPU
    # the same without the cross-attention's padding keys (16 of 256 caption tokens valid: the
    # skipped key blocks' products are exact zeros, VERDICT r03 asks for both figures)
    fwd_v, bwd_v = step_flops_per_sample(N, r=LORA_RANK, L_att=N_VALID_TXT)
    step_tflops_valid = step_tflops * (fwd_v + bwd_v) / (fwd + bwd)
    # the dominant kernel = the class with the most HIP-event time in the ranking step (all of them
    # are hand-written); its algorithmic TFLOP/s = its FLOPs / its summed launch durations
    for k in kernels + [dom]:
        k["tflops"] = k["flops"] / (k["ms"] * 1e-3) / 1e12
    achieved = dom["tflops"]
    if args.config == "a" and not full:
        traffic, traffic_src = load_traffic(dom["kernel"])
    else:
        traffic, traffic_src = None, "measured for config A LoRA only"
    line = {
        "metric": f"LTX-2B {'full (ZeRO-2)' if full else 'LoRA'} train-step samples/sec (latent-tokens/sec = samples/sec x {N})",
        "value": round(value, 4),
        "unit": "samples/s",
        "tokens_per_s": round(value * N, 1),
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic latents/pose/ref/prompt of the configured shapes; random-init LTX-2B weights",
        "config": {"lora_rank": None if full else LORA_RANK,
                   "workload": ("LTX-Video 2B train_mode='full' (attn*, scale_shift_table, adaln_single, "
                                "caption_projection, proj_out; %.0fM params) + ZeRO-2 AdamW, "
                                % (sum(p.numel() for p in trainable) / 1e6)
                                if full else f"LTX-Video 2B LoRA(r={LORA_RANK}, attn2 q/k/v/out) + caption_projection ")
                               + ("train step, 49f 512x512 -> latent 7x16x16 (N=1792), 1xMI355X per rank"
                                  if args.config == "a" else
                                  "train step, 97f 768x768 -> latent 13x24x24 (N=7488), 1xMI355X per rank")
                               + (", per-block gradient checkpointing" if args.grad_ckpt else ""),
                   "model": "LTX-Video-2B (28 layers, D 2048, 32x64 heads)", "global_batch": B_PER_GPU * world,
                   "micro_batch_per_gpu": B_PER_GPU, "seq_len": N, "text_len": L_TXT,
                   "grad_accum": ACCUM, "parallelism": f"zero2-dp{world}" if full else f"dp{world}",
                   # 16 of 256 caption tokens are valid: the cross-attention kernels skip all-padding
                   # key blocks (exact: bitwise-equal outputs); FLOPs still count Nk = 256
                   "attn2_padding_blocks": ("kept (LTX_ATTN_SKIP=0)" if os.environ.get("LTX_ATTN_SKIP") == "0"
                                            else "skipped, exact")},
        "step_tflops_per_gpu": round(step_tflops, 1),
        "step_mfma_frac": round(step_tflops / MFMA_BF16_PEAK_TFLOPS, 4),
        "step_tflops_per_gpu_excl_padding_keys": round(step_tflops_valid, 1),
        "step_mfma_frac_excl_padding_keys": round(step_tflops_valid / MFMA_BF16_PEAK_TFLOPS, 4),
        "roofline": {"bound": "mfma", "kernel": dom["kernel"],
                     "achieved": round(achieved, 1), "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / MFMA_BF16_PEAK_TFLOPS, 4),
                     "traffic": traffic,
                     "traffic_source": traffic_src,
                     "algorithmic_bytes": dom["bytes"] / dom["launches"],
                     "traffic_over_algorithmic": (round(traffic / (dom["bytes"] / dom["launches"]), 3)
                                                  if traffic and dom["bytes"] else None),
                     "launch_ms": round(dom["ms"] / dom["launches"], 4), "launches": dom["launches"],
                     "share_of_step": round(dom["ms"] / prof_steps / (elapsed * 1e3 / args.steps), 4),
                     "timing": f"HIP events around each of its launches in {prof_steps} steps after the timed region",
                     "flops_per_launch": dom["flops"] / dom["launches"]},
        # every GEMM / attention kernel class by total time (one step, every launch bracketed)
        "kernels": [{"kernel": k["kernel"], "launches_per_step": k["launches"],
                     "ms_per_step": round(k["ms"], 3), "tflops": round(k["tflops"], 1),
                     "frac": round(k["tflops"] / MFMA_BF16_PEAK_TFLOPS, 4)} for k in kernels[:10]],
    }
    line["selfcheck"] = selfcheck(device)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "a" and not full:
        try:
            line["cpu_baseline"] = cpu_baseline()
        except Exception as exc:  # the baseline must never hide the GPU measurement
            line["cpu_baseline"] = {"value": None, "error": repr(exc)[:200]}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
