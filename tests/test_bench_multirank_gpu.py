"""bench.py's N > 1 path, rehearsed on the one-GPU box (training_deepspeed.py:90-94,
DESIGN §6): `torch.distributed.run --nproc-per-node 2 bench.py` as a fresh child process with both
ranks on cuda:0 over gloo (LTX_BENCH_BACKEND=gloo, LTX_BENCH_SAME_DEVICE=1), so the barriers, the
max-over-ranks timing, GradAllReduce.arm() inside the timed loop (LoRA) and the ZeRO-2
reduce-scatter / all-gather optimizer (--mode full) run exactly as the driver's multi-GPU bench
will run them, across at least one gradient-accumulation boundary. The JSON line must parse with
n_gpus = 2 and finite, positive figures.
"""
import json
import math
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(extra, port, timeout):
    env = dict(os.environ, LTX_BENCH_BACKEND="gloo", LTX_BENCH_SAME_DEVICE="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--no-cpu-baseline"] + extra
    torch.cuda.empty_cache()
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, f"rc {p.returncode}\n{p.stdout[-3000:]}\n{p.stderr[-3000:]}"
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-3000:]  # rank 0 prints exactly one line
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2
    for k in ("value", "ms_per_step", "tokens_per_s", "step_tflops_per_gpu"):
        assert math.isfinite(line[k]) and line[k] > 0, (k, line[k])
    assert line["selfcheck"]["ok"], line["selfcheck"]
    return line


@pytest.mark.timeout(420)
def test_bench_two_ranks_lora_fixed_global_batch():
    # --fixed-global-batch at world 2: accumulation 16 -> 8, so warmup 1 + 8 timed steps end on the
    # boundary: the armed all-reduce and the AdamW step run inside the timed region
    line = _run(["--steps", "8", "--warmup", "1", "--fixed-global-batch"], 29531, 400)
    assert line["config"]["grad_accum"] == 8
    assert line["config"]["parallelism"] == "dp2"
    assert line["config"]["global_batch"] == 16


@pytest.mark.timeout(420)
def test_bench_two_ranks_full_zero2():
    # --mode full: ZeRO-2 AdamW, accumulation 3 (ds_config_zero2.json), so warmup 1 + 3 timed steps
    # cross one boundary inside the timed region (reduce-scatter + sharded AdamW + all-gather)
    line = _run(["--steps", "3", "--warmup", "1", "--mode", "full"], 29533, 400)
    assert line["config"]["grad_accum"] == 3
    assert line["config"]["parallelism"] == "zero2-dp2"
