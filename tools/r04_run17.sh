#!/bin/bash
# round 4, GPU call 17: kernel-trace stats of config X at B = 1 (the one-pass cross-attention
# kernels' per-step time under the query split) and at B = 8
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/x17
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/x17b1 -o run -- \
    python3 $R/bench.py --config x --batch 1 --steps 4 --warmup 1 --no-cpu-baseline > $R/gpurun_out/x17/bench_b1.jsonl 2> $R/gpurun_out/x17/b1.err || exit $?
cp /tmp/x17b1/run_kernel_stats.csv $R/gpurun_out/x17/kernel_stats_b1.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/x17b8 -o run -- \
    python3 $R/bench.py --config x --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/x17/bench_b8.jsonl 2> $R/gpurun_out/x17/b8.err || exit $?
cp /tmp/x17b8/run_kernel_stats.csv $R/gpurun_out/x17/kernel_stats_b8.csv
