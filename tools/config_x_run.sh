#!/bin/bash
# Config X (BASELINE configs[3]: 97f 768x768 -> N = 7488) on one GPU: the bench line at B = 8,
# then a kernel-trace pass of the same step for the per-kernel split (attention backward per step).
#   usage (GPU box): bash tools/config_x_run.sh ; env XB=<micro-batch> (default 8)
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/config_x
RAW=/tmp/ltx_cx
mkdir -p $OUT $RAW
cd /tmp
export TMPDIR=/tmp
B=${XB:-8}
timeout -k 10 400 python3 -u $R/bench.py --config x --batch $B --steps 5 --warmup 2 --no-cpu-baseline \
    > $OUT/bench_x_b$B.jsonl 2> $OUT/bench_x_b$B.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d $RAW/trace -o run -- \
    python3 $R/bench.py --config x --batch $B --steps 3 --warmup 1 --no-cpu-baseline \
    > $OUT/bench_x_b${B}_under_rocprof.jsonl 2> $RAW/trace.err
cp $RAW/trace/run_kernel_stats.csv $OUT/kernel_stats_x_b$B.csv
# 1 warm-up + 3 timed + 1 + 3 timer steps in the trace
python3 $R/tools/rocpd_summary.py $RAW/trace/run_results.db 8 30 > $OUT/trace_summary_x_b$B.txt
ls -la $OUT
