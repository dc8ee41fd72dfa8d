#!/bin/bash
# round 4, GPU call 21: kernel-trace stats of the step with the text k_norm per block (0) and
# grouped (1), for the per-kernel totals; then the step A/B three more times
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/k21
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for c in 0 1; do
  LTX_TEXT_KNORM_GROUPED=$c timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/k21_$c -o run -- \
      python3 $R/bench.py --steps 6 --warmup 2 --no-cpu-baseline > $R/gpurun_out/k21/bench_$c.jsonl 2> $R/gpurun_out/k21/err_$c.txt || exit $?
  cp /tmp/k21_$c/run_kernel_stats.csv $R/gpurun_out/k21/kernel_stats_$c.csv
done
cd $R
for i in 3 4 5; do
  for c in 0 1; do
    LTX_TEXT_KNORM_GROUPED=$c timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench20_g${c}_$i.json 2>> gpurun_out/r04_bench.err || exit $?
  done
done
